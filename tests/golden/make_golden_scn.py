"""Generate tests/golden/scn.npz (build container only): the reference
SparseConvUnet (ml3d/torch/models/sparseconvnet.py, imported with
tools/ref_loader.py; Open3D's SparseConv / SparseConvTranspose / voxelize /
reduce_subarrays_sum backed by the CPU oracle) evaluated with deterministic
parameters (randla_weights.fill) on a small room-like voxel cloud, for the
residual and the plain UNet.  Stores the state_dict manifest, the inputs and
the logits — data only."""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402


def cloud(seed=0):
    rng = np.random.default_rng(seed)
    pts = []
    for _ in range(5000):  # floor + two walls + a box, ~2 cm voxels in voxel units
        s = rng.integers(0, 4)
        u, v = rng.uniform(0, 60, 2)
        if s == 0:
            p = [u, v, rng.uniform(0, 1)]
        elif s == 1:
            p = [u, rng.uniform(0, 1), v * 0.5]
        elif s == 2:
            p = [rng.uniform(0, 1), u, v * 0.5]
        else:
            p = [20 + u / 6, 20 + v / 6, 10 + rng.uniform(0, 1)]
        pts.append(p)
    pos = np.floor(np.asarray(pts, np.float32)).astype(np.float32) + 0.5
    return pos, rng.random((len(pos), 3), dtype=np.float32)


def main():
    import ref_loader
    ref_loader.install()
    from ml3d.torch.models.sparseconvnet import SparseConvUnet
    pos, feat = cloud(0)
    out = {"pos": pos, "feat": feat}
    for tag, residual in (("res", True), ("plain", False)):
        torch.manual_seed(0)
        model = SparseConvUnet(multiplier=8, residual_blocks=residual, conv_block_reps=1, num_classes=5,
                               device="cpu").eval()
        sd = model.state_dict()
        keys = list(sd.keys())
        model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd))

        inp = types.SimpleNamespace(point=[torch.from_numpy(pos)], feat=[torch.from_numpy(feat)],
                                    batch_lengths=[len(pos)])
        with torch.no_grad():
            logits = model(inp).numpy()
        out[f"{tag}_logits"] = logits.astype(np.float32)
        out[f"{tag}_keys"] = np.array(keys)
        out[f"{tag}_shapes"] = np.array([",".join(map(str, sd[k].shape)) for k in keys])
        print(tag, len(keys), logits.shape, float(np.abs(logits).mean()))
    np.savez_compressed(os.path.join(HERE, "scn.npz"), **out)


if __name__ == "__main__":
    main()
