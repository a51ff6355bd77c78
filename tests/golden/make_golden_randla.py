"""Generate tests/golden/randla.npz (build container only): the reference
RandLANet (ml3d/torch/models/randlanet.py, imported with tools/ref_loader.py)
evaluated on CPU with deterministic parameters (randla_weights.fill) on a
4,096-point cloud whose per-layer kNN inputs follow RandLANet.transform
(randlanet.py:212-239, neighbour indices from scipy cKDTree).  Stores the
state_dict key/shape manifest, the inputs and the logits — data only."""
import os
import sys

import numpy as np
import torch
from scipy.spatial import cKDTree

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402


def knn(support, query, k):
    return cKDTree(support.astype(np.float64)).query(query.astype(np.float64), k)[1].reshape(len(query), k)


def main():
    import ref_loader
    ref_loader.install()
    from ml3d.torch.models.randlanet import RandLANet
    torch.manual_seed(0)
    model = RandLANet(num_points=4096, num_classes=19, in_channels=3)
    sd = model.state_dict()
    keys = list(sd.keys())
    shapes = [tuple(v.shape) for v in sd.values()]
    model.load_state_dict(randla_weights.state_dict_for(zip(keys, shapes)))
    model.eval()
    model.device = torch.device("cpu")
    rng = np.random.default_rng(7)
    n = 4096
    pc = np.stack([rng.uniform(-8, 8, n), rng.uniform(-8, 8, n), rng.uniform(-1.7, 1.5, n)], 1).astype(np.float32)
    out = {"points": pc}
    coords, nbrs, pools, ups = [], [], [], []
    cur = pc
    for i in range(4):
        nb = knn(cur, cur, 16)
        sub = cur[: cur.shape[0] // 4]
        up = knn(sub, cur, 1)
        coords.append(torch.from_numpy(cur)[None])
        nbrs.append(torch.from_numpy(nb.astype(np.int64))[None])
        pools.append(torch.from_numpy(nb[: cur.shape[0] // 4].astype(np.int64))[None])
        ups.append(torch.from_numpy(up.astype(np.int64))[None])
        out[f"nbr{i}"] = nb.astype(np.int32)
        out[f"up{i}"] = up.astype(np.int32)
        cur = sub
    inputs = {"coords": coords, "neighbor_indices": nbrs, "sub_idx": pools, "interp_idx": ups,
              "features": torch.from_numpy(pc)[None]}
    with torch.no_grad():
        logits = model(inputs)[0].numpy()
    out["logits"] = logits.astype(np.float32)
    out["keys"] = np.array(keys)
    out["shapes"] = np.array([",".join(map(str, s)) for s in shapes])
    out["n_params"] = np.int64(sum(p.numel() for p in model.parameters() if p.requires_grad))
    np.savez_compressed(os.path.join(HERE, "randla.npz"), **out)
    print("keys", len(keys), "params", int(out["n_params"]), "logits", logits.shape, float(np.abs(logits).mean()))


if __name__ == "__main__":
    main()
