"""Time the reference KPFCNN training step on this container's CPU (C3
proxy for DESIGN.md; never shipped): ml3d/torch/models/kpconv.py KPFCNN with
the kpconv_s3dis.yml model config and the reference collate
(concat_batcher.py segmentation_inputs), Open3D ops backed by the C oracle
(tools/ref_loader.py; OpenMP), torch CPU threads = host cores.  Same input
as bench.py make_c3."""
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def main(steps=3):
    import ref_loader
    ref_loader.install()
    import bench
    os.chdir("/tmp")
    import ml3d.torch.models.kpconv as K
    from ml3d.torch.dataloaders.concat_batcher import KPConvBatch
    cfg = dict(lbl_values=list(range(13)), num_classes=13, ignored_label_inds=[], first_subsampling_dl=0.04,
               in_features_dim=5, in_radius=1.5, batch_limit=20000, max_in_points=20000, batch_norm_momentum=0.98)
    torch.manual_seed(0)
    model = K.KPFCNN(**cfg).train()
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.98, weight_decay=0.001)
    pts, feats, labels, lengths = bench.make_c3(0)
    fake = types.SimpleNamespace(cfg=model.cfg, neighborhood_limits=[])
    fake.big_neighborhood_filter = lambda nb, layer: nb
    L = model.cfg.num_layers

    def step():
        t0 = time.perf_counter()
        li = KPConvBatch.segmentation_inputs(fake, pts, feats, labels, lengths)
        t1 = time.perf_counter()
        b = types.SimpleNamespace(points=[torch.from_numpy(li[l]) for l in range(L)],
                                  neighbors=[torch.from_numpy(li[L + l]) for l in range(L)],
                                  pools=[torch.from_numpy(li[2 * L + l]) for l in range(L)],
                                  upsamples=[torch.from_numpy(li[3 * L + l]) for l in range(L)],
                                  lengths=[torch.from_numpy(li[4 * L + l]) for l in range(L)],
                                  features=torch.from_numpy(feats), labels=torch.from_numpy(labels))
        loss = torch.nn.functional.cross_entropy(model(b), b.labels)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return t1 - t0, time.perf_counter() - t1

    step()
    ts = [step() for _ in range(steps)]
    col = float(np.median([t[0] for t in ts]))
    net = float(np.median([t[1] for t in ts]))
    print(f"reference KPFCNN C3 train step on CPU ({torch.get_num_threads()} threads): "
          f"collate {col:.3f} s + fwd/bwd/SGD {net:.3f} s = {col + net:.3f} s/step")


if __name__ == "__main__":
    main()
