"""Batched k = 16 kNN timing at RandLA-Net's shapes (one call over the 5
levels of a 45,056-point patch crop of the C2 scan, as randlanet.py batches
them), kernel time from HIP events; library from O3DML_AMD_LIB if set.
    python tools/knn_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-ml_amd"))
from bench import make_scan  # noqa: E402
from o3dml_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda:0")
    scan = torch.from_numpy(make_scan(0)[0][:, :3].astype(np.float32)).to(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    center = scan[torch.randint(0, scan.shape[0], (1,), generator=g)]
    d = ((scan - center) ** 2).sum(1)
    lvl = [scan[d.topk(45056, largest=False).indices]]
    for _ in range(4):
        prev = lvl[-1]
        lvl.append(prev[torch.randperm(prev.shape[0], generator=g)[: prev.shape[0] // 4].to(dev)])
    cat = torch.cat(lvl).contiguous()
    rs = torch.tensor(np.cumsum([0] + [x.shape[0] for x in lvl]), dtype=torch.int64)
    for _ in range(5):
        ops.knn_search(cat, cat, 16, rs, rs)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        t0.record()
        out = ops.knn_search(cat, cat, 16, rs, rs)
        t1.record()
        torch.cuda.synchronize()
        ms.append(t0.elapsed_time(t1))
    idx = out[0].view(-1, 16)
    print(f"queries {cat.shape[0]} call median {np.median(ms) * 1e3:.1f} us (min {min(ms) * 1e3:.1f}) "
          f"checksum {int(idx.long().sum())}")


if __name__ == "__main__":
    main()
