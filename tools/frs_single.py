"""One scene of N = 2^LG U[0,1)^3 points at C1 density (bench.py c1_sweep),
REPS layers.FixedRadiusSearch forwards — for rocprofv3 kernel stats.
usage: python tools/frs_single.py [LG=22] [REPS=10]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-ml_amd"))
from o3dml_amd import layers  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n = 1 << lg
dev = torch.device("cuda", 0)
pts = torch.from_numpy(np.random.default_rng(lg).random((n, 3), dtype=np.float32)).to(dev)
rs = torch.tensor([0, n], dtype=torch.int64)
r = 0.05 * (65536.0 / n) ** (1.0 / 3.0)
nns = layers.FixedRadiusSearch()
res = nns(pts, pts, r, rs, rs)  # warm-up
torch.cuda.synchronize(dev)
times = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    res = nns(pts, pts, r, rs, rs)
    e1.record()
    torch.cuda.synchronize(dev)
    times.append(e0.elapsed_time(e1))
ms = float(np.median(times))
print("pairs", int(res.neighbors_row_splits[-1]), f"median {ms:.3f} ms/call, {n / ms / 1e3:.1f} Mpoints/s")
