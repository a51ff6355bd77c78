"""Time layers.FixedRadiusSearch on one scene of N = 2^LG points at the C1
density (bench.py c1_sweep shape): median ms of REPS calls after 2 warm-up
calls.  usage: python tools/frs_big_time.py [LG=24] [REPS=7]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-ml_amd"))
from o3dml_amd import layers  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
n = 1 << lg
dev = torch.device("cuda", 0)
pts = torch.from_numpy(np.random.default_rng(lg).random((n, 3), dtype=np.float32)).to(dev)
rs = torch.tensor([0, n], dtype=torch.int64)
r = 0.05 * (65536.0 / n) ** (1.0 / 3.0)
nns = layers.FixedRadiusSearch()
for _ in range(2):
    res = nns(pts, pts, r, rs, rs)
torch.cuda.synchronize(dev)
ts = []
for _ in range(reps):
    t = time.perf_counter()
    res = nns(pts, pts, r, rs, rs)
    torch.cuda.synchronize(dev)
    ts.append((time.perf_counter() - t) * 1e3)
ms = float(np.median(ts))
print(f"2^{lg}: {ms:.3f} ms  {n / ms / 1e3:.1f} Mpoints/s  pairs {int(res.neighbors_row_splits[-1])}")
