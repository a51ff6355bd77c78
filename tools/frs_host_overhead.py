"""Host-side cost of one layers.FixedRadiusSearch call on a tiny input (GPU
work negligible): wall time per call, and the split by phase via cProfile."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "open3d-ml_amd"))
from o3dml_amd import layers  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
pts = torch.from_numpy(np.random.default_rng(0).random((n, 3), dtype=np.float32)).to(dev)
rs = torch.tensor([0, n], dtype=torch.int64)
nns = layers.FixedRadiusSearch()
for _ in range(20):
    nns(pts, pts, 0.05, rs, rs)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    nns(pts, pts, 0.05, rs, rs)
torch.cuda.synchronize()
print("ms per call", (time.perf_counter() - t) / 200 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    nns(pts, pts, 0.05, rs, rs)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
