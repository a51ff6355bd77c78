"""Time ops.knn_search (k=16 self, k=1 up) on RandLA-shaped LiDAR patches for
each kNN path (O3DML_KNN_PATH=ring|morton, set per process)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
pts, _ = bench.make_scan(0)
p = torch.from_numpy(pts).to(dev)
sub, _, _, _ = ops.grid_subsample(p, [p.shape[0]], 0.06)
c = sub[:1]
idx = ops.knn_search(sub, c, 45056).neighbors_index.long()
patch = sub[idx[torch.randperm(idx.shape[0], device=dev)]].contiguous()
res = {}
for n in (45056, 11264, 2816, 704):
    x = patch[:n].contiguous()
    for _ in range(2):
        ops.knn_search(x, x, 16)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        r = ops.knn_search(x, x, 16)
    torch.cuda.synchronize()
    res[n] = round((time.perf_counter() - t) / 10 * 1e3, 3)
print(os.environ.get("O3DML_KNN_PATH", "morton"), "ms per knn16 call by size:", res)
