"""Time ops.nms (HIP) on PointPillars-shaped inputs: nms_pre=100 boxes per class
(the reference's call, point_pillars.py:995-1005) and a 4,096-box stress case."""
import math
import os
import sys
import time

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, d) for d in ("open3d-ml_amd", "tests", "oracle")]
from o3dml_amd import ops  # noqa: E402
from test_nms import _boxes  # noqa: E402
import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
for n in (100, 1000, 4096):
    b = _boxes(n, 7, spread=1.5 * math.sqrt(n))
    s = np.random.default_rng(8).random(n, dtype=np.float32)
    tb, ts = torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev)
    for _ in range(5):
        ops.nms(tb, ts, 0.01)
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        k = ops.nms(tb, ts, 0.01)
    torch.cuda.synchronize()
    gpu_us = (time.perf_counter() - t0) / reps * 1e6
    t0 = time.perf_counter()
    ref = O.nms(b, s, 0.01)
    cpu_us = (time.perf_counter() - t0) * 1e6
    assert np.array_equal(k.cpu().numpy(), ref)
    print(f"nms n={n} kept={len(ref)} gpu_us_per_call={gpu_us:.1f} (incl. count readback) oracle_cpu_us={cpu_us:.0f}",
          flush=True)
