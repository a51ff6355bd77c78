"""Run layers.FixedRadiusSearch on the bench workload a few times (for
rocprofv3 kernel traces / PMC passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from o3dml_amd import layers  # noqa: E402

scenes = int(os.environ.get("SCENES", "64"))
reps = int(os.environ.get("REPS", "3"))
dev = torch.device("cuda", 0)
pts = np.concatenate([np.random.default_rng(s).random((65536, 3), dtype=np.float32) for s in range(scenes)])
rs = torch.from_numpy(np.arange(scenes + 1, dtype=np.int64) * 65536)
t = torch.from_numpy(pts).to(dev)
nns = layers.FixedRadiusSearch()
for _ in range(reps):
    res = nns(t, t, 0.05, rs, rs)
torch.cuda.synchronize()
print("pairs", int(res.neighbors_row_splits[-1]))
