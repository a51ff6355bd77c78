"""Run the C4 sparse-conv layer a few times (rocprofv3 kernel traces / PMC)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
print(bench.sparse_conv_bench(dev, int(os.environ.get("REPS", "5"))))
