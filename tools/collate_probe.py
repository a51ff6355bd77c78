"""KPFCNN GPU collate (segmentation_inputs) on the C3 batch: wall ms per call,
cProfile split of the host time, and (with KTRACE=1) nothing else — run under
rocprofv3 --kernel-trace for the per-call kernel timeline."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd.kpfcnn import KPFCNN, S3DIS, segmentation_inputs  # noqa: E402

dev = torch.device("cuda", 0)
np.random.seed(0)
model = KPFCNN(**S3DIS)
pts_np, feat_np, lab_np, lengths = bench.make_c3(0)
pts = torch.from_numpy(pts_np).to(dev)
feat = torch.from_numpy(feat_np).to(dev)
lab = torch.from_numpy(lab_np).to(dev)
for _ in range(3):
    segmentation_inputs(model.cfg, pts, feat, lab, lengths)
torch.cuda.synchronize()
reps = int(os.environ.get("REPS", "10"))
t = time.perf_counter()
for _ in range(reps):
    segmentation_inputs(model.cfg, pts, feat, lab, lengths)
torch.cuda.synchronize()
print("ms per collate", (time.perf_counter() - t) / reps * 1e3, flush=True)
each = []
for _ in range(30):  # one by one (synchronised): median and min are robust to host jitter
    t = time.perf_counter()
    segmentation_inputs(model.cfg, pts, feat, lab, lengths)
    torch.cuda.synchronize()
    each.append((time.perf_counter() - t) * 1e3)
print("ms per collate median %.3f min %.3f" % (float(np.median(each)), min(each)), flush=True)
if os.environ.get("PROFILE", "1") == "1":
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        segmentation_inputs(model.cfg, pts, feat, lab, lengths)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
