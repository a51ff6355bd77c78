"""Host-side split of the C3 train step (bench.kpconv_bench's step): per
phase, the time to return from the Python call (host: launches, autograd,
host reads) and the time until the GPU drains; then a cProfile of 5 steps."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [R, os.path.join(R, "open3d-ml_amd")]
import bench  # noqa: E402
from o3dml_amd.kpfcnn import KPFCNN, S3DIS, segmentation_inputs  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = KPFCNN(**S3DIS).to(dev).train()
opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.98, weight_decay=0.001, fused=bench._fused_opt())
pts_np, feat_np, lab_np, lengths = bench.make_c3(0)
pts, feat, lab = (torch.from_numpy(a).to(dev) for a in (pts_np, feat_np, lab_np))


def step(rec=None):
    t0 = time.perf_counter()
    batch = segmentation_inputs(model.cfg, pts, feat, lab, lengths)
    t1 = time.perf_counter()
    loss = model.get_loss(model(batch), batch.labels)
    t2 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    t3 = time.perf_counter()
    opt.step()
    t4 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t5 = time.perf_counter()
    if rec is not None:
        rec.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0))


for _ in range(3):
    step()
rec = []
for _ in range(10):
    step(rec)
m = np.median(np.array(rec) * 1e3, 0)
print("host ms: collate %.2f fwd %.2f bwd %.2f opt %.2f | drain %.2f | step %.2f" % tuple(m))
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    step()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
