"""Run the C4 SparseConvUnet forward (and, with TRAIN=1, forward+backward) a
few times for rocprofv3 kernel traces; prints the wall time per frame."""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd.sparseconvnet import SparseConvUnet  # noqa: E402

dev = torch.device("cuda", 0)
reps = int(os.environ.get("REPS", "5"))
train = os.environ.get("TRAIN", "0") == "1"
pos = torch.from_numpy(bench.make_room(0)[0]).to(dev)
torch.manual_seed(0)
m = SparseConvUnet(multiplier=32, residual_blocks=True, conv_block_reps=1, num_classes=20).to(dev)
m.train(train)
feat = torch.rand((pos.shape[0], 3), device=dev)
inp = types.SimpleNamespace(point=[pos], feat=[feat], batch_lengths=[pos.shape[0]])


def step():
    if train:
        out = m(inp)
        out.square().mean().backward()
    else:
        with torch.no_grad():
            m(inp)


step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    step()
torch.cuda.synchronize()
print("ms/frame", (time.perf_counter() - t) / reps * 1e3, "train" if train else "eval")
if os.environ.get("CPROFILE"):  # host-side split of one eval frame
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
if os.environ.get("TORCHPROF"):
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
        step()
        torch.cuda.synchronize()
    print(p.key_averages().table(sort_by="self_cuda_time_total", row_limit=30))
