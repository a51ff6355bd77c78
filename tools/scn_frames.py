"""SparseConvUnet eval frames (bench.scn_bench's model and input): median
ms per frame, host time to return vs GPU drain; for rocprofv3 runs.
  python tools/scn_frames.py N [prof | ops | split]"""
import os
import sys
import time
import types

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [R, os.path.join(R, "open3d-ml_amd")]
import bench  # noqa: E402
from o3dml_amd.sparseconvnet import SparseConvUnet  # noqa: E402

dev = torch.device("cuda", 0)
pos = torch.from_numpy(bench.make_room(0)[0]).to(dev)
torch.manual_seed(0)
m = SparseConvUnet(multiplier=32, residual_blocks=True, conv_block_reps=1, num_classes=20).to(dev).eval()
inp = types.SimpleNamespace(point=[pos], feat=[torch.rand((pos.shape[0], 3), device=dev)], batch_lengths=[pos.shape[0]])
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
with torch.no_grad():
    for _ in range(3):
        m(inp)
    torch.cuda.synchronize(dev)
    host, tot = [], []
    for _ in range(reps):
        t = time.perf_counter()
        m(inp)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        host.append(t1 - t)
        tot.append(t2 - t)
print(f"SCN frame: {np.median(tot)*1e3:.3f} ms (host return {np.median(host)*1e3:.3f} ms), voxels {pos.shape[0]}")

if len(sys.argv) > 2 and sys.argv[2] == "split":
    # mode 3: the plan call alone and the body replay alone (each synchronised)
    plan = m.__dict__["_o3dml_scn_plan"][1]
    bodies = m.__dict__["_o3dml_scn_plan_bodies"]
    body = next(iter(bodies.values()))
    tp, tb = [], []
    with torch.no_grad():
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            plan.run(inp.point[0], inp.feat[0])
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            body.graph.replay()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            tp.append(t1 - t)
            tb.append(t2 - t1)
    print(f"SCN plan call {np.median(tp)*1e3:.3f} ms, body replay {np.median(tb)*1e3:.3f} ms")

if len(sys.argv) > 2 and sys.argv[2] == "prof":
    import cProfile
    import pstats
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for _ in range(5):
            m(inp)
        torch.cuda.synchronize(dev)
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(40)

if len(sys.argv) > 2 and sys.argv[2] == "ops":
    # every aten op of one frame (count, device time) and where the memcpys come from
    from torch.profiler import ProfilerActivity, profile
    with torch.no_grad(), profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        m(inp)
        torch.cuda.synchronize(dev)
    print(prof.key_averages().table(sort_by="count", row_limit=45))
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25))
