"""Sparse-conv GEMM microbenchmark on the C4 room voxels: the lattice map is
built once (rulebook_cache), then for several channel widths the forward GEMM
kernel alone (library HIP-event timing, as bench.py's mfma_roofline), the whole
forward call and the backward (dIn + dW) with autograd are timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd import _lib, layers, sparse_conv as sc  # noqa: E402

dev = torch.device("cuda", 0)
pos = torch.from_numpy(bench.make_room(0)[0]).to(dev)
reps = int(os.environ.get("REPS", "20"))
shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ.get("SHAPES", "32x32,64x64,128x128,64x32").split(",")]
for cin, cout in shapes:
    torch.manual_seed(0)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=False).to(dev)
    x = torch.rand((pos.shape[0], cin), device=dev)
    with sc.rulebook_cache():
        with torch.no_grad():
            conv(x, pos, pos, 1.0)
            nb, _ = conv._rulebook(pos, pos, 1.0, None, False, 1.0)
            pairs = int(nb.neighbors_index.shape[0])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                conv(x, pos, pos, 1.0)
            e1.record()
            torch.cuda.synchronize()
            fwd = e0.elapsed_time(e1) / reps
            # the GEMM kernel alone (HIP events around its launch in the library):
            # the call above can be host-bound at these sizes
            lib = _lib.load()
            lib.o3dml_timing_reset()
            lib.o3dml_timing_enable(1)
            for _ in range(reps):
                conv(x, pos, pos, 1.0)
            torch.cuda.synchronize()
            kms, kcnt = _lib.kernel_times(["sparse_conv_gemm"])["sparse_conv_gemm"]
            lib.o3dml_timing_enable(0)
            kern = kms / max(kcnt, 1)
        xg = x.clone().requires_grad_(True)
        out = conv(xg, pos, pos, 1.0)
        g = torch.rand_like(out)
        out.backward(g, retain_graph=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            torch.autograd.grad(out, [xg, conv.kernel], g, retain_graph=True)
        e1.record()
        torch.cuda.synchronize()
        bwd = e0.elapsed_time(e1) / reps
    fl = 2.0 * pairs * cin * cout
    print(f"cin {cin:4d} cout {cout:4d} pairs {pairs} gemm {kern * 1e3:7.1f} us {fl / kern / 1e9:6.2f} TF/s | "
          f"fwd {fwd * 1e3:8.1f} us {fl / fwd / 1e9:7.2f} TF/s | "
          f"bwd {bwd * 1e3:8.1f} us {2 * fl / bwd / 1e9:7.2f} TF/s", flush=True)
