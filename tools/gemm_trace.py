"""Per-wave timeline of the sparse-conv LDS GEMM (implicit_gemm_lds_kernel) on
the C4 room voxels, from a diagnostic build of the library:
    make -C open3d-ml_amd/csrc BUILD=../build_trace LIBDIR=../lib_trace EXTRA=-DO3DML_GEMM_TRACE=1
One warm forward GEMM per shape is traced: every
wave stamps its phases with the 100-MHz real-time counter (slots documented at
O3DML_GEMM_TRACE in csrc/sparse_conv.hip).  Prints the phase durations
(median / p90 over waves), the resident-wave count over the kernel's span and
the waves per XCD.
usage: python tools/gemm_trace.py   (SHAPES=32x32,64x32 as tools/gemm_probe.py)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("O3DML_AMD_LIB", os.path.join(ROOT, "open3d-ml_amd", "lib_trace", "libo3dml_amd.so"))
os.environ.setdefault("O3DML_GEMM_PERSIST", "0")  # one wave per item: wave = tile
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd import _lib, layers, sparse_conv as sc  # noqa: E402

SLOTS, WAVES = 16, 1 << 16
TICK_NS = 10.0  # s_memrealtime: 100 MHz

lib = _lib.load()
lib.o3dml_gemm_trace_read.restype = ctypes.c_int
lib.o3dml_gemm_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.o3dml_gemm_trace_clear.restype = ctypes.c_int


def read_trace():
    buf = np.zeros(WAVES * SLOTS, dtype=np.uint64)
    assert lib.o3dml_gemm_trace_read(buf.ctypes.data, buf.nbytes) == 0
    return buf.reshape(WAVES, SLOTS)


def pct(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return "-"
    return f"{np.median(v):7.0f} / {np.percentile(v, 90):7.0f}"


def report(t):
    live = t[:, 13] != 0
    t = t[live].astype(np.int64)
    n = t.shape[0]
    if n == 0:
        print("  no waves traced (cout >= 64 runs the shared-A kernel, not traced)")
        return
    t0 = t[:, 0].min()
    span = (t[:, 13].max() - t0) * TICK_NS
    print(f"  waves traced {n}, kernel span {span / 1e3:.1f} us (first entry -> last store)")
    ns = lambda a, b: (t[:, b] - t[:, a]) * TICK_NS  # noqa: E731
    print("  phase (ns, median / p90):")
    print(f"    entry -> rows in LDS      {pct(ns(0, 1))}")
    print(f"    rows -> map tile in LDS   {pct(ns(1, 2))}")
    print(f"    map tile -> offset mask   {pct(ns(2, 3))}")
    st = t[:, 14]
    has = st > 0
    print(f"    mask -> stage 0 landed    {pct(ns(3, 4)[has])}")
    for k in range(1, 8):
        m = st > k
        if m.sum() > 0:
            print(f"    stage {k - 1} -> stage {k} landed  {pct((t[m, 4 + k] - t[m, 3 + k]) * TICK_NS)}  ({m.sum()} waves)")
    last = np.clip(st - 1, 0, 7)
    m = has & (st <= 8)
    print(f"    last stage -> stages done {pct((t[m, 12] - t[m, 4 + last[m]]) * TICK_NS)}")
    print(f"    stages done -> stored     {pct(ns(12, 13))}")
    print(f"    wave lifetime             {pct(ns(0, 13))}")
    print(f"  stages per wave: mean {st.mean():.2f}, max {st.max()}")
    # resident waves over the span (20 bins)
    bins = np.linspace(t0, t[:, 13].max(), 21)
    mid = 0.5 * (bins[1:] + bins[:-1])
    res = [int(((t[:, 0] <= x) & (t[:, 13] >= x)).sum()) for x in mid]
    print("  resident waves over the span (20 bins):", res)
    starts = np.histogram(t[:, 0], bins)[0]
    print("  wave starts per bin:                    ", starts.tolist())
    xcc = (t[:, 15] >> 32) & 0xF
    print("  waves per XCC:", np.bincount(xcc.astype(np.int64), minlength=8).tolist())


dev = torch.device("cuda", 0)
pos = torch.from_numpy(bench.make_room(0)[0]).to(dev)
shapes = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("SHAPES", "32x32,64x32").split(",")]
for cin, cout in shapes:
    torch.manual_seed(0)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=False).to(dev)
    x = torch.rand((pos.shape[0], cin), device=dev)
    with sc.rulebook_cache(), torch.no_grad():
        for _ in range(3):
            conv(x, pos, pos, 1.0)
        torch.cuda.synchronize()
        assert lib.o3dml_gemm_trace_clear() == 0
        conv(x, pos, pos, 1.0)
        torch.cuda.synchronize()
    print(f"cin {cin} cout {cout}:", flush=True)
    report(read_trace())
