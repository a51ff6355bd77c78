"""Does a hipMemsetAsync captured into a torch.cuda.graph take effect on
replay?  (the "wrong histograms" of the captured RandLA
crop selection and the miss counter of o3dml_randla_up_from_knn.)

Part 1: a raw hipMemsetAsync (ctypes into libamdhip64) between two torch
kernels inside a capture, for several sizes / offsets; the buffer is refilled
with a pattern before every replay, so a memset node that does not run (or
runs partly, or out of order) shows as pattern words left in the range.
Part 2: the library's own captured miss counter (up_from_knn: cntr zeroed by a
memset node, then appended to by the kernel) read back after each replay.
Prints one line per case; exit status 0 either way (it is a probe)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int
hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetD32Async.restype = ctypes.c_int

dev = torch.device("cuda", 0)
PAT = 0x12345678


def part1():
    for nbytes in (4, 8, 12, 16, 100, 4096, 24576, 26624, 1 << 20):
        for off in (0, 4):
            words = (off + nbytes) // 4 + 64
            buf = torch.full((words,), PAT, dtype=torch.int32, device=dev)
            out = torch.empty_like(buf)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st = torch.cuda.current_stream().cuda_stream
                buf.add_(1)  # a kernel before the memset (ordering)
                rc = hip.hipMemsetAsync(buf.data_ptr() + off, 0, nbytes, st)
                out.copy_(buf)  # a kernel after it (ordering)
            torch.cuda.synchronize()
            at_capture = int((buf[off // 4:(off + nbytes) // 4] == 0).sum())
            bad = []
            for rep in range(3):
                buf.fill_(PAT)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                b = buf.cpu().numpy()
                o = out.cpu().numpy()
                lo, hi = off // 4, (off + nbytes) // 4
                inside_nonzero = int((b[lo:hi] != 0).sum())
                outside_bad = int((b[:lo] != PAT + 1).sum() + (b[hi:] != PAT + 1).sum())
                out_diff = int((o != b).sum())
                bad.append((inside_nonzero, outside_bad, out_diff))
            ok = all(x == (0, 0, 0) for x in bad)
            print(f"memset node bytes={nbytes:8d} off={off}: rc={rc} zeroed_at_capture={at_capture} "
                  f"replays(inside_nonzero, outside_wrong, copy_diff)={bad} -> {'OK' if ok else 'BROKEN'}",
                  flush=True)
            del g


def part1b():
    """The same for a raw device-to-device hipMemcpyAsync node."""
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpyAsync.restype = ctypes.c_int
    for nbytes in (8, 16, 4096, 1 << 20):
        words = nbytes // 4
        src = torch.arange(words, dtype=torch.int32, device=dev)
        dst = torch.full((words,), PAT, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            rc = hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), nbytes, 3, torch.cuda.current_stream().cuda_stream)
        bad = []
        for rep in range(3):
            dst.fill_(PAT)
            src.add_(1)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            bad.append(int((dst != src).sum()))
        print(f"memcpy D2D node bytes={nbytes:8d}: rc={rc} replays(words differing)={bad} -> "
              f"{'OK' if not any(bad) else 'BROKEN'}", flush=True)
        del g


def part2():
    from o3dml_amd import _lib, ops
    from o3dml_amd._util import ptr, stream_handle
    lib = _lib.load()
    rng = np.random.default_rng(0)
    sizes = [8192, 2048, 512, 128, 32]  # RandLA levels: prefixes of one shuffled patch
    L = 4
    pc = torch.from_numpy(rng.random((sizes[0], 3), dtype=np.float32)).to(dev)
    cat = torch.cat([pc[:s] for s in sizes[:L]]).contiguous()
    rs = np.concatenate([[0], np.cumsum(sizes[:L])]).astype(np.int64)
    srs = np.concatenate([[0], np.cumsum(sizes[1:])]).astype(np.int64)
    nxt = np.asarray(sizes[1:], np.int64)
    nb0 = ops.knn_search(cat, cat, 16, rs, rs).neighbors_index.view(-1, 16).contiguous()
    total = int(rs[-1])
    nb = torch.empty_like(nb0)
    up = torch.empty(total, dtype=torch.int64, device=dev)
    ws = torch.empty(lib.o3dml_randla_up_workspace_size(total), dtype=torch.uint8, device=dev)

    def step():
        nb.copy_(nb0)
        _lib.call("o3dml_randla_up_from_knn", ptr(nb), 16, ptr(cat), L, rs.ctypes.data, nxt.ctypes.data,
                  srs.ctypes.data, ptr(up), ptr(ws), ws.numel(), stream_handle(dev))

    step()
    torch.cuda.synchronize()
    eager = int(ws[:4].view(torch.int32).item())
    ref_up = up.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    counts = []
    for _ in range(5):
        g.replay()
        torch.cuda.synchronize()
        counts.append(int(ws[:4].view(torch.int32).item()))
    same = torch.equal(up, ref_up)
    print(f"up_from_knn miss counter: eager {eager}, after each replay {counts}, list capacity {total}, "
          f"up equal {same} -> {'OK' if all(c == eager for c in counts) else 'COUNTER NOT RESET BY THE MEMSET NODE'}",
          flush=True)


if __name__ == "__main__":
    print("torch", torch.__version__, "hip", torch.version.hip, flush=True)
    part1()
    part1b()
    part2()
