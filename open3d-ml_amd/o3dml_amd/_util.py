"""Host-side plumbing shared by the op wrappers: device placement, streams,
workspaces and row-split handling.  PyTorch is used only for device memory and
streams; every computation runs in libo3dml_amd.so."""
from collections import OrderedDict

import numpy as np
import torch

from . import _lib


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError(
            "o3dml_amd: no ROCm GPU is visible. This build has no CPU fallback "
            "(the CPU restatement in oracle/ is test infrastructure only).")


def gpu_device(*tensors):
    """The GPU the op runs on: that of the first CUDA input, else the current one."""
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


class StreamHandle(int):
    """A hipStream_t (an int for ctypes) that remembers its device: _lib.call
    runs a call given one under a restoring device guard when that device is
    not the current one, so the library's launches, scratch streams and events
    (and torch's default stream handle, the null stream) belong to the device
    that holds the tensors, and the caller's current device is left as it was."""


def stream_handle(device):
    """The current torch stream of `device` (see StreamHandle); the raw handle
    straight from torch's stream registry (no Stream object per call)."""
    if not isinstance(device, torch.device):
        device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    h = StreamHandle(torch._C._cuda_getCurrentRawStream(idx))
    h.dev = idx
    return h


def ptr(t):
    return None if t is None else t.data_ptr()


def mm(a, b, ta=False, tb=False):
    """op(a) @ op(b) for contiguous row-major float32 CUDA matrices through
    rocBLAS (csrc/gemm.cpp o3dml_sgemm); ta / tb: use a.T / b.T."""
    from . import _lib
    m, k = (a.shape[1], a.shape[0]) if ta else a.shape
    n = b.shape[0] if tb else b.shape[1]
    c = torch.empty((m, n), dtype=torch.float32, device=a.device)
    if k >= 4096 and m * n <= (1 << 20):  # long reduction, few output tiles: split-K
        lib = _lib.load()
        ws = torch.empty(max(int(lib.o3dml_sgemm_splitk_workspace_size(m, n, k)), 1), dtype=torch.uint8,
                         device=a.device)
        _lib.call("o3dml_sgemm_splitk", int(ta), int(tb), m, n, k, a.data_ptr(), a.shape[1], b.data_ptr(),
                  b.shape[1], c.data_ptr(), n, ws.data_ptr(), ws.numel(), stream_handle(a.device))
        return c
    _lib.call("o3dml_sgemm", int(ta), int(tb), m, n, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1], 0.0,
              c.data_ptr(), n, stream_handle(a.device))
    return c


_SMALL_CACHE = OrderedDict()  # (device, stream, dtype, shape, bytes) -> device tensor
_SMALL_CACHE_MAX = 64
_SMALL_NUMEL = 4096


def to_dev(t, device, dtype=None):
    """Contiguous copy (or view) of t on device with dtype.  Host data goes
    through a pinned staging copy and a non-blocking transfer on the current
    stream (torch's caching host allocator keeps the staging buffer alive until
    the copy has run), so row splits and other small host arrays do not
    synchronise the stream with the host.  Small host integer arrays (row
    splits, table splits: the same few values call after call) are kept on the
    device in a small LRU cache keyed by their bytes, so a repeated batch
    layout costs no transfer at all; the ops only ever read these tensors.
    The cache key holds the current stream: an entry is only handed out on
    the stream its upload was queued on (so every use is ordered after the
    copy), and an evicted block returns to that stream's pool, the only one
    that ever used it."""
    if isinstance(t, torch.Tensor) and t.is_cuda and (dtype is None or t.dtype == dtype) and \
            t.device == (device if isinstance(device, torch.device) else torch.device(device)):
        return t if t.is_contiguous() else t.contiguous()  # already there: no copy, no device object
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(np.asarray(t))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if t.device.type == "cpu" and torch.device(device).type == "cuda":
        t = t.contiguous()
        if (t.numel() <= _SMALL_NUMEL and t.dtype in (torch.int32, torch.int64) and not t.requires_grad
                and not torch.cuda.is_current_stream_capturing()):
            key = (str(torch.device(device)), torch.cuda.current_stream(device).cuda_stream, t.dtype,
                   tuple(t.shape), t.numpy().tobytes())
            hit = _SMALL_CACHE.get(key)
            if hit is not None:
                _SMALL_CACHE.move_to_end(key)
                return hit
            d = t.pin_memory().to(device, non_blocking=True)
            _SMALL_CACHE[key] = d
            if len(_SMALL_CACHE) > _SMALL_CACHE_MAX:
                _SMALL_CACHE.popitem(last=False)
            return d
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device, non_blocking=False).contiguous()


class SizeCache:
    """Bounded memo of workspace-size queries (one ctypes call per new
    shape): keys carry per-batch point counts that change step to step, so
    the cache is an LRU of at most `cap` entries, not an ever-growing dict."""

    def __init__(self, query, cap=1024):
        self.query, self.cap, self.d = query, cap, OrderedDict()

    def __call__(self, *key):
        v = self.d.get(key)
        if v is None:
            v = self.d[key] = self.query(*key)
            if len(self.d) > self.cap:
                self.d.popitem(last=False)
        else:
            self.d.move_to_end(key)
        return v

    def __len__(self):
        return len(self.d)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def row_splits_host(rs, n):
    """int64 numpy row splits; None means one batch item [0, n]."""
    if rs is None:
        return np.array([0, n], np.int64)
    if isinstance(rs, torch.Tensor):
        rs = rs.detach().cpu().numpy()
    rs = np.ascontiguousarray(np.asarray(rs, dtype=np.int64))
    if rs.ndim != 1 or len(rs) < 2:
        raise RuntimeError("row_splits must be a 1-D tensor with at least 2 entries")
    if rs[0] != 0 or rs[-1] != n or np.any(np.diff(rs) < 0):
        raise RuntimeError(
            f"row_splits must start at 0, end at {n} and be non-decreasing (got {rs[0]}..{rs[-1]})")
    return rs


def scalar(x):
    if isinstance(x, torch.Tensor):
        return float(x.detach().cpu().reshape(-1)[0])
    return float(x)


def back_to(t, like):
    """Return t on the device of `like` (ops given CPU tensors return CPU tensors)."""
    if isinstance(like, torch.Tensor) and not like.is_cuda:
        return t.cpu()
    return t


def check_points(name, t, dims=3):
    if t.dim() != 2 or t.shape[1] != dims:
        raise RuntimeError(f"{name} must have shape [N, {dims}], got {list(t.shape)}")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32, got {t.dtype}")


INDEX_DTYPES = {torch.int32: 32, torch.int64: 64, 3: 32, 4: 64, "int32": 32, "int64": 64}


def index_bits(index_dtype):
    if index_dtype in INDEX_DTYPES:
        return INDEX_DTYPES[index_dtype]
    raise RuntimeError(f"index_dtype must be torch.int32 or torch.int64, got {index_dtype}")


METRICS = {"L1": 0, "L2": 1, "Linf": 2}


def metric_code(metric):
    if metric not in METRICS:
        raise RuntimeError(f"metric must be one of {list(METRICS)}, got {metric!r}")
    return METRICS[metric]


__all__ = ["require_gpu", "gpu_device", "stream_handle", "ptr", "to_dev", "workspace",
           "row_splits_host", "scalar", "SizeCache", "back_to", "check_points", "index_bits", "metric_code", "_lib"]
