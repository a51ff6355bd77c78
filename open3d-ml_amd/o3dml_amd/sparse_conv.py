"""Sparse convolution ops with autograd, mirroring
Open3D's ``ops.sparse_conv`` / ``ops.sparse_conv_transpose`` signatures.

The neighbourhood arrives as CSR pairs over OUTPUT points (neighbors_index,
neighbors_kernel_index, neighbors_row_splits); the HIP library turns it into a
dense kernel map and runs the MFMA implicit GEMM (forward), the inverse-map
GEMM with W^T (input gradient) and split-K slabs (filter gradient)."""
import collections
import contextlib

import numpy as np
import torch

from . import _lib
from ._util import SizeCache, gpu_device, ptr, stream_handle, to_dev, workspace


def _opt(t, dev, dtype=torch.float32):
    if t is None or (isinstance(t, torch.Tensor) and t.numel() == 0):
        return None
    return to_dev(t, dev, dtype)



# Tile order (o3dml_sparse_conv_tile_order) for a map used once: only when the
# GEMM is wide enough that the saved MFMA work beats the sort's few launches.
TILE_ORDER_MIN_CHANNELS = 64 * 64

def _build_map(nidx, kidx, nimp, rs, n_in, K, normalize, out_importance, want_inv, tile_order, dev, st):
    """Dense kernel map of the CSR pairs (o3dml_sparse_conv_build_map)."""
    lib = _lib.load()
    n_out = rs.shape[0] - 1
    mws = workspace(lib.o3dml_sparse_conv_map_workspace_size(n_out, n_in, K), dev)
    status = np.zeros(1, np.int32)
    _lib.call("o3dml_sparse_conv_build_map", ptr(nidx), ptr(kidx), ptr(nimp), ptr(rs), n_out, n_in, K,
              int(bool(normalize)), ptr(out_importance), int(bool(want_inv)), status.ctypes.data, ptr(mws),
              mws.numel(), st)
    if status[0] & 2:
        raise RuntimeError("sparse_conv: neighbors_kernel_index out of range for the filter")
    if status[0] & 8:
        raise RuntimeError(f"sparse_conv: neighbors_index out of range [0, {n_in})")
    if status[0] & 1:  # handled by _conv_layers
        raise _DuplicateKernelIndex()
    if tile_order:
        _lib.call("o3dml_sparse_conv_tile_order", ptr(mws), mws.numel(), n_out, n_in, K, int(bool(want_inv)), st)
    return mws, n_out


def _backward(W, x, mws, sscale, meta, grad_out, need_w, need_x):
    """(dW, dIn) through o3dml_sparse_conv_backward on a map built with the
    inverse map (want_inv)."""
    K, cin, cout, n_in, n_out, has_nimp, use_os, has_ss = meta[:8]
    dev = grad_out.device
    lib = _lib.load()
    g = grad_out.contiguous().float()
    gx = torch.empty((n_in, cin), dtype=torch.float32, device=dev) if need_x else None
    gw = torch.empty(W.shape, dtype=torch.float32, device=dev) if need_w else None
    ws = workspace(lib.o3dml_sparse_conv_backward_workspace_size(n_out, n_in, K, cin, cout), dev)
    _lib.call("o3dml_sparse_conv_backward", ptr(W), K, cin, cout, ptr(x), n_in, ptr(sscale) if has_ss else None,
              int(has_nimp), use_os, ptr(g), n_out, ptr(gx), ptr(gw), ptr(mws), mws.numel(), ptr(ws), ws.numel(),
              stream_handle(dev))
    return gw, gx


class _ConvFn(torch.autograd.Function):
    """out = oscale * sum_k gather(x * sscale * pscale) @ W[k] (+ bias)."""

    @staticmethod
    def forward(ctx, filters, inp_features, bias, nidx, kidx, nimp, rs, sscale, normalize, out_importance,
                want_grad, prebuilt=None):
        dev = inp_features.device
        lib = _lib.load()
        K = int(np.prod(filters.shape[:-2]))
        cin, cout = int(filters.shape[-2]), int(filters.shape[-1])
        if inp_features.dim() != 2 or inp_features.shape[1] != cin:
            raise RuntimeError(f"sparse_conv: inp_features must be [N, {cin}], got {list(inp_features.shape)}")
        n_in = inp_features.shape[0]
        st = stream_handle(dev)
        if prebuilt is not None:  # dense map already built (lattice rulebook)
            mws, n_out = prebuilt
        else:  # the inverse map serves dIn / dW only
            mws, n_out = _build_map(nidx, kidx, nimp, rs, n_in, K, normalize, out_importance, want_grad,
                                    cin * cout >= TILE_ORDER_MIN_CHANNELS, dev, st)
        W = filters.detach().contiguous()
        x = inp_features.detach().contiguous()
        out = torch.empty((n_out, cout), dtype=torch.float32, device=dev)
        use_os = int(bool(normalize) or out_importance is not None)
        fws = workspace(lib.o3dml_sparse_conv_forward_workspace_size(n_out, n_in, K, cin, cout), dev)
        _lib.call("o3dml_sparse_conv_forward", ptr(W), K, cin, cout, ptr(x), n_in, ptr(sscale), int(nimp is not None),
                  use_os, ptr(bias.detach().contiguous() if bias is not None else None), n_out, ptr(out), ptr(mws),
                  mws.numel(), ptr(fws), fws.numel(), st)
        ctx.save_for_backward(W, x, mws, sscale if sscale is not None else torch.empty(0, device=dev))
        ctx.meta = (K, cin, cout, n_in, n_out, nimp is not None, use_os, sscale is not None, bias is not None)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        W, x, mws, sscale = ctx.saved_tensors
        gw, gx = _backward(W, x, mws, sscale, ctx.meta, grad_out, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        gb = grad_out.float().sum(0) if (ctx.meta[8] and ctx.needs_input_grad[2]) else None
        return gw, gx, gb, None, None, None, None, None, None, None, None, None


def conv_grads(filters, inp_features, grad_out, neighbors_index, neighbors_kernel_index, neighbors_importance,
               neighbors_row_splits, sscale, normalize, out_importance, need_w=True, need_x=True):
    """(dW, dIn) of _conv's output given grad_out, without the forward GEMM:
    the map (with its inverse) is rebuilt and the backward kernels run —
    the backward of the registered ``torch.ops.open3d.sparse_conv*`` ops."""
    dev = gpu_device(inp_features, filters)
    W = filters.to(dev).detach().contiguous()
    x = inp_features.to(dev).detach().contiguous()
    nidx = to_dev(neighbors_index, dev, torch.int32)
    kidx = to_dev(neighbors_kernel_index, dev, torch.int32)
    rs = to_dev(neighbors_row_splits, dev, torch.int64)
    nimp = _opt(neighbors_importance, dev)
    oimp = _opt(out_importance, dev)
    K = int(np.prod(W.shape[:-2]))
    cin, cout = int(W.shape[-2]), int(W.shape[-1])
    try:
        mws, n_out = _build_map(nidx, kidx, nimp, rs, x.shape[0], K, normalize, oimp, True,
                                cin * cout >= TILE_ORDER_MIN_CHANNELS, dev, stream_handle(dev))
    except _DuplicateKernelIndex:
        # off-lattice rulebook (pairs sharing an (output, k) or (input, k)):
        # the forward split the pairs into layers (_conv_layers), so does this
        # backward — the layered forward re-run on detached leaves and
        # differentiated by autograd (each layer's backward is the HIP kernel)
        return _layered_grads(W, x, grad_out.to(dev), nidx, kidx, nimp, rs, sscale, normalize, oimp, K,
                              need_w, need_x)
    use_os = int(bool(normalize) or oimp is not None)
    meta = (K, cin, cout, x.shape[0], n_out, nimp is not None, use_os, sscale is not None)
    ss = sscale if sscale is not None else torch.empty(0, device=dev)
    return _backward(W, x, mws, ss, meta, grad_out.to(dev), need_w, need_x)


class _DuplicateKernelIndex(Exception):
    """Two neighbours of one output share a kernel index (see _conv_layers)."""


def _layered_grads(W, x, grad_out, nidx, kidx, nimp, rs, sscale, normalize, oimp, K, need_w, need_x):
    """(dW, dIn) of _conv_layers' output: its forward on fresh leaves, then
    torch.autograd.grad (every layer's backward runs the HIP dW / dIn kernels)."""
    if not (need_w or need_x):
        return None, None
    wl = W.detach().requires_grad_(need_w)
    xl = x.detach().requires_grad_(need_x)
    with torch.enable_grad():
        out = _conv_layers(wl, xl, None, nidx, kidx, nimp, rs, sscale, bool(normalize), oimp, K)
        leaves = [t for t, need in ((wl, need_w), (xl, need_x)) if need]
        grads = torch.autograd.grad(out, leaves, grad_out.float(), allow_unused=True)
    it = iter(grads)
    gw = next(it) if need_w else None
    gx = next(it) if need_x else None
    if need_w and gw is None:
        gw = torch.zeros_like(W)
    if need_x and gx is None:
        gx = torch.zeros_like(x)
    return gw, gx


def _conv_layers(f, x, b, nidx, kidx, nimp, rs, sscale, normalize, oimp, K):
    """Open3D sums EVERY (neighbour, kernel index) pair of an output; the dense
    kernel map holds one input per (output, kernel index) and its inverse (the
    input gradient) one output per (input, kernel index).  Off one voxel
    lattice (layers.SparseConv on arbitrary positions) pairs share those, so
    the pairs are split into layers, each a valid pair of maps: every round
    takes each remaining pair that comes first (in CSR order) among the
    remaining pairs of its (output, k) AND of its (input, k) — a matching,
    never empty (the first remaining pair qualifies).  out = sum of the
    layers' HIP GEMMs (each its own autograd node), then the per-output
    normalisation / importance over ALL the output's pairs.  Index
    bookkeeping only in torch."""
    dev = x.device
    n_out = rs.shape[0] - 1
    n_in = x.shape[0]
    P = nidx.shape[0]
    counts = rs[1:] - rs[:-1]
    o = torch.repeat_interleave(torch.arange(n_out, device=dev), counts)
    ko = o * K + kidx.long()
    ki = nidx.long() * K + kidx.long()
    pos = torch.arange(P, device=dev)
    left = torch.ones(P, dtype=torch.bool, device=dev)
    big = torch.iinfo(torch.int64).max
    layers = []
    while bool(left.any()):
        p_left = torch.where(left, pos, torch.full_like(pos, big))
        m_o = torch.full((n_out * K,), big, dtype=torch.int64, device=dev).scatter_reduce_(0, ko, p_left, "amin")
        m_i = torch.full((n_in * K,), big, dtype=torch.int64, device=dev).scatter_reduce_(0, ki, p_left, "amin")
        take = left & (m_o[ko] == pos) & (m_i[ki] == pos)
        layers.append(torch.nonzero(take).squeeze(1))  # CSR order kept: rows stay grouped by output
        left &= ~take
    want_grad = torch.is_grad_enabled() and (f.requires_grad or x.requires_grad or (b is not None and b.requires_grad))
    out = None
    for layer, sel in enumerate(layers):
        c = torch.bincount(o[sel], minlength=n_out)
        lrs = torch.zeros(n_out + 1, dtype=torch.int64, device=dev)
        lrs[1:] = torch.cumsum(c, 0)
        part = _ConvFn.apply(f, x, b if layer == 0 else None, nidx[sel].contiguous(), kidx[sel].contiguous(),
                             None if nimp is None else nimp[sel].contiguous(), lrs, sscale, False, None, want_grad)
        out = part if out is None else out + part
    scale = None
    if normalize:
        w = nimp if nimp is not None else torch.ones(P, dtype=torch.float32, device=dev)
        den = torch.zeros(n_out, dtype=torch.float32, device=dev).index_add_(0, o, w)
        scale = torch.where(den != 0, 1.0 / den, torch.ones_like(den))  # as Open3D: no division by 0
    if oimp is not None:
        scale = oimp if scale is None else scale * oimp
    if scale is not None:
        if b is not None:  # Open3D scales the convolution, then adds the bias
            out = (out - b) * scale[:, None] + b
        else:
            out = out * scale[:, None]
    return out


def _conv(filters, inp_features, bias, neighbors_index, neighbors_kernel_index, neighbors_importance,
          neighbors_row_splits, sscale, normalize, out_importance):
    dev = gpu_device(inp_features, filters)
    back_cpu = not inp_features.is_cuda
    f = filters.to(dev) if not filters.is_cuda else filters
    x = inp_features.to(dev) if back_cpu else inp_features
    if f.dtype != torch.float32 or x.dtype != torch.float32:
        raise RuntimeError("sparse_conv: filters and features must be float32")
    nidx = to_dev(neighbors_index, dev, torch.int32)
    kidx = to_dev(neighbors_kernel_index, dev, torch.int32)
    rs = to_dev(neighbors_row_splits, dev, torch.int64)
    nimp = _opt(neighbors_importance, dev)
    oimp = _opt(out_importance, dev)
    b = None if bias is None else (bias.to(dev) if not bias.is_cuda else bias)
    want_grad = torch.is_grad_enabled() and (f.requires_grad or x.requires_grad or
                                             (b is not None and b.requires_grad))
    try:
        out = _ConvFn.apply(f, x, b, nidx, kidx, nimp, rs, sscale, bool(normalize), oimp, want_grad)
    except _DuplicateKernelIndex:
        out = _conv_layers(f, x, b, nidx, kidx, nimp, rs, sscale, bool(normalize), oimp,
                           int(np.prod(f.shape[:-2])))
    return out.cpu() if back_cpu else out


def sparse_conv(filters, inp_features, inp_importance, neighbors_index, neighbors_kernel_index,
                neighbors_importance, neighbors_row_splits, normalize=False, max_temp_mem_MB=64):
    """Open3D ``ops.sparse_conv``: out[o] = sum over o's neighbours n of
    W[kidx_n]^T (in[idx_n] * inp_importance[idx_n] * neighbors_importance[n]),
    divided by the neighbour count (or importance sum) if normalize.
    filters [*kernel_size, Cin, Cout]; empty importance tensors mean none."""
    dev = gpu_device(inp_features, filters)
    ss = _opt(inp_importance, dev)
    return _conv(filters, inp_features, None, neighbors_index, neighbors_kernel_index, neighbors_importance,
                 neighbors_row_splits, ss, normalize, None)


def sparse_conv_transpose(filters, out_importance, inp_features, inp_neighbors_index,
                          inp_neighbors_importance_sum, inp_neighbors_row_splits, neighbors_index,
                          neighbors_kernel_index, neighbors_importance, neighbors_row_splits, normalize=False,
                          max_temp_mem_MB=64):
    """Open3D ``ops.sparse_conv_transpose``.  neighbors_* is the CSR over the
    OUTPUT points (their input neighbours, with the kernel index of the pair);
    inp_neighbors_* is the same relation per INPUT point and, with normalize,
    each input's contribution is divided by its importance sum (or neighbour
    count).  out_importance scales the outputs."""
    ss = transpose_scale(inp_features, filters, inp_neighbors_importance_sum, inp_neighbors_row_splits, normalize,
                         neighbors_importance)
    return _conv(filters, inp_features, None, neighbors_index, neighbors_kernel_index, neighbors_importance,
                 neighbors_row_splits, ss, False, out_importance)


def transpose_scale(inp_features, filters, inp_neighbors_importance_sum, inp_neighbors_row_splits, normalize,
                    neighbors_importance=None):
    """Per-input scale of sparse_conv_transpose(normalize=True): 1 / (importance
    sum or neighbour count), 1 where that is 0; None without normalize.  The
    importance sum counts only when per-pair importances are given (Open3D's
    NEIGHBOR_IMPORTANCE switch is neighbors_importance being non-empty †);
    otherwise the neighbour count divides, whatever sum the caller passes."""
    if not normalize:
        return None
    dev = gpu_device(inp_features, filters)
    has_imp = neighbors_importance is not None and neighbors_importance.numel() > 0
    s = _opt(inp_neighbors_importance_sum, dev) if has_imp else None
    if s is None:
        irs = to_dev(inp_neighbors_row_splits, dev, torch.int64)
        s = (irs[1:] - irs[:-1]).float()
    ss = torch.where(s != 0, 1.0 / s, torch.ones_like(s)).contiguous()
    if ss.numel() != inp_features.shape[0]:
        raise RuntimeError("sparse_conv_transpose: inp_neighbors_* must describe every input point")
    return ss


def conv_with_bias(filters, bias, inp_features, neighbors_index, neighbors_kernel_index, neighbors_row_splits,
                   inp_importance=None, normalize=False):
    """Fused forward used by the layers: bias added in the MFMA epilogue."""
    dev = gpu_device(inp_features, filters)
    return _conv(filters, inp_features, bias, neighbors_index, neighbors_kernel_index, None, neighbors_row_splits,
                 _opt(inp_importance, dev), normalize, None)


class _RulebookScope:
    """Kernel maps of one rulebook_cache() scope, and the lattice checks whose
    device status words are still to be read (defer_checks)."""

    def __init__(self, defer_checks):
        self.maps = {}
        self.defer = defer_checks
        self.pending = []
        self.derived = 0  # transpose maps derived from their convolution partner (_transpose_of_cached)
        self.searches = 0  # layers that built the search rulebook (host round trips: not graph-capturable)
        self.ready = {}  # key -> event of a map built on another stream (prefetch_lattice_map)
        # maps still to be built ahead on `ahead_stream`: callables, one per map,
        # returning True when they launched work; pump() runs the next one
        self.ahead = collections.deque()
        self.ahead_stream = None

    def pump(self):
        """Builds the next queued map on the ahead stream (called after every
        lattice convolution's GEMM launch, so the map builds interleave with the
        GEMMs in launch order — and in a captured graph's node order)."""
        while self.ahead:
            job = self.ahead.popleft()
            with torch.cuda.stream(self.ahead_stream):
                if job():
                    return

    def check(self):
        """One host round trip for every deferred lattice check of the scope:
        True when all were lattice sets (their maps are valid)."""
        if not self.pending:
            return True
        st = torch.cat(self.pending).cpu()
        self.pending.clear()
        if bool((st & 1).any()):
            raise RuntimeError("sparse_conv: two neighbours of one output share a kernel index")
        return not bool((st & 4).any())


_SCOPE = None  # the active rulebook_cache() scope


def active_scope():
    """The active rulebook_cache() scope, or None."""
    return _SCOPE


def note_search_rulebook():
    """A layer built its rulebook with the fixed-radius search (not the lattice
    map): counted in the active scope (sparseconvnet._ScnHead / _ScnTail then do not
    capture the body: the search reads sizes back to the host)."""
    if _SCOPE is not None:
        _SCOPE.searches += 1


@contextlib.contextmanager
def rulebook_scope(scope):
    """Make an existing _RulebookScope the active one (a graph captured in
    parts continues one scope: the later part finds the earlier part's maps)."""
    global _SCOPE
    prev, _SCOPE = _SCOPE, scope
    try:
        yield scope
    finally:
        _SCOPE = prev


def scope_from(maps, defer_checks=True):
    """A fresh scope that starts with the given kernel maps."""
    sc_ = _RulebookScope(defer_checks)
    sc_.maps = dict(maps)
    return sc_


@contextlib.contextmanager
def rulebook_cache(defer_checks=False):
    """Reuse dense kernel maps inside the scope: layers with the same input /
    output positions, kernel size and offset (every same-level submanifold
    convolution of a SparseConvUnet) share one rulebook.
    Entries hold the position tensors, so their identities stay unique.

    defer_checks: the lattice test of each new map stays on the device (no
    host sync per layer; a failed test leaves an all-empty map); the caller
    must call scope.check() before using the results and recompute without
    deferral when it returns False."""
    global _SCOPE
    prev, _SCOPE = _SCOPE, _RulebookScope(defer_checks)
    try:
        yield _SCOPE
    finally:
        _SCOPE = prev


def _build_lattice_map(scope, key, cache_key, ip, qp, query_shift, n_in, n_out, ks, voxel_size, mirror, normalize,
                       oimp, want_grad, chans, dev):
    """Builds (on the current stream) and, with a key, caches in the scope one
    lattice kernel map: (map workspace, host status, late status word)."""
    lib = _lib.load()
    K = ks ** 3
    late = None
    # the lattice test stays on the device in a deferring scope and in a
    # standalone call; the latter reads it once after the GEMM (a failed
    # test leaves an all-empty, safe map, and the caller recomputes with the
    # search rulebook), so no host round trip sits between map and GEMM
    defer = (scope is None or scope.defer) and n_in > 0 and n_out > 0
    mws = workspace(lib.o3dml_sparse_conv_map_workspace_size(n_out, n_in, K), dev)
    lws = workspace(lib.o3dml_sparse_conv_lattice_workspace_size(n_in), dev)
    status = np.zeros(1, np.int32)
    qsh = None if query_shift is None else np.asarray(query_shift, np.float32).reshape(3)
    _lib.call("o3dml_sparse_conv_lattice_map_shifted", ptr(ip), n_in, ptr(qp),
              None if qsh is None else qsh.ctypes.data, n_out, float(voxel_size), ks,
              int(bool(mirror)), int(bool(normalize)), ptr(oimp), int(bool(want_grad)), int(defer),
              status.ctypes.data, ptr(mws), mws.numel(), ptr(lws), lws.numel(), stream_handle(dev))
    status0 = int(status[0])
    if K > 8 and (scope is not None or chans >= TILE_ORDER_MIN_CHANNELS) and not status0 & 4:
        # (no tile orders for K <= 8, csrc use_order) cached maps serve several
        # convolutions: sort the GEMM tiles by offset mask once
        _lib.call("o3dml_sparse_conv_tile_order", ptr(mws), mws.numel(), n_out, n_in, K, int(bool(want_grad)),
                  stream_handle(dev))
    if defer:
        off = lib.o3dml_sparse_conv_map_status_offset(n_out, n_in, K)
        if scope is None:
            late = mws[off:off + 4].view(torch.int32)
        else:
            scope.pending.append(mws[off:off + 4].view(torch.int32))
    if key is not None:
        scope.maps[key] = (mws, status0, cache_key[0], cache_key[1])
    return mws, status0, late


def _scope_key(ks, mirror, normalize, want_grad, voxel_size, cache_key):
    key = (ks, bool(mirror), bool(normalize), bool(want_grad), float(voxel_size)) + tuple(cache_key[2:])
    return key + (id(cache_key[0]), cache_key[0]._version, id(cache_key[1]), cache_key[1]._version)


def prefetch_lattice_map(ks, inp_positions, out_positions, voxel_size, mirror, sign, offset, query_shift):
    """Builds, on the CURRENT stream, the eval-mode lattice map a layer of
    kernel size ks, offset (host floats) and direction (mirror, sign) would
    build for (inp_positions -> out_positions) in the active scope, and records
    an event the layer's stream waits for when it finds the map
    (conv_lattice).  A SparseConvTranspose whose SparseConv partner is in the
    scope is derived from it, as conv_lattice does.  No-op outside a scope or
    when the map is there already."""
    scope = _SCOPE
    if scope is None:
        return False
    dev = out_positions.device
    cache_key = (inp_positions, out_positions, sign) + tuple(offset)
    key = _scope_key(ks, mirror, False, False, voxel_size, cache_key)
    if key in scope.maps:
        return False
    n_in, n_out = int(inp_positions.shape[0]), int(out_positions.shape[0])
    hit = _transpose_of_cached(scope, key, cache_key, ks, n_in, n_out, False, dev) if mirror else None
    if hit is None:
        _build_lattice_map(scope, key, cache_key, inp_positions, out_positions, query_shift, n_in, n_out, ks,
                           voxel_size, mirror, False, None, False, 0, dev)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    scope.ready[key] = ev
    return True


def conv_lattice(filters, bias, inp_features, inp_positions, query_positions, voxel_size, mirror=False,
                 inp_importance=None, normalize=False, out_importance=None, cache_key=None, pre=None, residual=None,
                 query_shift=None):
    """Layer forward with the lattice rulebook (dense kernel map straight from a
    voxel hash; csrc/sparse_conv.hip o3dml_sparse_conv_lattice_map).  Returns
    None when the positions are not on one voxel lattice — the caller then
    builds the rulebook with the Linf fixed-radius search (same map).
    query_shift: 3 floats (f32 values) the map kernels subtract from
    query_positions (the layer's offset * voxel size, same bits as the torch
    expression)."""
    dev = gpu_device(inp_features, filters)
    ks = int(filters.shape[0])
    if tuple(filters.shape[:3]) != (ks, ks, ks) or ks > 3:
        return None
    x = to_dev(inp_features, dev)
    ip = to_dev(inp_positions, dev, torch.float32)
    lazy_q = callable(query_positions)  # layers pass a builder: only a cache miss needs the queries
    qp = None if lazy_q else to_dev(query_positions, dev, torch.float32)
    lib = _lib.load()
    K = ks ** 3
    n_in = ip.shape[0]
    n_out = cache_key[1].shape[0] if lazy_q else qp.shape[0]
    b = None if bias is None else bias.to(dev)
    want_grad = torch.is_grad_enabled() and (filters.requires_grad or x.requires_grad or
                                             (b is not None and b.requires_grad))
    oimp = _opt(out_importance, dev)
    key = None
    scope = _SCOPE
    if scope is not None and cache_key is not None and out_importance is None:
        key = _scope_key(ks, mirror, normalize, want_grad, voxel_size, cache_key)
    hit = scope.maps.get(key) if key is not None else None
    if hit is None and key is not None and mirror:
        hit = _transpose_of_cached(scope, key, cache_key, ks, n_in, n_out, want_grad, dev)
    late = None  # status word read after the GEMM (standalone call, no scope)
    if hit is not None:
        mws, status0 = hit[0], hit[1]
        ev = scope.ready.pop(key, None)
        if ev is not None:  # built on the scope's map stream (prefetch_lattice_map)
            torch.cuda.current_stream(dev).wait_event(ev)
    else:
        if lazy_q:
            qp = to_dev(query_positions(), dev, torch.float32)
        mws, status0, late = _build_lattice_map(scope, key, cache_key, ip, qp, query_shift, n_in, n_out, ks,
                                                voxel_size, mirror, normalize, oimp, want_grad,
                                                int(filters.shape[3]) * int(filters.shape[4]), dev)
    if status0 & 4:
        return None
    if status0 & 1:
        raise RuntimeError("sparse_conv: two neighbours of one output share a kernel index")
    f = filters.to(dev)
    if pre is not None or residual is not None:
        # inference-only fused form: relu(x * pre[0] + pre[1]) gathered, + residual
        if want_grad or inp_importance is not None or normalize or out_importance is not None:
            raise RuntimeError("sparse_conv: fused prologue/residual is inference-only without importance")
        cin, cout = int(f.shape[3]), int(f.shape[4])
        out = torch.empty((n_out, cout), dtype=torch.float32, device=dev)
        ps, pb = (None, None) if pre is None else (pre[0].contiguous(), pre[1].contiguous())
        res = None if residual is None else residual.contiguous()
        if res is not None and tuple(res.shape) != (n_out, cout):
            raise ValueError("sparse_conv: residual must be [n_out, cout]")
        fws = workspace(_forward_ws_bytes(lib, n_out, n_in, K, cin, cout), dev)
        x_c, b_c = x.detach().contiguous(), None if b is None else b.detach().contiguous()
        _lib.call("o3dml_sparse_conv_forward_fused", ptr(_transposed_filters(f)), K, cin, cout,
                  ptr(x_c), n_in, ptr(ps), ptr(pb), ptr(res),
                  ptr(b_c), n_out, ptr(out), ptr(mws), mws.numel(),
                  ptr(fws), fws.numel(), stream_handle(dev))
        if scope is not None and scope.ahead:
            scope.pump()  # after this GEMM's launch: the next map build follows it in launch order
        return out if _late_ok(late) else None
    empty = torch.empty(0, dtype=torch.int64, device=dev)
    out = _ConvFn.apply(f, x, b, empty, empty, None, empty, _opt(inp_importance, dev), bool(normalize), oimp,
                        want_grad, (mws, n_out))
    if scope is not None and scope.ahead:
        scope.pump()
    if not _late_ok(late):
        return None
    return out if inp_features.is_cuda else out.cpu()


def _transpose_of_cached(scope, key, cache_key, ks, n_in, n_out, want_grad, dev):
    """The kernel map of a SparseConvTranspose whose SparseConv partner (same
    kernel size, voxel size and offset, input and output positions swapped —
    SparseConvUnet's DeConvolution after its Convolution) is already in the
    scope: derived from the partner's map (o3dml_sparse_conv_transpose_map:
    the same pairs at the same kernel indices) instead of a voxel hash and K
    lookups per output.  None when there is no such partner."""
    inp, out = cache_key[0], cache_key[1]
    conv_key = key[:1] + (False,) + key[2:5] + (-key[5],) + key[6:9] + (id(out), out._version, id(inp), inp._version)
    hit = scope.maps.get(conv_key)
    if hit is None or hit[1] & 4:
        return None
    lib = _lib.load()
    K = ks ** 3
    n_coarse, n_fine = n_in, n_out
    cmws = hit[0]
    mws = workspace(lib.o3dml_sparse_conv_map_workspace_size(n_fine, n_coarse, K), dev)
    _lib.call("o3dml_sparse_conv_transpose_map", ptr(cmws), cmws.numel(), n_coarse, n_fine, K, int(bool(want_grad)),
              ptr(mws), mws.numel(), stream_handle(dev))
    if K > 8:  # a scope map, as conv_lattice's own-built ones: GEMM tiles sorted by offset mask once
        _lib.call("o3dml_sparse_conv_tile_order", ptr(mws), mws.numel(), n_fine, n_coarse, K, int(bool(want_grad)),
                  stream_handle(dev))
    scope.derived += 1
    if scope.defer:
        off = lib.o3dml_sparse_conv_map_status_offset(n_fine, n_coarse, K)
        scope.pending.append(mws[off:off + 4].view(torch.int32))
    entry = (mws, hit[1], inp, out)
    scope.maps[key] = entry
    return entry


# (n_out, n_in, K, cin, cout) -> forward workspace bytes (one ctypes query per shape)
_FWS = SizeCache(lambda *key: int(_lib.load().o3dml_sparse_conv_forward_workspace_size(*key)))


def _forward_ws_bytes(lib, n_out, n_in, K, cin, cout):
    return _FWS(n_out, n_in, K, cin, cout)


def _late_ok(status):
    """Lattice status word read after the GEMM: True when the map was a
    lattice map (the result stands), False when the caller must recompute with
    the search rulebook; duplicate kernel indices raise."""
    if status is None:
        return True
    st = int(status.item())
    if st & 1:
        raise RuntimeError("sparse_conv: two neighbours of one output share a kernel index")
    return not st & 4


def _transposed_filters(f):
    """[k,k,k,Cin,Cout] -> contiguous [K, Cout, Cin] (what the GEMM reads),
    cached on the tensor until its data changes (eval weights: once)."""
    key = (f._version, f.data_ptr(), tuple(f.shape))
    hit = getattr(f, "_o3dml_wt", None)
    if hit is None or hit[0] != key:
        wt = f.detach().reshape(-1, f.shape[-2], f.shape[-1]).transpose(1, 2).contiguous()
        f._o3dml_wt = (key, wt)
        return wt
    return hit[1]


def kernel_index(inp_positions, query_positions, neighbors_index, neighbors_row_splits, kernel_size, voxel_size,
                 mirror=False):
    """Rulebook of layers.SparseConv: kernel index of every (query, input) pair."""
    dev = gpu_device(inp_positions, query_positions)
    ip = to_dev(inp_positions, dev, torch.float32)
    qp = to_dev(query_positions, dev, torch.float32)
    ni = to_dev(neighbors_index, dev, torch.int32)
    rs = to_dev(neighbors_row_splits, dev, torch.int64)
    ks = np.ascontiguousarray(np.asarray(kernel_size, np.int32).reshape(3))
    out = torch.empty(ni.shape[0], dtype=torch.int32, device=dev)
    _lib.call("o3dml_sparse_conv_kernel_index", ptr(ip), ptr(qp), ptr(ni), ptr(rs), qp.shape[0], ks.ctypes.data,
              float(voxel_size), int(bool(mirror)), ptr(out), stream_handle(dev))
    return out
