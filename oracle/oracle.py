"""numpy front-end of the C oracle (oracle/o3d_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (open3d-ml_amd/) never does.  Each function
restates one Open3D-ML hot-path op with the same argument
meaning as the op the reference calls; the C file's header documents the
semantics and the pinning status ("parity unpinned" against Open3D itself,
pinned against scipy/numpy exact oracles in tests/golden/).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# O3DML_ORACLE_LIB selects another build of the same source (the sanitizer
# build `make -C oracle asan`, tests/test_sanitizers.py)
_LIB_PATH = os.environ.get("O3DML_ORACLE_LIB", os.path.join(_HERE, "_build", "liboracle.so"))
_lib = None

METRICS = {"L1": 0, "L2": 1, "Linf": 2}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_hash_table_splits.restype = ctypes.c_int64
        _lib.orc_grid_subsample.restype = ctypes.c_int64
        _lib.orc_nms.restype = ctypes.c_int64
        _lib.orc_bev_iou.restype = ctypes.c_float
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _splits(rs, n):
    return _i64([0, n] if rs is None else rs)


def default_threads():
    return min(16, os.cpu_count() or 1)


# --------------------------------------------------------------------------
# spatial hash + fixed radius search  
# --------------------------------------------------------------------------
def build_spatial_hash_table(points, radius, points_row_splits=None,
                             hash_table_size_factor=1 / 64,
                             max_hash_table_size=33554432):
    points = _f32(points)
    prs = _splits(points_row_splits, len(points))
    B = len(prs) - 1
    splits = np.zeros(B + 1, np.uint32)
    T = lib().orc_hash_table_splits(ctypes.c_int64(B), _p(prs),
                                    ctypes.c_double(hash_table_size_factor),
                                    ctypes.c_int64(max_hash_table_size),
                                    _p(splits))
    index = np.zeros(len(points), np.uint32)
    cell_splits = np.zeros(T + 1, np.uint32)
    lib().orc_build_spatial_hash_table(_p(points), ctypes.c_int64(len(points)),
                                       ctypes.c_float(radius), ctypes.c_int64(B),
                                       _p(prs), _p(splits), _p(index),
                                       _p(cell_splits))
    return index, cell_splits, splits


def fixed_radius_search(points, queries, radius, points_row_splits=None,
                        queries_row_splits=None, hash_table=None,
                        metric="L2", ignore_query_point=False,
                        return_distances=False, index_dtype=np.int32,
                        hash_table_size_factor=1 / 64, nthreads=None):
    """Returns (neighbors_index, neighbors_row_splits, neighbors_distance)."""
    points, queries = _f32(points), _f32(queries)
    prs = _splits(points_row_splits, len(points))
    qrs = _splits(queries_row_splits, len(queries))
    if hash_table is None:
        hash_table = build_spatial_hash_table(points, radius, prs,
                                              hash_table_size_factor)
    index, cell_splits, splits = hash_table
    M = len(queries)
    rs = np.zeros(M + 1, np.int64)
    nt = default_threads() if nthreads is None else nthreads
    args = [_p(points), ctypes.c_int64(len(points)), _p(queries), ctypes.c_int64(M),
            ctypes.c_float(radius), ctypes.c_int64(len(prs) - 1), _p(prs), _p(qrs),
            _p(splits), _p(index), _p(cell_splits), ctypes.c_int(METRICS[metric]),
            ctypes.c_int(int(ignore_query_point)), _p(rs)]
    lib().orc_fixed_radius_search(*args, None, None, None, ctypes.c_int(nt), ctypes.c_int(0))
    P = int(rs[-1])
    idx = np.zeros(P, index_dtype)
    dist = np.zeros(P if return_distances else 0, np.float32)
    i32 = _p(idx) if idx.dtype == np.int32 else None
    i64 = _p(idx) if idx.dtype == np.int64 else None
    lib().orc_fixed_radius_search(*args, i32, i64, _p(dist) if return_distances else None,
                                  ctypes.c_int(nt), ctypes.c_int(1))
    return idx, rs, dist


def fixed_radius_search_fast(points, radius, points_row_splits=None, nthreads=None, capacity=None,
                             hash_table_size_factor=1 / 64, max_hash_table_size=33554432, simd=True):
    """cpu_frs.c: the optimised CPU self search (parallel hash build + one
    search pass, AVX2 + FMA candidate tests when the host has them and simd),
    L2, int32 — the bench's C1 CPU baseline.  Same result as
    fixed_radius_search(points, points, radius, rs, rs).  Returns (idx, rs)."""
    points = _f32(points)
    prs = _splits(points_row_splits, len(points))
    n = len(points)
    rs = np.zeros(n + 1, np.int64)
    nt = default_threads() if nthreads is None else nthreads
    cap = int(capacity) if capacity is not None else 48 * n
    f = lib().orc_frs_fast
    f.restype = ctypes.c_int64
    while True:
        idx = np.empty(cap, np.int32)
        total = f(_p(points), ctypes.c_int64(n), ctypes.c_float(radius), ctypes.c_int64(len(prs) - 1), _p(prs),
                  ctypes.c_double(hash_table_size_factor), ctypes.c_int64(max_hash_table_size), ctypes.c_int(nt),
                  ctypes.c_int(int(simd)), _p(rs), _p(idx), ctypes.c_int64(cap))
        if total <= cap:
            return idx[:total], rs
        cap = int(total)


def knn_search(points, queries, k, points_row_splits=None, queries_row_splits=None,
               metric="L2", ignore_query_point=False, return_distances=False,
               index_dtype=np.int32, nthreads=None):
    points, queries = _f32(points), _f32(queries)
    prs = _splits(points_row_splits, len(points))
    qrs = _splits(queries_row_splits, len(queries))
    M = len(queries)
    rs = np.zeros(M + 1, np.int64)
    nt = default_threads() if nthreads is None else nthreads
    args = [_p(points), ctypes.c_int64(len(points)), _p(queries), ctypes.c_int64(M),
            ctypes.c_int64(k), ctypes.c_int64(len(prs) - 1), _p(prs), _p(qrs),
            ctypes.c_int(METRICS[metric]), ctypes.c_int(int(ignore_query_point)), _p(rs)]
    lib().orc_knn_search(*args, None, None, None, ctypes.c_int(nt), ctypes.c_int(0))
    P = int(rs[-1])
    idx = np.zeros(P, index_dtype)
    dist = np.zeros(P if return_distances else 0, np.float32)
    lib().orc_knn_search(*args, _p(idx) if idx.dtype == np.int32 else None,
                         _p(idx) if idx.dtype == np.int64 else None,
                         _p(dist) if return_distances else None,
                         ctypes.c_int(nt), ctypes.c_int(1))
    return idx, rs, dist


def radius_search(points, queries, radii, points_row_splits=None,
                  queries_row_splits=None, metric="L2", ignore_query_point=False,
                  return_distances=False, normalize_distances=False,
                  index_dtype=np.int32, nthreads=None):
    points, queries, radii = _f32(points), _f32(queries), _f32(radii)
    prs = _splits(points_row_splits, len(points))
    qrs = _splits(queries_row_splits, len(queries))
    M = len(queries)
    rs = np.zeros(M + 1, np.int64)
    nt = default_threads() if nthreads is None else nthreads
    args = [_p(points), ctypes.c_int64(len(points)), _p(queries), ctypes.c_int64(M),
            _p(radii), ctypes.c_int64(len(prs) - 1), _p(prs), _p(qrs),
            ctypes.c_int(METRICS[metric]), ctypes.c_int(int(ignore_query_point)),
            ctypes.c_int(int(normalize_distances)), _p(rs)]
    lib().orc_radius_search(*args, None, None, None, ctypes.c_int(nt), ctypes.c_int(0))
    P = int(rs[-1])
    idx = np.zeros(P, index_dtype)
    dist = np.zeros(P if return_distances else 0, np.float32)
    lib().orc_radius_search(*args, _p(idx) if idx.dtype == np.int32 else None,
                            _p(idx) if idx.dtype == np.int64 else None,
                            _p(dist) if return_distances else None,
                            ctypes.c_int(nt), ctypes.c_int(1))
    return idx, rs, dist


# --------------------------------------------------------------------------
# ragged helpers (A6, A10)
# --------------------------------------------------------------------------
def ragged_to_dense(values, row_splits, out_col_size, default_value):
    values = np.asarray(values)
    row_splits = np.asarray(row_splits, np.int64)
    M = len(row_splits) - 1
    default_value = np.asarray(default_value, values.dtype)
    out = np.empty((M, out_col_size) + values.shape[1:], values.dtype)
    out[...] = default_value
    for r in range(M):
        s, e = row_splits[r], row_splits[r + 1]
        n = min(e - s, out_col_size)
        out[r, :n] = values[s:s + n]
    return out


def reduce_subarrays_sum(values, row_splits):
    values = _f32(values)
    rs = _i64(row_splits)
    out = np.zeros(len(rs) - 1, np.float32)
    lib().orc_reduce_subarrays_sum(_p(values), _p(rs), ctypes.c_int64(len(rs) - 1), _p(out))
    return out


# --------------------------------------------------------------------------
# voxelize (A9)
# --------------------------------------------------------------------------
def voxelize(points, row_splits, voxel_size, points_range_min, points_range_max,
             max_points_per_voxel=2**63 - 1, max_voxels=2**63 - 1):
    points = _f32(points)
    ndim = points.shape[1]
    rs = _i64(row_splits)
    vs, mn, mx = _f32(voxel_size), _f32(points_range_min), _f32(points_range_max)
    counts = np.zeros(2, np.int64)
    common = [_p(points), ctypes.c_int64(len(points)), ctypes.c_int(ndim),
              ctypes.c_int64(len(rs) - 1), _p(rs), _p(vs), _p(mn), _p(mx),
              ctypes.c_int64(max_points_per_voxel), ctypes.c_int64(max_voxels), _p(counts)]
    lib().orc_voxelize(*common, None, None, None, None, ctypes.c_int(0))
    V, P = int(counts[0]), int(counts[1])
    coords = np.zeros((V, ndim), np.int32)
    pidx = np.zeros(P, np.int64)
    prs = np.zeros(V + 1, np.int64)
    bs = np.zeros(len(rs), np.int64)
    lib().orc_voxelize(*common, _p(coords), _p(pidx), _p(prs), _p(bs), ctypes.c_int(1))
    return coords, pidx, prs, bs


# --------------------------------------------------------------------------
# grid subsampling (A7/A8)
# --------------------------------------------------------------------------
def _grid_one(points, feat, classes, dl, max_p=0):
    points = _f32(points)
    n = len(points)
    fdim = 0 if feat is None else feat.reshape(n, -1).shape[1]
    ldim = 0 if classes is None else classes.reshape(n, -1).shape[1]
    f = None if feat is None else _f32(feat.reshape(n, fdim))
    c = None if classes is None else np.ascontiguousarray(classes.reshape(n, ldim), np.int32)
    args = [_p(points), ctypes.c_int64(n), _p(f), ctypes.c_int64(fdim), _p(c),
            ctypes.c_int64(ldim), ctypes.c_float(dl), ctypes.c_int64(max_p)]
    S = lib().orc_grid_subsample(*args, None, None, None, ctypes.c_int(0))
    sp = np.zeros((S, 3), np.float32)
    sf = np.zeros((S, fdim), np.float32)
    sc = np.zeros((S, ldim), np.int32)
    lib().orc_grid_subsample(*args, _p(sp), _p(sf), _p(sc), ctypes.c_int(1))
    return sp, sf, sc


def subsample(points, features=None, classes=None, sampleDl=0.1, verbose=0):
    """contrib.subsample: returns points[, features][, classes] (dataprocessing.py:33-49)."""
    sp, sf, sc = _grid_one(points, features, classes, sampleDl)
    out = [sp]
    if features is not None:
        out.append(sf)
    if classes is not None:
        out.append(sc.reshape(-1) if np.asarray(classes).ndim == 1 else sc)
    return out[0] if len(out) == 1 else tuple(out)


def subsample_batch(points, batches, features=None, classes=None, sampleDl=0.1,
                    method="barycenters", max_p=0, verbose=0):
    """contrib.subsample_batch (kpconv.py:2099-2155): per batch element, first max_p cells."""
    points = _f32(points)
    batches = np.asarray(batches, np.int64)
    outs_p, outs_f, outs_c, lens = [], [], [], []
    s = 0
    for n in batches:
        f = None if features is None else np.asarray(features)[s:s + n]
        c = None if classes is None else np.asarray(classes)[s:s + n]
        sp, sf, sc = _grid_one(points[s:s + n], f, c, sampleDl, max_p)
        outs_p.append(sp); outs_f.append(sf); outs_c.append(sc); lens.append(len(sp))
        s += n
    out = [np.concatenate(outs_p, 0), np.asarray(lens, np.int32)]
    if features is not None:
        out.append(np.concatenate(outs_f, 0))
    if classes is not None:
        c = np.concatenate(outs_c, 0)
        out.append(c.reshape(-1) if np.asarray(classes).ndim == 1 else c)
    return tuple(out)


# --------------------------------------------------------------------------
# PointNet++ (A15-A17)
# --------------------------------------------------------------------------
def furthest_point_sampling(points, sample_size):
    points = _f32(points)
    B, N, _ = points.shape
    out = np.zeros((B, sample_size), np.int32)
    lib().orc_furthest_point_sampling(_p(points), ctypes.c_int64(B), ctypes.c_int64(N),
                                      ctypes.c_int64(sample_size), _p(out))
    return out


def ball_query(xyz, center, radius, nsample):
    xyz, center = _f32(xyz), _f32(center)
    B, N, _ = xyz.shape
    M = center.shape[1]
    out = np.zeros((B, M, nsample), np.int32)
    lib().orc_ball_query(_p(xyz), _p(center), ctypes.c_int64(B), ctypes.c_int64(N),
                         ctypes.c_int64(M), ctypes.c_float(radius), ctypes.c_int64(nsample),
                         _p(out))
    return out


def three_nn(query, data):
    query, data = _f32(query), _f32(data)
    B, n, _ = query.shape
    m = data.shape[1]
    d = np.zeros((B, n, 3), np.float32)
    i = np.zeros((B, n, 3), np.int32)
    lib().orc_three_nn(_p(query), _p(data), ctypes.c_int64(B), ctypes.c_int64(n),
                       ctypes.c_int64(m), _p(d), _p(i))
    return d, i


def three_interpolate(feats, idx, weights):
    feats = _f32(feats)
    idx = np.ascontiguousarray(idx, np.int32)
    weights = _f32(weights)
    B, C, m = feats.shape
    n = idx.shape[1]
    out = np.zeros((B, C, n), np.float32)
    lib().orc_three_interpolate(_p(feats), _p(idx), _p(weights), ctypes.c_int64(B),
                                ctypes.c_int64(C), ctypes.c_int64(m), ctypes.c_int64(n), _p(out))
    return out


def three_interpolate_grad(grad, idx, weights, M):
    grad = _f32(grad)
    idx = np.ascontiguousarray(idx, np.int32)
    weights = _f32(weights)
    B, C, n = grad.shape
    out = np.zeros((B, C, M), np.float32)
    lib().orc_three_interpolate_grad(_p(grad), _p(idx), _p(weights), ctypes.c_int64(B),
                                     ctypes.c_int64(C), ctypes.c_int64(n), ctypes.c_int64(M),
                                     _p(out))
    return out


# --------------------------------------------------------------------------
# sparse conv (A12-A14)
# --------------------------------------------------------------------------
def sparse_conv(filters, inp_features, neighbors_index, neighbors_kernel_index,
                neighbors_row_splits, inp_importance=None, neighbors_importance=None,
                normalize=False, nthreads=None):
    filters = _f32(filters)
    cin, cout = filters.shape[-2], filters.shape[-1]
    K = int(np.prod(filters.shape[:-2]))
    inp = _f32(inp_features)
    idx = np.ascontiguousarray(neighbors_index, np.int32)
    kidx = np.ascontiguousarray(neighbors_kernel_index, np.int32)
    rs = _i64(neighbors_row_splits)
    n_out = len(rs) - 1
    out = np.zeros((n_out, cout), np.float32)
    ii = None if inp_importance is None or len(inp_importance) == 0 else _f32(inp_importance)
    ni = None if neighbors_importance is None or len(neighbors_importance) == 0 else _f32(neighbors_importance)
    nt = default_threads() if nthreads is None else nthreads
    lib().orc_sparse_conv(_p(filters), ctypes.c_int64(K), ctypes.c_int64(cin),
                          ctypes.c_int64(cout), _p(inp), _p(ii), _p(idx), _p(kidx), _p(ni),
                          _p(rs), ctypes.c_int64(n_out), ctypes.c_int(int(normalize)), _p(out),
                          ctypes.c_int(nt))
    return out


def kernel_index(inp_positions, query_positions, neighbors_index, neighbors_row_splits,
                 kernel_size, voxel_size, mirror=False):
    inp = _f32(inp_positions)
    qp = _f32(query_positions)
    idx = np.ascontiguousarray(neighbors_index, np.int32)
    rs = _i64(neighbors_row_splits)
    ks = np.ascontiguousarray(kernel_size, np.int32)
    out = np.zeros(len(idx), np.int32)
    lib().orc_kernel_index(_p(inp), _p(qp), _p(idx), _p(rs), ctypes.c_int64(len(rs) - 1),
                           _p(ks), ctypes.c_float(voxel_size), ctypes.c_int(int(mirror)),
                           _p(out))
    return out


def calculate_grid(in_positions):
    """Literal numpy restatement of sparseconvnet.py:388-401: expand each
    trunc(pos) by the 8 offsets {-1,0}^3, keep non-negative all-even rows,
    lexicographic unique, + 0.5."""
    p = np.trunc(np.asarray(in_positions, np.float32)).astype(np.int64)
    offs = np.array([[-1, -1, -1], [-1, -1, 0], [-1, 0, -1], [-1, 0, 0],
                     [0, -1, -1], [0, -1, 0], [0, 0, -1], [0, 0, 0]], np.int64)
    out = (p[:, None, :] + offs[None]).reshape(-1, 3)
    out = out[out.min(1) >= 0]
    out = out[~(out % 2).astype(bool).any(1)]
    out = np.unique(out, axis=0)
    return (out + 0.5).astype(np.float32)


def bev_iou(a, b):
    """Rotated BEV IoU of two (x1,y1,x2,y2,yaw) boxes (o3d_oracle.c orc_bev_iou)."""
    a, b = _f32(a), _f32(b)
    return float(lib().orc_bev_iou(_p(a), _p(b)))


def nms(boxes, scores, thresh):
    """open3d.ml.torch.ops.nms (objdet_helper.py:27,346): kept original indices, int64,
    in stable descending score order (o3d_oracle.c orc_nms)."""
    boxes, scores = _f32(boxes).reshape(-1, 5), _f32(scores).reshape(-1)
    n = scores.shape[0]
    keep = np.zeros(max(n, 1), np.int64)
    cnt = lib().orc_nms(_p(boxes), _p(scores), ctypes.c_int64(n), ctypes.c_float(thresh), _p(keep))
    return keep[:cnt].copy()
