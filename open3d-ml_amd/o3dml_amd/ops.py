"""Drop-in for ``open3d.ml.torch.ops`` on the point-cloud hot path.

Every function keeps the Open3D signature, argument meaning, output dtypes and
namedtuple field names the reference models bind to, and runs
on the HIP kernels of libo3dml_amd.so.  Inputs may live on the CPU (the
reference calls some ops from DataLoader workers on CPU tensors); they are then
staged to the GPU and the results returned on the CPU.  There is no CPU
compute path.
"""
from collections import namedtuple

import numpy as np
import torch

from . import _lib
from ._util import (back_to, check_points, gpu_device, index_bits, metric_code, ptr,
                    row_splits_host, scalar, stream_handle, to_dev, workspace)

BuildSpatialHashTableResult = namedtuple(
    "build_spatial_hash_table", ["hash_table_index", "hash_table_cell_splits", "hash_table_splits"])
FixedRadiusSearchResult = namedtuple(
    "fixed_radius_search", ["neighbors_index", "neighbors_row_splits", "neighbors_distance"])
KnnSearchResult = namedtuple("knn_search", ["neighbors_index", "neighbors_row_splits", "neighbors_distance"])
RadiusSearchResult = namedtuple("radius_search", ["neighbors_index", "neighbors_row_splits", "neighbors_distance"])


# ---------------------------------------------------------------------------
# spatial hash table + fixed radius search  
# ---------------------------------------------------------------------------
def build_spatial_hash_table(points, radius, points_row_splits=None, hash_table_size_factor=1 / 64,
                             max_hash_table_size=33554432):
    """Open3D ``ops.build_spatial_hash_table`` (used by layers.FixedRadiusSearch;
    reference caller kpconv.py:2021-2023).  Cell size 2*radius; bins sized
    ``min(max(factor*N_b, 1), max_hash_table_size)`` per batch item.
    Returns (hash_table_index int32 [N], hash_table_cell_splits int32 [T+1],
    hash_table_splits int32 [B+1] on the CPU)."""
    dev = gpu_device(points)
    check_points("points", points)
    lib = _lib.load()
    n = points.shape[0]
    r = scalar(radius)
    if not r > 0:
        raise RuntimeError("radius must be > 0")
    prs = row_splits_host(points_row_splits, n)
    B = len(prs) - 1
    splits = np.zeros(B + 1, np.uint32)
    T = lib.o3dml_hash_table_splits(B, prs.ctypes.data, float(hash_table_size_factor),
                                    int(max_hash_table_size), splits.ctypes.data)
    pts = to_dev(points, dev)
    prs_d = torch.from_numpy(prs).to(dev)
    hts_d = torch.from_numpy(splits.view(np.int32)).to(dev)
    index = torch.empty(n, dtype=torch.int32, device=dev)
    cells = torch.empty(T + 1, dtype=torch.int32, device=dev)
    ws = workspace(lib.o3dml_build_spatial_hash_table_workspace_size(n, T), dev)
    _lib.call("o3dml_build_spatial_hash_table", ptr(pts), n, r, B, ptr(prs_d), ptr(hts_d), T, ptr(index),
              ptr(cells), ptr(ws), ws.numel(), stream_handle(dev))
    return BuildSpatialHashTableResult(back_to(index, points), back_to(cells, points),
                                       torch.from_numpy(splits.astype(np.int32)))


def _same_cloud(points, queries, prs, qrs):
    return (points.data_ptr() == queries.data_ptr() and points.shape == queries.shape
            and np.array_equal(prs, qrs))


def fixed_radius_search(points, queries, radius, points_row_splits=None, queries_row_splits=None,
                        hash_table_splits=None, hash_table_index=None, hash_table_cell_splits=None,
                        index_dtype=torch.int32, metric="L2", ignore_query_point=False,
                        return_distances=False):
    """Open3D ``ops.fixed_radius_search``: for every query all
    points with dist <= radius (L2: squared distance <= r^2; L1; Linf), in the
    query's batch item.  Neighbour order: hash bins ascending, point id
    ascending inside a bin (the canonical order).  Distances are
    squared for L2.  Returns (neighbors_index [P], neighbors_row_splits int64
    [M+1], neighbors_distance [P] or [0])."""
    dev = gpu_device(points, queries)
    check_points("points", points)
    check_points("queries", queries)
    bits = index_bits(index_dtype)
    mcode = metric_code(metric)
    lib = _lib.load()
    n, m = points.shape[0], queries.shape[0]
    r = scalar(radius)
    if not r > 0:
        raise RuntimeError("radius must be > 0")
    prs = row_splits_host(points_row_splits, n)
    qrs = row_splits_host(queries_row_splits, m)
    if len(prs) != len(qrs):
        raise RuntimeError("points_row_splits and queries_row_splits must have the same length")
    if hash_table_index is None:
        ht = build_spatial_hash_table(points, r, prs)
        hash_table_splits, hash_table_index, hash_table_cell_splits = (
            ht.hash_table_splits, ht.hash_table_index, ht.hash_table_cell_splits)
    same = _same_cloud(points, queries, prs, qrs)
    pts = to_dev(points, dev)
    qry = pts if same else to_dev(queries, dev)
    prs_d = torch.from_numpy(prs).to(dev)
    qrs_d = prs_d if same else torch.from_numpy(qrs).to(dev)
    hts_d = to_dev(hash_table_splits, dev, torch.int32)
    hti_d = to_dev(hash_table_index, dev, torch.int32)
    hcs_d = to_dev(hash_table_cell_splits, dev, torch.int32)
    order = hti_d if same else None
    B = len(prs) - 1
    st = stream_handle(dev)
    rs = torch.empty(m + 1, dtype=torch.int64, device=dev)
    ws = workspace(lib.o3dml_fixed_radius_search_workspace_size(n, m), dev)
    common = (ptr(pts), n, ptr(qry), m, r, B, ptr(prs_d), ptr(qrs_d), ptr(hts_d), ptr(hti_d), ptr(hcs_d),
              ptr(order), mcode, int(bool(ignore_query_point)))
    _lib.call("o3dml_fixed_radius_search_count", *common, ptr(rs), ptr(ws), ws.numel(), st)
    total = int(rs[-1].item())
    idx = torch.empty(total, dtype=torch.int32 if bits == 32 else torch.int64, device=dev)
    dist = torch.empty(total if return_distances else 0, dtype=torch.float32, device=dev)
    _lib.call("o3dml_fixed_radius_search_fill", *common, ptr(rs), bits, ptr(idx),
              ptr(dist) if return_distances else None, ptr(ws), ws.numel(), st)
    return FixedRadiusSearchResult(back_to(idx, points), back_to(rs, points), back_to(dist, points))


# ---------------------------------------------------------------------------
# ragged helpers
# ---------------------------------------------------------------------------
def ragged_to_dense(values, row_splits, out_col_size, default_value):
    """Open3D ``ops.ragged_to_dense``: rows of a ragged tensor into
    [M, out_col_size, ...], truncated / padded with default_value
    (kpconv.py:2030-2032, point_pillars.py:364-366)."""
    dev = gpu_device(values, row_splits)
    vals = to_dev(values, dev)
    rs = to_dev(row_splits, dev, torch.int64)
    inner_shape = tuple(vals.shape[1:])
    inner = int(np.prod(inner_shape)) if inner_shape else 1
    dflt = to_dev(torch.as_tensor(default_value), dev, vals.dtype)
    if dflt.numel() == 1 and inner != 1:
        dflt = dflt.reshape(1).expand(inner).contiguous()
    if dflt.numel() != inner:
        raise RuntimeError(f"default_value must have shape {list(inner_shape)}, got {list(dflt.shape)}")
    M = rs.shape[0] - 1
    out_col_size = int(out_col_size)
    out = torch.empty((M, out_col_size) + inner_shape, dtype=vals.dtype, device=dev)
    _lib.call("o3dml_ragged_to_dense", ptr(vals), ptr(rs), M, out_col_size, inner, vals.element_size(), ptr(dflt), ptr(out),
              stream_handle(dev))
    return back_to(out, values)


def reduce_subarrays_sum(values, row_splits):
    """Open3D ``ops.reduce_subarrays_sum``: per-row sums (fp32, left to right;
    empty rows give 0) — sparseconvnet.py:319-324."""
    dev = gpu_device(values, row_splits)
    if values.dtype != torch.float32:
        raise RuntimeError(f"reduce_subarrays_sum: values must be float32, got {values.dtype}")
    vals = to_dev(values, dev)
    rs = to_dev(row_splits, dev, torch.int64)
    M = rs.shape[0] - 1
    out = torch.empty(M, dtype=torch.float32, device=dev)
    _lib.call("o3dml_reduce_subarrays_sum", ptr(vals), ptr(rs), M, ptr(out), stream_handle(dev))
    return back_to(out, values)
