"""``torch.ops.open3d.*`` — the hot-path ops registered with the PyTorch
dispatcher (SURVEY.md §7 step 2, §8b "Mechanism upstream": Open3D ships a
TorchScript custom-op library under the ``open3d`` namespace, loaded with
``torch.ops.load_library``).

Each op is a ``torch.library.custom_op`` whose implementation is the
``o3dml_amd.ops`` function of the same name (HIP kernels through the C ABI),
so TorchScript and ``torch.compile`` callers see opaque ops with schemas;
ragged outputs get fake (meta) implementations with data-dependent sizes.
Autograd is registered for ``sparse_conv`` / ``sparse_conv_transpose``
(filter and feature gradients, the map rebuilt with its inverse — no forward
GEMM recomputed) and ``three_interpolate`` (its gradient op).  Importing this
module registers everything once; ``o3dml_amd`` imports it lazily through
``o3dml_amd.register_torch_ops()``."""
from typing import Optional

import torch
from torch import Tensor

from . import ops
from . import sparse_conv as sc

_NS = "open3d"


def _op(name):
    return torch.library.custom_op(f"{_NS}::{name}", mutates_args=())


def _dyn():
    return torch.library.get_ctx().new_dynamic_size()


def _idx_dtype(index_dtype):
    return torch.int64 if index_dtype in (torch.int64, 4) else torch.int32


# ----------------------------------------------------------------- searches
@_op("build_spatial_hash_table")
def build_spatial_hash_table(points: Tensor, radius: float, points_row_splits: Tensor,
                             hash_table_size_factor: float, max_hash_table_size: int = 33554432
                             ) -> tuple[Tensor, Tensor, Tensor]:
    r = ops.build_spatial_hash_table(points, radius, points_row_splits, hash_table_size_factor,
                                     max_hash_table_size)
    return r.hash_table_index, r.hash_table_cell_splits, r.hash_table_splits.clone()


@build_spatial_hash_table.register_fake
def _(points, radius, points_row_splits, hash_table_size_factor, max_hash_table_size=33554432):
    n_cells = _dyn()
    return (points.new_empty((points.shape[0],), dtype=torch.int32), points.new_empty((n_cells,), dtype=torch.int32),
            torch.empty((points_row_splits.shape[0],), dtype=torch.int32))


def _search_fake(points, queries, index_dtype, return_distances):
    p = _dyn()
    return (points.new_empty((p,), dtype=_idx_dtype(index_dtype)),
            points.new_empty((queries.shape[0] + 1,), dtype=torch.int64),
            points.new_empty((p if return_distances else 0,), dtype=torch.float32))


@_op("fixed_radius_search")
def fixed_radius_search(points: Tensor, queries: Tensor, radius: float, points_row_splits: Tensor,
                        queries_row_splits: Tensor, hash_table_splits: Tensor, hash_table_index: Tensor,
                        hash_table_cell_splits: Tensor, index_dtype: torch.dtype = torch.int32, metric: str = "L2",
                        ignore_query_point: bool = False, return_distances: bool = False
                        ) -> tuple[Tensor, Tensor, Tensor]:
    return tuple(ops.fixed_radius_search(points, queries, radius, points_row_splits, queries_row_splits,
                                         hash_table_splits, hash_table_index, hash_table_cell_splits, index_dtype,
                                         metric, ignore_query_point, return_distances))


@fixed_radius_search.register_fake
def _(points, queries, radius, points_row_splits, queries_row_splits, hash_table_splits, hash_table_index,
      hash_table_cell_splits, index_dtype=torch.int32, metric="L2", ignore_query_point=False,
      return_distances=False):
    return _search_fake(points, queries, index_dtype, return_distances)


@_op("knn_search")
def knn_search(points: Tensor, queries: Tensor, k: int, points_row_splits: Tensor, queries_row_splits: Tensor,
               index_dtype: torch.dtype = torch.int32, metric: str = "L2", ignore_query_point: bool = False,
               return_distances: bool = False) -> tuple[Tensor, Tensor, Tensor]:
    return tuple(ops.knn_search(points, queries, k, points_row_splits, queries_row_splits, index_dtype, metric,
                                ignore_query_point, return_distances))


@knn_search.register_fake
def _(points, queries, k, points_row_splits, queries_row_splits, index_dtype=torch.int32, metric="L2",
      ignore_query_point=False, return_distances=False):
    return _search_fake(points, queries, index_dtype, return_distances)


@_op("radius_search")
def radius_search(points: Tensor, queries: Tensor, radii: Tensor, points_row_splits: Tensor,
                  queries_row_splits: Tensor, index_dtype: torch.dtype = torch.int32, metric: str = "L2",
                  ignore_query_point: bool = False, return_distances: bool = False,
                  normalize_distances: bool = False) -> tuple[Tensor, Tensor, Tensor]:
    return tuple(ops.radius_search(points, queries, radii, points_row_splits, queries_row_splits, index_dtype,
                                   metric, ignore_query_point, return_distances, normalize_distances))


@radius_search.register_fake
def _(points, queries, radii, points_row_splits, queries_row_splits, index_dtype=torch.int32, metric="L2",
      ignore_query_point=False, return_distances=False, normalize_distances=False):
    return _search_fake(points, queries, index_dtype, return_distances)


# ----------------------------------------------------------------- ragged / voxels
@_op("ragged_to_dense")
def ragged_to_dense(values: Tensor, row_splits: Tensor, out_col_size: int, default_value: Tensor) -> Tensor:
    return ops.ragged_to_dense(values, row_splits, out_col_size, default_value)


@ragged_to_dense.register_fake
def _(values, row_splits, out_col_size, default_value):
    return values.new_empty((row_splits.shape[0] - 1, out_col_size) + tuple(values.shape[1:]))


@_op("reduce_subarrays_sum")
def reduce_subarrays_sum(values: Tensor, row_splits: Tensor) -> Tensor:
    return ops.reduce_subarrays_sum(values, row_splits)


@reduce_subarrays_sum.register_fake
def _(values, row_splits):
    return values.new_empty((row_splits.shape[0] - 1,))


@_op("voxelize")
def voxelize(points: Tensor, row_splits: Tensor, voxel_size: Tensor, points_range_min: Tensor,
             points_range_max: Tensor, max_points_per_voxel: int = 9223372036854775807,
             max_voxels: int = 9223372036854775807) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    return tuple(ops.voxelize(points, row_splits, voxel_size, points_range_min, points_range_max,
                              max_points_per_voxel, max_voxels))


@voxelize.register_fake
def _(points, row_splits, voxel_size, points_range_min, points_range_max, max_points_per_voxel=2**63 - 1,
      max_voxels=2**63 - 1):
    v, p = _dyn(), _dyn()
    return (points.new_empty((v, points.shape[1]), dtype=torch.int32), points.new_empty((p,), dtype=torch.int64),
            points.new_empty((v + 1,), dtype=torch.int64),
            points.new_empty((row_splits.shape[0],), dtype=torch.int64))


# ----------------------------------------------------------------- PointNet++ ops
@_op("furthest_point_sampling")
def furthest_point_sampling(points: Tensor, sample_size: int) -> Tensor:
    return ops.furthest_point_sampling(points, sample_size)


@furthest_point_sampling.register_fake
def _(points, sample_size):
    return points.new_empty((points.shape[0], sample_size), dtype=torch.int32)


@_op("ball_query")
def ball_query(xyz: Tensor, center: Tensor, radius: float, nsample: int) -> Tensor:
    return ops.ball_query(xyz, center, radius, nsample)


@ball_query.register_fake
def _(xyz, center, radius, nsample):
    return xyz.new_empty((center.shape[0], center.shape[1], nsample), dtype=torch.int32)


@_op("three_nn")
def three_nn(query_pts: Tensor, data_pts: Tensor) -> tuple[Tensor, Tensor]:
    return ops.three_nn(query_pts, data_pts)


@three_nn.register_fake
def _(query_pts, data_pts):
    s = (query_pts.shape[0], query_pts.shape[1], 3)
    return query_pts.new_empty(s), query_pts.new_empty(s, dtype=torch.int32)


@_op("three_interpolate_grad")
def three_interpolate_grad(grad_out: Tensor, idx: Tensor, weights: Tensor, M: int) -> Tensor:
    return ops.three_interpolate_grad(grad_out, idx, weights, M)


@three_interpolate_grad.register_fake
def _(grad_out, idx, weights, M):
    return grad_out.new_empty((grad_out.shape[0], grad_out.shape[1], M))


@_op("three_interpolate")
def three_interpolate(points: Tensor, idx: Tensor, weights: Tensor) -> Tensor:
    return ops.three_interpolate(points, idx, weights)


@three_interpolate.register_fake
def _(points, idx, weights):
    return points.new_empty((points.shape[0], points.shape[1], idx.shape[1]))


def _ti_setup(ctx, inputs, output):
    points, idx, weights = inputs
    ctx.save_for_backward(idx, weights)
    ctx.m = points.shape[2]


def _ti_backward(ctx, grad):
    idx, weights = ctx.saved_tensors
    return torch.ops.open3d.three_interpolate_grad(grad.contiguous(), idx, weights, ctx.m), None, None


three_interpolate.register_autograd(_ti_backward, setup_context=_ti_setup)


@_op("nms")
def nms(boxes: Tensor, scores: Tensor, nms_overlap_thresh: float) -> Tensor:
    return ops.nms(boxes, scores, nms_overlap_thresh)


@nms.register_fake
def _(boxes, scores, nms_overlap_thresh):
    return boxes.new_empty((_dyn(),), dtype=torch.int64)


# ----------------------------------------------------------------- sparse convolution
@_op("sparse_conv")
def sparse_conv(filters: Tensor, inp_features: Tensor, inp_importance: Optional[Tensor], neighbors_index: Tensor,
                neighbors_kernel_index: Tensor, neighbors_importance: Optional[Tensor],
                neighbors_row_splits: Tensor, normalize: bool = False, max_temp_mem_MB: int = 64) -> Tensor:
    with torch.no_grad():
        return sc.sparse_conv(filters, inp_features, inp_importance, neighbors_index, neighbors_kernel_index,
                              neighbors_importance, neighbors_row_splits, normalize, max_temp_mem_MB)


@sparse_conv.register_fake
def _(filters, inp_features, inp_importance, neighbors_index, neighbors_kernel_index, neighbors_importance,
      neighbors_row_splits, normalize=False, max_temp_mem_MB=64):
    return inp_features.new_empty((neighbors_row_splits.shape[0] - 1, filters.shape[-1]))


def _sc_setup(ctx, inputs, output):
    filters, x, inp_imp, nidx, kidx, nimp, rs, normalize, _ = inputs
    ctx.save_for_backward(filters, x, inp_imp, nidx, kidx, nimp, rs)
    ctx.normalize = normalize


def _sc_backward(ctx, grad):
    filters, x, inp_imp, nidx, kidx, nimp, rs = ctx.saved_tensors
    ss = None if inp_imp is None or inp_imp.numel() == 0 else inp_imp.to(x.device).float().contiguous()
    gw, gx = sc.conv_grads(filters, x, grad, nidx, kidx, nimp, rs, ss, ctx.normalize, None,
                           ctx.needs_input_grad[0], ctx.needs_input_grad[1])
    if gw is not None and not filters.is_cuda:
        gw = gw.cpu()
    if gx is not None and not x.is_cuda:
        gx = gx.cpu()
    return gw, gx, None, None, None, None, None, None, None


sparse_conv.register_autograd(_sc_backward, setup_context=_sc_setup)


@_op("sparse_conv_transpose")
def sparse_conv_transpose(filters: Tensor, out_importance: Optional[Tensor], inp_features: Tensor,
                          inp_neighbors_index: Tensor, inp_neighbors_importance_sum: Optional[Tensor],
                          inp_neighbors_row_splits: Tensor, neighbors_index: Tensor, neighbors_kernel_index: Tensor,
                          neighbors_importance: Optional[Tensor], neighbors_row_splits: Tensor,
                          normalize: bool = False, max_temp_mem_MB: int = 64) -> Tensor:
    with torch.no_grad():
        return sc.sparse_conv_transpose(filters, out_importance, inp_features, inp_neighbors_index,
                                        inp_neighbors_importance_sum, inp_neighbors_row_splits, neighbors_index,
                                        neighbors_kernel_index, neighbors_importance, neighbors_row_splits,
                                        normalize, max_temp_mem_MB)


@sparse_conv_transpose.register_fake
def _(filters, out_importance, inp_features, inp_neighbors_index, inp_neighbors_importance_sum,
      inp_neighbors_row_splits, neighbors_index, neighbors_kernel_index, neighbors_importance, neighbors_row_splits,
      normalize=False, max_temp_mem_MB=64):
    return inp_features.new_empty((neighbors_row_splits.shape[0] - 1, filters.shape[-1]))


def _sct_setup(ctx, inputs, output):
    (filters, out_imp, x, inp_nidx, inp_nimp_sum, inp_rs, nidx, kidx, nimp, rs, normalize, _) = inputs
    ctx.save_for_backward(filters, out_imp, x, inp_nimp_sum, inp_rs, nidx, kidx, nimp, rs)
    ctx.normalize = normalize


def _sct_backward(ctx, grad):
    filters, out_imp, x, inp_nimp_sum, inp_rs, nidx, kidx, nimp, rs = ctx.saved_tensors
    ss = sc.transpose_scale(x, filters, inp_nimp_sum, inp_rs, ctx.normalize, nimp)
    gw, gx = sc.conv_grads(filters, x, grad, nidx, kidx, nimp, rs, ss, False, out_imp,
                           ctx.needs_input_grad[0], ctx.needs_input_grad[2])
    if gw is not None and not filters.is_cuda:
        gw = gw.cpu()
    if gx is not None and not x.is_cuda:
        gx = gx.cpu()
    return gw, None, gx, None, None, None, None, None, None, None, None, None


sparse_conv_transpose.register_autograd(_sct_backward, setup_context=_sct_setup)

OPS = ("build_spatial_hash_table", "fixed_radius_search", "knn_search", "radius_search", "ragged_to_dense",
       "reduce_subarrays_sum", "voxelize", "furthest_point_sampling", "ball_query", "three_nn", "three_interpolate",
       "three_interpolate_grad", "nms", "sparse_conv", "sparse_conv_transpose")
