"""ctypes binding of libo3dml_amd.so (the C ABI declared in include/o3dml_amd.h).

The library is built in-tree by ``make -C open3d-ml_amd/csrc`` (or
``__graft_entry__.build()``).  There is deliberately NO fallback: if the
shared library or a ROCm GPU is missing, every op raises ``RuntimeError``.
torch is imported first so that the HIP runtime torch ships is the one the
library binds to (both carry the soname libamdhip64.so.7), which makes torch's
streams and allocations valid handles inside the library.
"""
import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "O3DML_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libo3dml_amd.so"))

_lib = None

c_i64, c_i32, c_u64, c_f32, c_f64, c_p, c_sz = (
    ctypes.c_int64, ctypes.c_int, ctypes.c_uint64, ctypes.c_float,
    ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t)

# name -> (restype, [argtypes]); must match include/o3dml_amd.h
SIGNATURES = {
    "o3dml_last_error": (ctypes.c_char_p, []),
    "o3dml_version": (c_i32, []),
    "o3dml_device_info": (c_i32, [c_i32, c_p, c_p, c_p]),
    "o3dml_timing_enable": (None, [c_i32]),
    "o3dml_timing_reset": (None, []),
    "o3dml_timing_get": (c_i32, [ctypes.c_char_p, c_p, c_p]),
    # nns_hash.hip
    "o3dml_hash_table_splits": (c_i64, [c_i64, c_p, c_f64, c_i64, c_p]),
    "o3dml_build_spatial_hash_table_workspace_size": (c_sz, [c_i64, c_i64]),
    "o3dml_build_spatial_hash_table": (c_i32, [c_p, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_i64, c_p, c_p,
                                               c_p, c_sz, c_p]),
    "o3dml_fixed_radius_search_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "o3dml_fixed_radius_search_count": (c_i32, [c_p, c_i64, c_p, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_p,
                                                c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_sz, c_p]),
    "o3dml_fixed_radius_search_fill": (c_i32, [c_p, c_i64, c_p, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_p,
                                               c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_p, c_i32, c_p, c_p,
                                               c_p, c_sz, c_p]),
    "o3dml_fixed_radius_search_totals": (c_i32, [c_p, c_i64, c_p, c_p, c_p]),
    "o3dml_fixed_radius_search_sizes": (c_i32, [c_p, c_i64, c_p, c_p, c_p]),
    "o3dml_fixed_radius_search_fill_bounded": (c_i32, [c_p, c_i64, c_p, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_p,
                                                       c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_p, c_i32, c_p, c_p,
                                                       c_i64, c_i32, c_p, c_sz, c_p]),
    "o3dml_fixed_radius_search_layer_workspace_size": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "o3dml_fixed_radius_search_layer": (c_i32, [c_p, c_i64, c_p, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_p, c_p,
                                                c_i64, c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_p,
                                                c_i32, c_p, c_p, c_i64, c_i32, c_p, c_p, c_sz, c_p]),
    "o3dml_fixed_radius_search_fill_dense": (c_i32, [c_p, c_i64, c_i64, c_f32, c_i64, c_p, c_p, c_p, c_p, c_p,
                                                     c_i32, c_i32, c_p, c_i64, c_i32, c_p, c_i32, c_p, c_sz, c_p]),
    # nns_knn.hip
    "o3dml_knn_search_workspace_size": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "o3dml_knn_search_count": (c_i32, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i32, c_i32,
                                       c_i32, c_p, c_p, c_sz, c_p]),
    "o3dml_knn_search_fill": (c_i32, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_i32, c_i32, c_p,
                                      c_i32, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_knn_select_workspace_size": (c_sz, [c_i64]),
    "o3dml_knn_select": (c_i32, [c_p, c_i64, c_p, c_i64, c_i32, c_p, c_p, c_sz, c_p]),
    # nns_many.hip
    "o3dml_radius_search_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "o3dml_radius_search_count": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i32, c_i32, c_p, c_p,
                                          c_sz, c_p]),
    "o3dml_radius_search_totals": (c_i32, [c_p, c_i64, c_p, c_p, c_p]),
    "o3dml_radius_search_fill": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_i32, c_p, c_i64,
                                         c_i32, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_radius_search_sort_long_rows": (c_i32, [c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_p, c_p, c_sz, c_p]),
    # voxel.hip
    "o3dml_voxelize_workspace_size": (c_sz, [c_i64, c_i64]),
    "o3dml_voxelize_count": (c_i32, [c_p, c_i64, c_i32, c_i64, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_sz,
                                     c_p]),
    "o3dml_voxelize_fill": (c_i32, [c_i64, c_i32, c_i64, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_lattice_workspace_size": (c_sz, [c_i64]),
    "o3dml_sparse_conv_lattice_map": (c_i32, [c_p, c_i64, c_p, c_i64, c_f32, c_i32, c_i32, c_i32, c_p, c_i32, c_i32,
                                              c_p, c_p, c_sz, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_lattice_map_shifted": (c_i32, [c_p, c_i64, c_p, c_p, c_i64, c_f32, c_i32, c_i32, c_i32, c_p,
                                                      c_i32, c_i32, c_p, c_p, c_sz, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_map_status_offset": (c_sz, [c_i64, c_i64, c_i32]),
    "o3dml_sparse_conv_tile_order": (c_i32, [c_p, c_sz, c_i64, c_i64, c_i32, c_i32, c_p]),
    "o3dml_sparse_conv_transpose_map": (c_i32, [c_p, c_sz, c_i64, c_i64, c_i32, c_i32, c_p, c_sz, c_p]),
    "o3dml_kpconv_weighted_features": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_i32,
                                               c_i32, c_f32, c_i32, c_i32, c_p, c_p, c_p]),
    "o3dml_kpconv_weighted_features_backward": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p,
                                                        c_i32, c_i32, c_f32, c_i32, c_i32, c_p, c_p]),
    "o3dml_kpconv_inverse_workspace_size": (c_sz, [c_i64, c_i32, c_i64]),
    "o3dml_kpconv_weighted_features_backward_det": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32,
                                                            c_p, c_i32, c_i32, c_f32, c_i32, c_i32, c_p, c_p, c_sz,
                                                            c_p]),
    "o3dml_kpconv_kernel_point_grad": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_p,
                                               c_i32, c_f32, c_i32, c_i32, c_p, c_p, c_p, c_p]),
    "o3dml_kpconv_min_d2_columns": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_p]),
    "o3dml_sgemm": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_p, c_i64, c_f32, c_p, c_i64, c_p]),
    "o3dml_sgemm_splitk_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "o3dml_sgemm_splitk": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_sz,
                                   c_p]),
    "o3dml_linear_bn_workspace_size": (c_sz, [c_i64, c_i32, c_i32]),
    "o3dml_linear_bn_forward": (c_i32, [c_p, c_i64, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_f32, c_f32, c_i32,
                                        c_i32, c_f32, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_linear_bn_backward": (c_i32, [c_p, c_p, c_i64, c_i32, c_p, c_i32, c_p, c_p, c_i32, c_i32, c_f32, c_p, c_p,
                                         c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_kpconv_rigid_workspace_size": (c_sz, [c_i64, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32]),
    "o3dml_kpconv_rigid_forward": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_i32, c_f32,
                                           c_i32, c_i32, c_p, c_i32, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_kpconv_rigid_backward": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i32, c_p, c_i32, c_f32,
                                            c_i32, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_i32, c_p, c_sz, c_p]),
    "o3dml_batch_norm_workspace_size": (c_sz, [c_i64, c_i32]),
    "o3dml_batch_norm_forward": (c_i32, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_f32, c_f32, c_i32, c_i32, c_f32,
                                         c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_batch_norm_backward": (c_i32, [c_p, c_p, c_i64, c_i32, c_p, c_i32, c_i32, c_f32, c_p, c_p, c_p, c_p, c_sz,
                                          c_p]),
    "o3dml_kpconv_pool_max": (c_i32, [c_p, c_i64, c_i32, c_p, c_i32, c_i64, c_i64, c_i32, c_p, c_p, c_p]),
    "o3dml_kpconv_pool_max_backward": (c_i32, [c_p, c_p, c_i64, c_i32, c_i64, c_p, c_p]),
    "o3dml_kpconv_pool_max_backward_det": (c_i32, [c_p, c_p, c_p, c_i32, c_i64, c_i64, c_i32, c_i32, c_i64, c_p, c_p,
                                                   c_sz, c_p]),
    "o3dml_pillar_features": (c_i32, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_i64, c_i32, c_f32, c_f32, c_f32, c_f32,
                                      c_p, c_p]),
    "o3dml_pillar_scatter": (c_i32, [c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p]),
    "o3dml_pillar_gather": (c_i32, [c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p]),
    "o3dml_randla_relative_encoding": (c_i32, [c_p, c_i64, c_p, c_i32, c_p, c_p]),
    "o3dml_randla_attentive_pool": (c_i32, [c_p, c_p, c_i64, c_i32, c_i32, c_p, c_p]),
    "o3dml_concat_rows": (c_i32, [c_p, c_i32, c_p, c_i32, c_p, c_i32, c_p, c_i32, c_i64, c_p, c_p]),
    "o3dml_randla_att_pool": (c_i32, [c_p, c_p, c_p, c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "o3dml_randla_gather_max": (c_i32, [c_p, c_i32, c_p, c_i64, c_i32, c_p, c_p]),
    # randla_sampler.hip
    "o3dml_randla_possibility_min": (c_i32, [c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_randla_possibility_min_workspace_size": (c_sz, []),
    "o3dml_random_permute": (c_i32, [c_p, c_i64, c_u64, c_p, c_p]),
    "o3dml_random_permute_dev": (c_i32, [c_p, c_i64, c_p, c_p, c_p]),
    "o3dml_randla_update_probs": (c_i32, [c_p, c_p, c_p, c_i64, c_i32, c_f64, c_i32, c_p, c_p]),
    "o3dml_randla_patch_workspace_size": (c_sz, [c_i64]),
    "o3dml_randla_patch_update": (c_i32, [c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_randla_up_from_knn": (c_i32, [c_p, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_randla_up_workspace_size": (c_sz, [c_i64]),
    # dense.hip
    "o3dml_dense_act_workspace_size": (c_sz, [c_i64, c_i32, c_i32]),
    "o3dml_dense_act": (c_i32, [c_p, c_i32, c_p, c_i32, c_p, c_p, c_p, c_i64, c_i32, c_i32, c_f32, c_p, c_p, c_sz,
                                c_p]),
    "o3dml_calculate_grid_workspace_size": (c_sz, [c_i64]),
    "o3dml_calculate_grid_count": (c_i32, [c_p, c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_calculate_grid_fill": (c_i32, [c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_scn_plan_workspace_size": (c_sz, [c_i64]),
    "o3dml_scn_plan": (c_i32, [c_p, c_p, c_i64, c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "o3dml_grid_subsample_workspace_size": (c_sz, [c_i64, c_i64]),
    "o3dml_grid_subsample_count": (c_i32, [c_p, c_i64, c_i64, c_p, c_p, c_f32, c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_grid_subsample_count_async": (c_i32, [c_p, c_i64, c_i64, c_p, c_f32, c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_rotate_batched": (c_i32, [c_p, c_i64, c_i64, c_p, c_p, c_i32, c_p, c_p]),
    "o3dml_grid_subsample_fill": (c_i32, [c_p, c_i64, c_i64, c_p, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_sz,
                                          c_p]),
    # pointnet2.hip
    "o3dml_furthest_point_sampling_workspace_size": (c_sz, [c_i64, c_i64]),
    "o3dml_furthest_point_sampling": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_ball_query": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_f32, c_i64, c_p, c_p]),
    "o3dml_three_nn": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "o3dml_three_interpolate": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "o3dml_three_interpolate_grad": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "o3dml_three_interpolate_grad_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "o3dml_three_interpolate_grad_det": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_sz, c_p]),
    "o3dml_nms_workspace_size": (c_sz, [c_i64]),
    "o3dml_nms": (c_i32, [c_p, c_p, c_i64, c_f32, c_p, c_p, c_p, c_sz, c_p]),
    # sparse_conv.hip
    "o3dml_sparse_conv_map_workspace_size": (c_sz, [c_i64, c_i64, c_i32]),
    "o3dml_sparse_conv_build_map": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i32, c_i32, c_p, c_i32, c_p, c_p,
                                            c_sz, c_p]),
    "o3dml_sparse_conv_forward_workspace_size": (c_sz, [c_i64, c_i64, c_i32, c_i32, c_i32]),
    "o3dml_sparse_conv_set_presplit": (c_i32, [c_i32]),
    "o3dml_sparse_conv_set_bsplit": (c_i32, [c_i32]),
    "o3dml_sparse_conv_forward_fused": (c_i32, [c_p, c_i32, c_i32, c_i32, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                                c_p, c_p, c_sz, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_forward": (c_i32, [c_p, c_i32, c_i32, c_i32, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i64, c_p,
                                          c_p, c_sz, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_backward_workspace_size": (c_sz, [c_i64, c_i64, c_i32, c_i32, c_i32]),
    "o3dml_sparse_conv_backward": (c_i32, [c_p, c_i32, c_i32, c_i32, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_i64, c_p,
                                           c_p, c_p, c_sz, c_p, c_sz, c_p]),
    "o3dml_sparse_conv_set_exact": (c_i32, [c_i32]),
    "o3dml_sparse_conv_kernel_index": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_p, c_f32, c_i32, c_p, c_p]),
    # ragged.hip
    "o3dml_ragged_to_dense": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p, c_p, c_p]),
    "o3dml_reduce_subarrays_sum": (c_i32, [c_p, c_p, c_i64, c_p, c_p]),
    "o3dml_sort_pairs_workspace_size": (c_sz, [c_i64, c_i32]),
    "o3dml_sort_pairs": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_sz, c_p]),
}


def load():
    """Load the library (idempotent).  Raises RuntimeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"o3dml_amd: HIP library not found at {LIB_PATH}; build it with "
            "`make -C open3d-ml_amd/csrc` (or __graft_entry__.build()).")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def kernel_times(names):
    """{name: (total_ms, launches)} recorded since the last o3dml_timing_reset."""
    import numpy as np
    lib = load()
    out = {}
    for n in names:
        ms = np.zeros(1, np.float64)
        cnt = np.zeros(1, np.int64)
        lib.o3dml_timing_get(n.encode(), ms.ctypes.data, cnt.ctypes.data)
        out[n] = (float(ms[0]), int(cnt[0]))
    return out


def exported_symbols():
    return list(SIGNATURES)


def check(status, what):
    if status != 0:
        msg = load().o3dml_last_error().decode(errors="replace")
        raise RuntimeError(f"o3dml_amd.{what} failed: {msg}")


def _stream_device(args):
    """Device of the StreamHandle among args (the stream is usually last)."""
    from ._util import StreamHandle
    if args and isinstance(args[-1], StreamHandle):
        return args[-1].dev
    for a in args:
        if isinstance(a, StreamHandle):
            return a.dev
    return None


def call(name, *args):
    """Call a status-returning entry point and raise on failure.  A call given
    a stream of a device other than the current one runs under a restoring
    device guard (the caller's current device is unchanged afterwards)."""
    if name not in SIGNATURES:  # ctypes would pass untyped ints as 32-bit: pointers truncated
        raise RuntimeError(f"o3dml_amd: no ctypes signature for {name} (add it to _lib.SIGNATURES)")
    fn = getattr(load(), name)
    dev = _stream_device(args)
    if dev is not None and dev != torch.cuda.current_device():
        with torch.cuda.device(dev):
            rc = fn(*args)
    else:
        rc = fn(*args)
    check(rc, name)
