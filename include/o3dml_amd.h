/*
 * o3dml_amd.h — C ABI of libo3dml_amd.so, the MI355X-native (gfx950 HIP)
 * implementation of Open3D-ML's point-cloud hot path.
 *
 * Every entry point replaces one Open3D op the reference binds to (Open3D
 * itself is un-vendored; the citations are the reference CALL SITES that bind
 * the op).  Conventions:
 *   - all tensor arguments are DEVICE pointers unless the name ends in _host;
 *   - sizes are int64; row splits are int64 prefix sums [B+1] (Open3D's);
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream);
 *   - variable-size outputs are two-phase: *_count writes row splits on the
 *     device, the caller reads the total, allocates, then calls *_fill;
 *   - temporary memory comes from a caller-provided `workspace` of at least
 *     *_workspace_size(...) bytes (no allocation inside a launch function, so
 *     every call is capturable in a hipGraph); a *_count/_fill pair must be
 *     given the same, unmodified workspace;
 *   - status: 0 = success, nonzero = error; o3dml_last_error() has the text.
 *     The Python layer turns nonzero into RuntimeError (Open3D's TORCH_CHECK).
 */
#ifndef O3DML_AMD_H
#define O3DML_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ----------------------------------------------------------- */
const char* o3dml_last_error(void);
int o3dml_version(void);
int o3dml_device_info(int device, int* cu_count, int* arch_major, int* arch_minor);

/* ---- spatial hash table: replaces open3d.ml.torch.ops.build_spatial_hash_table
 * (bound by layers.FixedRadiusSearch; ml3d/torch/models/kpconv.py:2021-2023,
 *  sparseconvnet.py:362-367 via layers.SparseConv).  Metric-independent. ---- */
/* Host helper: per-batch table sizes min(max(trunc(factor*N_b),1),max) and
 * their prefix sums into hash_table_splits_host[B+1]; returns the total. */
int64_t o3dml_hash_table_splits(int64_t n_batch, const int64_t* points_row_splits_host,
                                double hash_table_size_factor, int64_t max_hash_table_size,
                                uint32_t* hash_table_splits_host);
size_t o3dml_build_spatial_hash_table_workspace_size(int64_t n_points, int64_t total_bins);
/* points f32[N,3]; hash_table_splits u32[B+1] (device copy of the host
 * helper's output) -> hash_table_index u32[N] (point ids by bin, ascending id
 * inside a bin), hash_table_cell_splits u32[T+1]. */
int o3dml_build_spatial_hash_table(const float* points, int64_t n_points, float radius, int64_t n_batch,
                                   const int64_t* points_row_splits, const uint32_t* hash_table_splits,
                                   int64_t total_bins, uint32_t* hash_table_index,
                                   uint32_t* hash_table_cell_splits, void* workspace, size_t workspace_bytes,
                                   void* stream);

/* ---- fixed radius search: replaces open3d.ml.torch.ops.fixed_radius_search
 * (layers.FixedRadiusSearch; kpconv.py:2016-2034 batch_neighbors, called from
 * ml3d/torch/dataloaders/concat_batcher.py:228,257,261).
 * metric: 0 = L1, 1 = L2, 2 = Linf.  query_order (nullable): thread t handles
 * query query_order[t] (pass hash_table_index for a self search). ------------ */
size_t o3dml_fixed_radius_search_workspace_size(int64_t n_points, int64_t n_queries);
int o3dml_fixed_radius_search_count(const float* points, int64_t n_points, const float* queries,
                                    int64_t n_queries, float radius, int64_t n_batch,
                                    const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                    const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                    const uint32_t* hash_table_cell_splits, const uint32_t* query_order,
                                    int metric, int ignore_query_point, int64_t* neighbors_row_splits,
                                    void* workspace, size_t workspace_bytes, void* stream);
/* index_bits 32 or 64 (index_dtype); neighbors_distance nullable (squared for L2). */
int o3dml_fixed_radius_search_fill(const float* points, int64_t n_points, const float* queries,
                                   int64_t n_queries, float radius, int64_t n_batch,
                                   const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                   const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                   const uint32_t* hash_table_cell_splits, const uint32_t* query_order,
                                   int metric, int ignore_query_point, const int64_t* neighbors_row_splits,
                                   int index_bits, void* neighbors_index, float* neighbors_distance,
                                   void* workspace, size_t workspace_bytes, void* stream);

/* ---- ragged helpers ------------------------------------------------------
 * o3dml_ragged_to_dense replaces open3d.ml.torch.ops.ragged_to_dense
 * (kpconv.py:2030-2032, point_pillars.py:364-366): values [P, inner] of
 * elem_bytes each -> out [M, out_col_size, inner].
 * o3dml_reduce_subarrays_sum replaces ops.reduce_subarrays_sum
 * (sparseconvnet.py:319-324): f32 left-to-right per-row sums. */
int o3dml_ragged_to_dense(const void* values, const int64_t* row_splits, int64_t n_rows, int64_t out_col_size,
                          int64_t inner, int elem_bytes, const void* default_value, void* out, void* stream);
int o3dml_reduce_subarrays_sum(const float* values, const int64_t* row_splits, int64_t n_rows, float* out,
                               void* stream);

#ifdef __cplusplus
}
#endif

#endif /* O3DML_AMD_H */
