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
/* Optional kernel timing: HIP events on the launch stream around the main
 * kernels (names e.g. "frs_group_search", "frs_group_rows");
 * o3dml_timing_get synchronises on the recorded events. */
void o3dml_timing_enable(int on);
void o3dml_timing_reset(void);
int o3dml_timing_get(const char* name, double* total_ms, int64_t* count);

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
 * helper's output; hash_table_splits_host: the host copy, nullable — with it,
 * tables of <= 4096 bins per batch item take a chunked counting sort instead
 * of radix passes) -> hash_table_index u32[N] (point ids by bin, ascending id
 * inside a bin), hash_table_cell_splits u32[T+1]. */
int o3dml_build_spatial_hash_table(const float* points, int64_t n_points, float radius, int64_t n_batch,
                                   const int64_t* points_row_splits, const uint32_t* hash_table_splits,
                                   const uint32_t* hash_table_splits_host, int64_t total_bins,
                                   uint32_t* hash_table_index, uint32_t* hash_table_cell_splits, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* ---- fixed radius search: replaces open3d.ml.torch.ops.fixed_radius_search
 * (layers.FixedRadiusSearch; kpconv.py:2016-2034 batch_neighbors, called from
 * ml3d/torch/dataloaders/concat_batcher.py:228,257,261; layers.SparseConv's
 * Linf search, sparseconvnet.py:362-367).  metric: 0 = L1, 1 = L2, 2 = Linf.
 * Neighbour order per query: Open3D hash bins ascending, point ids ascending
 * inside a bin (the canonical order).  points_row_splits_host: host copy of
 * the point row splits; self_search = 1 when queries are the points (same
 * splits) so the spatial order of the points is reused for the queries;
 * with_distances must be the same for _count and _fill. ------------------- */
size_t o3dml_fixed_radius_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t n_batch);
int o3dml_fixed_radius_search_count(const float* points, int64_t n_points, const float* queries,
                                    int64_t n_queries, float radius, int64_t n_batch,
                                    const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                    const int64_t* points_row_splits_host, const uint32_t* hash_table_splits,
                                    const uint32_t* hash_table_index, const uint32_t* hash_table_cell_splits,
                                    int metric, int ignore_query_point, int self_search, int with_distances,
                                    int64_t* neighbors_row_splits, void* workspace, size_t workspace_bytes,
                                    void* stream);
/* totals[0] = neighbors_row_splits[M], totals[1] = the count of rows longer
 * than 64 (the workspace's first int64), written by one small kernel on the
 * stream — totals may be pinned host memory, so the host reads both after an
 * event without a separate device-to-host copy. */
int o3dml_fixed_radius_search_totals(const int64_t* neighbors_row_splits, int64_t n_queries, void* workspace,
                                     int64_t* totals, void* stream);
/* device int64 [3] = total, number of rows longer than 64, widest row (no
 * host transfer: the caller batches several sizes into one read) */
int o3dml_fixed_radius_search_sizes(const int64_t* neighbors_row_splits, int64_t n_queries, const void* workspace,
                                    int64_t* sizes, void* stream);
/* index_bits 32 or 64 (index_dtype); neighbors_distance nullable (squared for L2). */
int o3dml_fixed_radius_search_fill(const float* points, int64_t n_points, const float* queries,
                                   int64_t n_queries, float radius, int64_t n_batch,
                                   const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                   const int64_t* points_row_splits_host, const uint32_t* hash_table_splits,
                                   const uint32_t* hash_table_index, const uint32_t* hash_table_cell_splits,
                                   int metric, int ignore_query_point, int self_search, int with_distances,
                                   const int64_t* neighbors_row_splits, int index_bits, void* neighbors_index,
                                   float* neighbors_distance, void* workspace, size_t workspace_bytes, void* stream);
/* _fill into caller buffers of `capacity` entries allocated before the total
 * is known (capacity < 0: unbounded = _fill).  When neighbors_row_splits[M] >
 * capacity nothing is written; the caller reads the total and re-runs _fill.
 * parts: 1 = the row copy, 2 = the re-run of rows longer than 64 (3 = both,
 * as _fill); a caller that read the overflow count (the first int64 of the
 * workspace, see o3dml_fixed_radius_search_count) as zero may omit 2.
 * Lets the host queue the fill before its read of the total (no idle GPU
 * while the host waits).  Extension: Open3D's op (outside this repository's
 * reference tree) reads the total before it allocates the outputs. */
int o3dml_fixed_radius_search_fill_bounded(const float* points, int64_t n_points, const float* queries,
                                           int64_t n_queries, float radius, int64_t n_batch,
                                           const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                           const int64_t* points_row_splits_host,
                                           const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                           const uint32_t* hash_table_cell_splits, int metric,
                                           int ignore_query_point, int self_search, int with_distances,
                                           const int64_t* neighbors_row_splits, int index_bits,
                                           void* neighbors_index, float* neighbors_distance, int64_t capacity,
                                           int parts, void* workspace, size_t workspace_bytes, void* stream);

/* layers.FixedRadiusSearch forward in one call (kpconv.py:2021-2023 builds the
 * table, then searches; Open3D's layer does the same in two ops).  workspace
 * >= _layer_workspace_size (the search plan + scratch for the table build).
 * stage 0: the table build into hash_table_index / hash_table_cell_splits
 * when build_table (else they hold a table of these points at this radius),
 * the count, totals[0..1] = (total, rows longer than 64) written by the
 * scan's last tile (nullable; may be pinned host memory), sizes[0..2] = (total,
 * rows longer than 64, widest row) on the device (nullable), count_done
 * (nullable hipEvent_t) recorded, and — when capacity >= 0 — the row copy into
 * buffers of `capacity` entries (as _fill_bounded parts 1; nothing written
 * when the total exceeds it); stage 4 = stage 0 with the re-run of rows
 * longer than 64 queued beside that copy too (it reads the overflow count on
 * the device).  stage 1..3: _fill_bounded with parts = stage (the re-run of
 * long rows; exact buffers after a short capacity). */
size_t o3dml_fixed_radius_search_layer_workspace_size(int64_t n_points, int64_t n_queries, int64_t n_batch,
                                                      int64_t total_bins);
int o3dml_fixed_radius_search_layer(const float* points, int64_t n_points, const float* queries,
                                    int64_t n_queries, float radius, int64_t n_batch,
                                    const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                    const int64_t* points_row_splits_host, const uint32_t* hash_table_splits,
                                    const uint32_t* hash_table_splits_host, int64_t total_bins,
                                    uint32_t* hash_table_index, uint32_t* hash_table_cell_splits, int build_table,
                                    int metric, int ignore_query_point, int self_search, int with_distances,
                                    int64_t* neighbors_row_splits, int64_t* totals, int64_t* sizes, int index_bits,
                                    void* neighbors_index, float* neighbors_distance, int64_t capacity, int stage,
                                    void* count_done, void* workspace, size_t workspace_bytes, void* stream);
/* The fill of a counted search (_layer or _count workspace) as KPConv's dense
 * neighbour matrix (kpconv.py:2002-2034 batch_neighbors = fixed_radius_search
 * + ragged_to_dense): int32 [M, width] (width >= the widest row), row q = its
 * neighbours in the canonical order then pad_value.  parts as _fill_bounded. */
int o3dml_fixed_radius_search_fill_dense(const float* queries, int64_t n_points, int64_t n_queries, float radius,
                                         int64_t n_batch, const int64_t* points_row_splits,
                                         const int64_t* queries_row_splits, const int64_t* points_row_splits_host,
                                         const uint32_t* hash_table_splits, const uint32_t* hash_table_cell_splits,
                                         int metric, int ignore_query_point, const int64_t* neighbors_row_splits,
                                         int64_t width, int32_t pad_value, int32_t* neighbors_dense, int parts,
                                         void* workspace, size_t workspace_bytes, void* stream);

/* ---- kNN: replaces open3d.ml.torch.ops.knn_search / layers.KNNSearch
 * (ml3d/torch/models/point_transformer.py:724-729) and
 * open3d.core.nns.NearestNeighborSearch.knn_search
 * (ml3d/datasets/utils/dataprocessing.py:99-101 <- randlanet.py:218-229).
 * Per query the min(k, N_b) nearest points of its batch item, ascending
 * (distance, index); distances squared for L2.  k <= 64: grid ring search;
 * 64 < k <= 2048: batched, one workgroup per query over the cell cube that
 * holds its k nearest, LDS bitonic sort (nns_many.hip); larger k (few
 * queries, e.g. the 45,056-point patch crop) and queries whose candidates
 * overflow the LDS list: per-query full sort.  ignore_query_point drops every
 * point at the query's exact position, for every k.
 * The *_host row splits are host copies (grid planning); self_search = 1
 * when queries are the points themselves (same splits). ------------------- */
size_t o3dml_knn_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t k, int64_t n_batch);
int o3dml_knn_search_count(const float* points, int64_t n_points, const float* queries, int64_t n_queries, int64_t k,
                           int64_t n_batch, const int64_t* points_row_splits, const int64_t* queries_row_splits,
                           const int64_t* points_row_splits_host, const int64_t* queries_row_splits_host, int metric,
                           int ignore_query_point, int self_search, int64_t* neighbors_row_splits, void* workspace,
                           size_t workspace_bytes, void* stream);
int o3dml_knn_search_fill(const float* points, int64_t n_points, const float* queries, int64_t n_queries, int64_t k,
                          int64_t n_batch, const int64_t* queries_row_splits, const int64_t* points_row_splits_host,
                          const int64_t* queries_row_splits_host, int metric, int ignore_query_point,
                          const int64_t* neighbors_row_splits, int index_bits, void* neighbors_index,
                          float* neighbors_distance, void* workspace, size_t workspace_bytes, void* stream);
/* The patch crop of the spatially-regular sampler (KDTree.query(center,
 * k=num_points) then random.shuffle, ml3d/datasets/samplers/
 * semseg_spatially_regular.py:94-100, randlanet.py:175-180): the SET of the
 * k nearest points of `center` (device float[3]) among points[0, n) by
 * (distance, index), written as int64 ids in INDEX order (the caller shuffles
 * it; knn_search's distance order is not needed).  Radix selection in one
 * workgroup, no host synchronisation (graph-capturable); k <= n_points. */
size_t o3dml_knn_select_workspace_size(int64_t n_points);
int o3dml_knn_select(const float* points, int64_t n_points, const float* center, int64_t k, int metric,
                     int64_t* out_index, void* workspace, size_t workspace_bytes, void* stream);

/* ---- radius search: replaces open3d.ml.torch.ops.radius_search /
 * layers.RadiusSearch (Open3D ml ops API; SURVEY.md §2.2, no reference model
 * calls it).  Per query q every point of its batch item with
 * dist <= radii[q] (L2: squared distance <= radii[q]^2; L1; Linf), ascending
 * (distance, index); ignore_query_point drops points at the query's exact
 * position; normalize_distances divides each distance by radii[q] (L2:
 * radii[q]^2).  Phases: _count (grid build + counts -> neighbors_row_splits,
 * device), _totals ([total, longest row] into a host buffer), _fill (rows up
 * to 8192 sorted in LDS; longer rows written unsorted WITH distances), then,
 * only if the longest row exceeds 8192, _sort_long_rows with the host copy of
 * the row splits.  radii: device f32 [M]. -------------------------------- */
size_t o3dml_radius_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t n_batch);
int o3dml_radius_search_count(const float* points, int64_t n_points, const float* queries, int64_t n_queries,
                              const float* radii, int64_t n_batch, const int64_t* points_row_splits,
                              const int64_t* queries_row_splits, int metric, int ignore_query_point,
                              int64_t* neighbors_row_splits, void* workspace, size_t workspace_bytes, void* stream);
int o3dml_radius_search_totals(const int64_t* neighbors_row_splits, int64_t n_queries, void* workspace,
                               int64_t* totals, void* stream);
int o3dml_radius_search_fill(const float* points, int64_t n_points, const float* queries, int64_t n_queries,
                             const float* radii, int64_t n_batch, const int64_t* queries_row_splits, int metric,
                             int ignore_query_point, int normalize_distances, const int64_t* neighbors_row_splits,
                             int64_t max_row, int index_bits, void* neighbors_index, float* neighbors_distance,
                             void* workspace, size_t workspace_bytes, void* stream);
int o3dml_radius_search_sort_long_rows(int64_t n_points, int64_t n_queries, int64_t n_batch,
                                       const int64_t* rows_host, int index_bits, void* neighbors_index,
                                       float* neighbors_distance, void* workspace, size_t workspace_bytes,
                                       void* stream);

/* ---- RandLA-Net inference bookkeeping (randla_sampler.hip): the
 * spatially-regular sampler's per-patch steps
 * (ml3d/datasets/samplers/semseg_spatially_regular.py:79-109) and
 * RandLANet.transform's up-sampling indices (randlanet.py:212-239).
 * _possibility_min: min + first argmin of f64 possibilities [n], the centre
 *   point sub[argmin] (f32 [3], device), the min into *host_min (pinned host
 *   memory, may be NULL).
 * _patch_update: pc[i] = sub[idxs[i]], d = (dx^2 + dy^2) + dz^2 (f32),
 *   possibility[idxs[i]] += (1 - d / max d)^2 for i with keep[i] (keep NULL:
 *   all; duplicates must be masked to one), pc x, y recentred on their mean.
 * _up_from_knn: up[q] for every point q of the concatenated levels
 *   (level i = rs[i] .. rs[i+1]) = position (within level i+1) of q's
 *   nearest point among the first nxt[i] points of its level, from the
 *   (distance, index)-sorted k-lists nb (int32, indices into the
 *   concatenation; rewritten IN PLACE relative to each row's own level) —
 *   equal to knn_search(level i+1, level i, 1) minus srs[i]; the points whose
 *   list holds none are searched by brute force (srs: unused, kept for the
 *   caller's bookkeeping). ------------------------------------------------ */
size_t o3dml_randla_possibility_min_workspace_size(void);
int o3dml_randla_possibility_min(const double* possibility, int64_t n, const float* sub, int64_t* argmin,
                                 float* center, double* host_min, void* workspace, size_t workspace_bytes,
                                 void* stream);
/* dst[i] = src[perm(i)], perm a keyed (seed) bijection of [0, n) (Feistel
 * network + cycle walking): the patch shuffle. */
int o3dml_random_permute(const int64_t* src, int64_t n, uint64_t seed, int64_t* dst, void* stream);
/* keyed from device state: seed_state u64 [2] (base, counter), key =
 * splitmix64(base + counter), then counter += 1 (capturable patch step) */
int o3dml_random_permute_dev(const int64_t* src, int64_t n, uint64_t* seed_state, int64_t* dst, void* stream);
/* test_probs[idxs[i]] = smooth * test_probs[idxs[i]] + (1 - smooth) * probs[i]
 * (randlanet.py:441-465), probs f32 [n, c]; store f16 (store_half: the
 * reference's float16 test_probs arithmetic) or f32; keep masks duplicates. */
int o3dml_randla_update_probs(const float* probs, const int64_t* idxs, const uint8_t* keep, int64_t n, int c,
                              double smooth, int store_half, void* test_probs, void* stream);
size_t o3dml_randla_patch_workspace_size(int64_t n);
int o3dml_randla_patch_update(const float* sub, const int64_t* idxs, int64_t n, const float* center,
                              const uint8_t* keep, double* possibility, float* pc, void* workspace,
                              size_t workspace_bytes, void* stream);
size_t o3dml_randla_up_workspace_size(int64_t total);
int o3dml_randla_up_from_knn(int32_t* nb, int k, const float* cat, int nlev, const int64_t* rs,
                             const int64_t* nxt, const int64_t* srs, int64_t* up, void* workspace,
                             size_t workspace_bytes, void* stream);

/* ---- fused dense layer (RandLA-Net SharedMLP in eval mode,
 * ml3d/torch/models/randlanet.py:469-512, BatchNorm folded by the caller):
 * out[r] = act([a1[r] | a2[a2_index ? a2_index[r] : r]] @ weight^T + bias),
 * a1 f32 [n, k1], a2 f32 [*, k2] (k2 = 0: none), weight f32 [m, k1 + k2]
 * (torch Linear layout), bias f32 [m] or NULL, act 1 = LeakyReLU(slope),
 * 0 = identity.  Covers LocalFeatureAggregation's lrelu(mlp2(x) +
 * shortcut(feat)) (:689-692) and the decoder's [skip | upsampled] concat.
 * Workspace: split-K partial slabs when the grid is small (deep levels). */
size_t o3dml_dense_act_workspace_size(int64_t n, int k, int m);
int o3dml_dense_act(const float* a1, int k1, const float* a2, int k2, const int64_t* a2_index, const float* weight,
                    const float* bias, int64_t n, int m, int act, float slope, float* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/* ---- voxelize: replaces open3d.ml.torch.ops.voxelize
 * (ml3d/torch/models/point_pillars.py:352-357, sparseconvnet.py:293-298).
 * points f32 [N, ndim] (ndim <= 8); voxel_size / range_min / range_max are
 * HOST arrays of ndim floats.  Canonical semantics: coord_d =
 * floor((p_d - min_d) / vs_d) in double, valid iff 0 <= coord_d < extent_d,
 * voxels ordered by (batch, linear id with dim 0 fastest), points of a voxel
 * by index; first max_voxels voxels per batch item, first
 * max_points_per_voxel points per voxel.  _count writes counts_host[0] = V,
 * counts_host[1] = P.  Outputs: voxel_coords int32 [V, ndim],
 * voxel_point_indices int64 [P], voxel_point_row_splits int64 [V+1],
 * voxel_batch_splits int64 [B+1]. ------------------------------------------ */
size_t o3dml_voxelize_workspace_size(int64_t n_points, int64_t n_batch);
int o3dml_voxelize_count(const float* points, int64_t n_points, int ndim, int64_t n_batch, const int64_t* row_splits,
                         const float* voxel_size_host, const float* range_min_host, const float* range_max_host,
                         int64_t max_points_per_voxel, int64_t max_voxels, int64_t* counts_host, void* workspace,
                         size_t workspace_bytes, void* stream);
int o3dml_voxelize_fill(int64_t n_points, int ndim, int64_t n_batch, const float* voxel_size_host,
                        const float* range_min_host, const float* range_max_host, int64_t n_voxels,
                        int32_t* voxel_coords, int64_t* voxel_point_indices, int64_t* voxel_point_row_splits,
                        int64_t* voxel_batch_splits, void* workspace, size_t workspace_bytes, void* stream);

/* ---- calculate_grid: replaces ml3d/torch/models/sparseconvnet.py:388-401
 * (stride-2 output positions of Convolution, sparseconvnet.py:432).
 * positions f32 [N,3] -> unique parents 2*floor-even(trunc(p)) + 0.5 of the
 * inputs whose truncated coords are all >= 0, in lexicographic (x,y,z) order
 * (torch.unique(dim=0)).  Coordinates must be < 2^21.  _count writes M to
 * *n_out_host; _fill writes out_positions f32 [M,3]. ----------------------- */
size_t o3dml_calculate_grid_workspace_size(int64_t n_points);
int o3dml_calculate_grid_count(const float* positions, int64_t n_points, int64_t* n_out_host, void* workspace,
                               size_t workspace_bytes, void* stream);
int o3dml_calculate_grid_fill(int64_t n_points, float* out_positions, void* workspace, size_t workspace_bytes,
                              void* stream);

/* ---- SparseConvUnet eval plan: the reference InputLayer
 * (ml3d/torch/models/sparseconvnet.py:296-331: voxelize at vs = 1 in
 * [0, 40960)^3, per voxel its first point's position and its points' mean
 * features, every point's voxel) and calculate_grid of every level
 * (:388-401; level l's input = level l-1's grid / 2) in one call.
 * points f32 [n,3], features f32 [n,fdim]; outputs in caller buffers of
 * cap >= n rows per level: vox_pos f32 [cap,3], vox_feat f32 [cap,fdim],
 * index_map int64 [cap], grids f32 [n_levels][cap][3], halves f32
 * [n_levels][cap][3] or NULL (each grid / 2, the next level's positions);
 * sizes_host int64 [1 + n_levels] = voxels, then each level's grid
 * points. -------------- */
size_t o3dml_scn_plan_workspace_size(int64_t n_points);
int o3dml_scn_plan(const float* points, const float* features, int64_t n_points, int64_t cap, int fdim, int n_levels,
                   float* vox_pos, float* vox_feat, int64_t* index_map, float* grids, float* halves,
                   int64_t* sizes_host, void* workspace, size_t workspace_bytes, void* stream);

/* ---- grid subsampling: replaces open3d.ml.contrib.subsample / subsample_batch
 * (ml3d/datasets/utils/dataprocessing.py:33-49 <- randlanet.py:133-139;
 * kpconv.py:2099-2155 <- dataloaders/concat_batcher.py:245-247).  KPConv
 * grid_subsampling fp32 arithmetic; cells in ascending key order per batch
 * item, first max_p cells kept (max_p <= 0: all). _count writes the number of
 * output points to *n_out_host. -------------------------------------------- */
size_t o3dml_grid_subsample_workspace_size(int64_t n_points, int64_t n_batch);
/* count without a host synchronisation (KPFCNN collate: several counts read
 * back in one transfer): out device int64 [2 + n_batch] = output points,
 * grid-too-large flag (must be 0), output points per batch item. */
int o3dml_grid_subsample_count_async(const float* points, int64_t n_points, int64_t n_batch,
                                     const int64_t* row_splits, float dl, int64_t max_p, int64_t* out,
                                     void* workspace, size_t workspace_bytes, void* stream);
int o3dml_grid_subsample_count(const float* points, int64_t n_points, int64_t n_batch, const int64_t* row_splits,
                               const int64_t* row_splits_host, float dl, int64_t max_p, int64_t* n_out_host,
                               void* workspace, size_t workspace_bytes, void* stream);
/* The random grid orientation of KPConv's batch_grid_subsampling
 * (kpconv.py:2063-2090): out = p @ R_b (transpose: p @ R_b^T) for the points
 * of batch item b, rotations f32 [B,3,3] on the device, the reference's fp32
 * rounding ((p0 R0j + p1 R1j) + p2 R2j); out may alias points. */
int o3dml_rotate_batched(const float* points, int64_t n_points, int64_t n_batch, const int64_t* row_splits,
                         const float* rotations, int transpose, float* out, void* stream);
int o3dml_grid_subsample_fill(const float* points, int64_t n_points, int64_t n_batch, const float* features, int fdim,
                              const int32_t* classes, int ldim, float* out_points, float* out_features,
                              int32_t* out_classes, int64_t* out_lengths, void* workspace, size_t workspace_bytes,
                              void* stream);

/* ---- PointNet++ ops: replace open3d.ml.torch.ops.furthest_point_sampling,
 * ball_query, three_nn, three_interpolate, three_interpolate_grad
 * (ml3d/torch/utils/pointnet/pointnet2_utils.py:33-36, 55, 94, 129, 162, 184,
 * 212; point_transformer.py:518). ------------------------------------------ */
size_t o3dml_furthest_point_sampling_workspace_size(int64_t B, int64_t n);
int o3dml_furthest_point_sampling(const float* xyz, int64_t B, int64_t n, int64_t m, int32_t* out, void* workspace,
                                  size_t workspace_bytes, void* stream);
int o3dml_ball_query(const float* xyz, const float* center, int64_t B, int64_t n, int64_t m, float radius,
                     int64_t nsample, int32_t* out, void* stream);
int o3dml_three_nn(const float* unknown, const float* known, int64_t B, int64_t n, int64_t m, float* dist2,
                   int32_t* idx, void* stream);
int o3dml_three_interpolate(const float* features, const int32_t* idx, const float* weight, int64_t B, int64_t C,
                            int64_t m, int64_t n, float* out, void* stream);
int o3dml_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight, int64_t B, int64_t C,
                                 int64_t n, int64_t m, float* grad_features, void* stream);
/* deterministic three_interpolate_grad: fixed summation order (pairs grouped
 * by source point with a stable radix sort); grad_features fully written */
size_t o3dml_three_interpolate_grad_workspace_size(int64_t B, int64_t n, int64_t m);
int o3dml_three_interpolate_grad_det(const float* grad_out, const int32_t* idx, const float* weight, int64_t B,
                                     int64_t C, int64_t n, int64_t m, float* grad_features, void* workspace,
                                     size_t workspace_bytes, void* stream);

/* ---- rotated BEV NMS: replaces open3d.ml.torch.ops.nms
 * (ml3d/torch/utils/objdet_helper.py:27, called by multiclass_nms :346 from
 * point_pillars.py:1005).  boxes f32 [N,5] (x1,y1,x2,y2,yaw), scores f32 [N];
 * keep int64 [N] receives the kept original indices in descending-score order
 * and *keep_count (device int64) their number.  N <= 65536. -------------- */
size_t o3dml_nms_workspace_size(int64_t n);
int o3dml_nms(const float* boxes, const float* scores, int64_t n, float nms_overlap_thresh, int64_t* keep,
              int64_t* keep_count, void* workspace, size_t workspace_bytes, void* stream);

/* ---- sparse convolution: replaces open3d.ml.torch.ops.sparse_conv,
 * sparse_conv_transpose and their gradients, bound by layers.SparseConv /
 * layers.SparseConvTranspose (ml3d/torch/models/sparseconvnet.py:344-482;
 * filters [k,k,k,Cin,Cout] per load_unet_wts :660-677).
 * 1) o3dml_sparse_conv_build_map: CSR pairs (over OUTPUT points) -> dense
 *    kernel map [n_out*K] (+ inverse map for the input gradient) in
 *    `workspace`; status_host[0] bit0 = duplicate (o,k), bit1 = kernel index
 *    out of [0, K), bit3 = neighbour index out of [0, n_in) (pair dropped).
 * 2) o3dml_sparse_conv_forward: implicit GEMM on MFMA (f32-accurate bf16x6
 *    products by default, see o3dml_sparse_conv_set_exact).
 * 3) o3dml_sparse_conv_backward: grad_inp (inverse map, W^T) and
 *    grad_filters (per-offset pair lists, split-K slabs, fixed-order reduce).
 * o3dml_sparse_conv_kernel_index: the layer's rulebook — kernel index of
 * each (query, input) pair, per axis floor((p-q)/vs + k/2) (mirror:
 * floor(k/2 - (p-q)/vs)), linearised (z*k1 + y)*k2 + x. -------------------- */
size_t o3dml_sparse_conv_map_workspace_size(int64_t n_out, int64_t n_in, int K);
int o3dml_sparse_conv_build_map(const int32_t* neighbors_index, const int32_t* neighbors_kernel_index,
                                const float* neighbors_importance, const int64_t* neighbors_row_splits, int64_t n_out,
                                int64_t n_in, int K, int normalize, const float* out_importance, int want_inverse,
                                int* status_host, void* workspace, size_t workspace_bytes, void* stream);
/* split-K partial sums for the forward GEMM (deep levels with few output
 * rows split the offset x Cin reduction across waves; 0 when unsplit) */
size_t o3dml_sparse_conv_forward_workspace_size(int64_t n_out, int64_t n_in, int K, int cin, int cout);
int o3dml_sparse_conv_forward(const float* filters, int K, int cin, int cout, const float* inp_features, int64_t n_in,
                              const float* inp_importance, int has_neighbors_importance, int use_out_scale,
                              const float* bias, int64_t n_out, float* out_features, void* map_workspace,
                              size_t map_workspace_bytes, void* workspace, size_t workspace_bytes, void* stream);
/* forward with an input prologue relu(x * pre_scale + pre_shift) (eval-mode
 * BatchNorm + ReLU folded per channel) and a residual added in the epilogue;
 * pre_* [cin] and residual [n_out, cout] nullable; no importance / normalize.
 * filters_t: the filters TRANSPOSED, [K][cout][cin] (constant eval weights,
 * transposed once by the host). */
int o3dml_sparse_conv_forward_fused(const float* filters_t, int K, int cin, int cout, const float* inp_features,
                                    int64_t n_in, const float* pre_scale, const float* pre_shift,
                                    const float* residual, const float* bias, int64_t n_out, float* out_features,
                                    void* map_workspace, size_t map_workspace_bytes, void* workspace,
                                    size_t workspace_bytes, void* stream);
size_t o3dml_sparse_conv_backward_workspace_size(int64_t n_out, int64_t n_in, int K, int cin, int cout);
int o3dml_sparse_conv_backward(const float* filters, int K, int cin, int cout, const float* inp_features, int64_t n_in,
                               const float* inp_importance, int has_neighbors_importance, int use_out_scale,
                               const float* grad_out, int64_t n_out, float* grad_inp, float* grad_filters,
                               void* map_workspace, size_t map_workspace_bytes, void* workspace,
                               size_t workspace_bytes, void* stream);
/* Product precision of the sparse-conv gather-GEMMs (forward, input
 * gradient and filter gradient), all accumulating in f32:
 *   0 (default) "bf16x6": each f32 operand split into three bf16 terms
 *     (hi + mid + lo holds all 24 mantissa bits) and the six products down to
 *     2^-16 relative taken on the bf16 MFMA pipe — the dropped terms are below
 *     the f32 rounding level;
 *   1 exact f32-input MFMA (v_mfma_f32_32x32x2_f32, bitwise an fmaf chain);
 *   2 "bf16x3": hi + mid only, three products (~2^-17 relative per product).
 * Env O3DML_SPARSE_CONV_EXACT sets the initial mode.  Returns the previous
 * mode (-1 for a mode > 2, nothing changed); exact < 0 only queries. */
int o3dml_sparse_conv_set_exact(int exact);
/* Operand presplit for the bf16x6 / bf16x3 products (default OFF, measured
 * slower on MI355X; see sparse_conv.hip): the hi /
 * mid / lo bf16 planes of the source rows and filters are made once per GEMM
 * (workspace from the *_workspace_size functions) and the GEMM kernel only
 * loads them; the sums are bit-identical to the in-kernel split.  on = 0 / 1
 * sets, < 0 queries; returns the previous setting. */
int o3dml_sparse_conv_set_presplit(int on);
/* Filters split into bf16 hi / mid / lo once per call for the narrow-output
 * GEMM (default on; same bits either way).  on < 0 only queries; returns the
 * previous setting. */
int o3dml_sparse_conv_set_bsplit(int on);
int o3dml_sparse_conv_kernel_index(const float* inp_positions, const float* query_positions,
                                   const int32_t* neighbors_index, const int64_t* neighbors_row_splits,
                                   int64_t n_query, const int32_t* ksize_host, float voxel_size, int mirror,
                                   int32_t* kernel_index, void* stream);

/* Lattice rulebook for cubic ks^3 (ks <= 3) layers.SparseConv /
 * SparseConvTranspose (sparseconvnet.py:344-482): when every input position
 * and every query (out_pos -/+ offset*vs) lies on one voxel lattice, the Linf
 * neighbourhood of radius ks*vs/2 is exactly the ks^3 lattice offsets, so the
 * dense kernel map (same workspace layout as _build_map) comes from a voxel
 * hash with K lookups per output.  status_host[0] bit 2 (value 4): not a
 * lattice set — use the fixed-radius-search rulebook instead.  The test runs
 * on the device; defer_status = 1 skips the host round trip (status_host
 * stays 0 unless a set is empty) and leaves the status word in the map
 * workspace at o3dml_sparse_conv_map_status_offset — a failed test leaves an
 * all-empty (safe) map. */
/* Tile order of a built kernel map (and of its inverse with inverse = 1): the
 * map rows stably sorted by a hash of their offset mask, so that every
 * 32-row GEMM tile walks (almost) only offsets all its rows use; the GEMMs
 * use it from then on (a device flag in the map workspace).  It also writes
 * the map rows in that order (padded to 128-row blocks), so a tile loads its
 * rows as one contiguous block (map workspace size includes both).  Optional;
 * pays off when the map serves several convolutions or wide channels.
 * Results are unchanged (absent offsets only ever added exact zeros). */
int o3dml_sparse_conv_tile_order(void* map_workspace, size_t map_workspace_bytes, int64_t n_out, int64_t n_in, int K,
                                 int inverse, void* stream);
size_t o3dml_sparse_conv_lattice_workspace_size(int64_t n_in);
size_t o3dml_sparse_conv_map_status_offset(int64_t n_out, int64_t n_in, int K);
int o3dml_sparse_conv_lattice_map(const float* inp_pos, int64_t n_in, const float* query_pos, int64_t n_out,
                                  float voxel_size, int ksize, int mirror, int normalize, const float* out_importance,
                                  int want_inverse, int defer_status, int* status_host, void* workspace,
                                  size_t workspace_bytes, void* lattice_workspace, size_t lattice_workspace_bytes,
                                  void* stream);
/* o3dml_sparse_conv_lattice_map with the queries query_pos - query_shift
 * (host float[3], or NULL): the layer's out_pos - offset * voxel_size
 * (sparseconvnet.py:363-370 queries) subtracted in f32 inside the map
 * kernels, bit-identical to materialising it. */
int o3dml_sparse_conv_lattice_map_shifted(const float* inp_pos, int64_t n_in, const float* query_pos,
                                          const float* query_shift, int64_t n_out, float voxel_size, int ksize,
                                          int mirror, int normalize, const float* out_importance, int want_inverse,
                                          int defer_status, int* status_host, void* workspace, size_t workspace_bytes,
                                          void* lattice_workspace, size_t lattice_workspace_bytes, void* stream);
/* The kernel map of the SparseConvTranspose that undoes a built SparseConv
 * map (same positions swapped, same kernel size, voxel size and offset: a
 * pair (coarse c, fine f) of the convolution at kernel index k is the pair
 * (f, c) of the transpose at the same index — SparseConvUnet's DeConvolution
 * after its Convolution, sparseconvnet.py:404-482): out_workspace (a map
 * workspace for n_out = n_fine, n_in = n_coarse) gets the inverse of the
 * convolution's map (and, with want_inverse, the map itself as its inverse)
 * and the convolution's status word — no voxel hash, no lookups. */
int o3dml_sparse_conv_transpose_map(const void* conv_workspace, size_t conv_workspace_bytes, int64_t n_coarse,
                                    int64_t n_fine, int K, int want_inverse, void* out_workspace,
                                    size_t out_workspace_bytes, void* stream);

/* ---- KPConv neighbourhood aggregation (ml3d/torch/models/
 * kpconv.py:1005-1159).  q_pts f32 [n,3], s_pts f32 [n_support,3], neighbors
 * [n, nb] (int32/int64 per index_bits; index n_support = shadow, zero
 * contribution), features f32 [n_support, cin], kernel_points f32 [K,3] or
 * per query [n,K,3] (kp_per_query), influence 0 constant / 1 linear /
 * 2 gaussian, closest = nearest-kernel-point aggregation, modulations f32
 * [n,K] nullable -> out WF f32 [n, K, cin] with WF[q,k] = sum_j infl * x[j].
 * The backward accumulates grad_features [n_support, cin] (must be zeroed)
 * from grad WF with fp32 atomics. ---------------------------------------- */
int o3dml_kpconv_weighted_features(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                   const void* neighbors, int index_bits, int nb, const float* features, int cin,
                                   const float* kernel_points, int K, int kp_per_query, float extent, int influence,
                                   int closest, const float* modulations, float* out, void* stream);
int o3dml_kpconv_weighted_features_backward(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                            const void* neighbors, int index_bits, int nb, const float* grad_wf,
                                            int cin, const float* kernel_points, int K, int kp_per_query,
                                            float extent, int influence, int closest, float* grad_features,
                                            void* stream);
/* Deterministic variant (selected under torch.use_deterministic_algorithms):
 * grad_features fully written (no zeroing needed), each support summing its
 * (query, column) pairs in ascending order after a stable radix sort of the
 * neighbour matrix by support index; workspace from
 * o3dml_kpconv_inverse_workspace_size(n, nb, n_support). */
size_t o3dml_kpconv_inverse_workspace_size(int64_t n, int nb, int64_t n_support);
int o3dml_kpconv_weighted_features_backward_det(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                                const void* neighbors, int index_bits, int nb, const float* grad_wf,
                                                int cin, const float* kernel_points, int K, int kp_per_query,
                                                float extent, int influence, int closest, float* grad_features,
                                                void* workspace, size_t workspace_bytes, void* stream);
/* Deformable training (kp_per_query): per-query neighbours with no kernel
 * point within extent are dropped in forward and backward, as the
 * reference's in_range filter (kpconv.py:1076-1103).  _kernel_point_grad:
 * grad_kp f32 [n,K,3] and grad_mod f32 [n,K] (nullable) from grad WF
 * (before the modulation) for per-query kernel points [n,K,3].
 * _min_d2_columns: per (query, kernel point) the neighbour column nearest
 * to it (shadow at 1e6 included; min_d2 of kpconv.py:1071). */
int o3dml_kpconv_kernel_point_grad(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                   const void* neighbors, int index_bits, int nb, const float* features, int cin,
                                   const float* grad_wf, const float* kernel_points, int K, float extent,
                                   int influence, int closest, const float* modulations, float* grad_kp,
                                   float* grad_mod, void* stream);
int o3dml_kpconv_min_d2_columns(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                const void* neighbors, int index_bits, int nb, const float* kernel_points, int K,
                                int32_t* columns, void* stream);

/* ---- KPFCNN pooling (kpconv.py:821-858 max_pool /
 * closest_pool).  x f32 [n_support, c]; inds [n, ld] int32/int64 (index
 * n_support = shadow row of zeros); the first nb columns are pooled
 * (closest_pool: nb = 1) -> out f32 [n, c], argmax int32 [n, c] (nullable;
 * winning support index, n_support = shadow).  Backward adds grad_out into
 * grad_x [n_support, c] (must be zeroed) at argmax with fp32 atomics. */
int o3dml_kpconv_pool_max(const float* x, int64_t n_support, int c, const void* inds, int index_bits, int64_t ld,
                          int64_t n, int nb, float* out, int32_t* argmax, void* stream);
int o3dml_kpconv_pool_max_backward(const float* grad_out, const int32_t* argmax, int64_t n, int c, int64_t n_support,
                                   float* grad_x, void* stream);
/* deterministic: gathers over the inverse of inds (workspace
 * o3dml_kpconv_inverse_workspace_size(n, nb, n_support)); grad_x fully written */
int o3dml_kpconv_pool_max_backward_det(const float* grad_out, const int32_t* argmax, const void* inds, int index_bits,
                                       int64_t ld, int64_t n, int nb, int c, int64_t n_support, float* grad_x,
                                       void* workspace, size_t workspace_bytes, void* stream);

/* ---- fp32 GEMM through rocBLAS (the KPFCNN Linear / KPConv GEMMs, forward
 * and backward; replaces torch.matmul in UnaryBlock.mlp and KPConv.forward,
 * ml3d/torch/models/kpconv.py:1155-1159, 1290).  Row-major C[m, n] = alpha
 * op(A) op(B) + beta C; trans_a: A stored [k, m], trans_b: B stored [n, k];
 * leading dimensions of the stored matrices, in elements. */
int o3dml_sgemm(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, float alpha, const float* a, int64_t lda,
                const float* b, int64_t ldb, float beta, float* c, int64_t ldc, void* stream);

/* o3dml_sgemm (alpha 1, beta 0) for a long reduction k with few output tiles
 * (weight gradients; deep-layer WF @ W): k split into up to 64 parts of >=
 * 2,048 (strided-batched rocBLAS), the parts summed in order (deterministic).
 * Workspace: _workspace_size(m, n, k). */
size_t o3dml_sgemm_splitk_workspace_size(int64_t m, int64_t n, int64_t k);
int o3dml_sgemm_splitk(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, const float* a, int64_t lda,
                       const float* b, int64_t ldb, float* c, int64_t ldc, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---- KPFCNN layers as one call per direction (UnaryBlock: Linear without
 * bias + BatchNorm1d + LeakyReLU, kpconv.py:1255-1295; rigid KPConv:
 * aggregation + WF @ W, kpconv.py:1005-1159), composed from o3dml_sgemm*,
 * o3dml_batch_norm_* and o3dml_kpconv_weighted_features* on one stream.
 * linear_bn: w [cout, cin]; z [n, cout] = x w^T (kept for the backward); y =
 * act(bn(z)); backward: dz scratch [n, cout], dx / dw / dgamma / dbeta nullable.
 * kpconv_rigid: w [K cin, cout]; wf [n, K, cin] kept for the backward; gwf
 * scratch [n, K cin]; dx [n_support, cin] zeroed by the call. */
size_t o3dml_linear_bn_workspace_size(int64_t n, int cin, int cout);
int o3dml_linear_bn_forward(const float* x, int64_t n, int cin, const float* w, int cout, const float* gamma,
                            const float* beta, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                            float momentum, float eps, int training, int act, float slope, float* z, float* y,
                            float* save, void* workspace, size_t workspace_bytes, void* stream);
int o3dml_linear_bn_backward(const float* gy, const float* x, int64_t n, int cin, const float* w, int cout,
                             const float* z, const float* save, int training, int act, float slope, float* dz,
                             float* dx, float* dw, float* dgamma, float* dbeta, void* workspace,
                             size_t workspace_bytes, void* stream);
size_t o3dml_kpconv_rigid_workspace_size(int64_t n, int nb, int64_t n_support, int K, int cin, int cout,
                                         int deterministic);
int o3dml_kpconv_rigid_forward(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                               const void* neighbors, int index_bits, int nb, const float* x, int cin,
                               const float* kernel_points, int K, float extent, int influence, int closest,
                               const float* w, int cout, float* wf, float* out, void* workspace,
                               size_t workspace_bytes, void* stream);
int o3dml_kpconv_rigid_backward(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                const void* neighbors, int index_bits, int nb, const float* g, int cin,
                                const float* kernel_points, int K, float extent, int influence, int closest,
                                const float* w, int cout, const float* wf, float* gwf, float* dx, float* dw,
                                int deterministic, void* workspace, size_t workspace_bytes, void* stream);

/* ---- KPFCNN BatchNorm1d (+ LeakyReLU) over [N, C] rows (replaces
 * nn.BatchNorm1d + nn.LeakyReLU of BatchNormBlock / UnaryBlock / SimpleBlock /
 * ResnetBottleneckBlock, ml3d/torch/models/kpconv.py:1213-1464).
 * forward: training -> batch statistics (biased variance for y; running_mean /
 * running_var updated with the unbiased one, momentum as torch; num_batches_tracked
 * += 1; any of the three may be NULL), eval -> running statistics.  y = act((x -
 * mean) * weight * invstd + bias), act = LeakyReLU(slope) when act != 0; weight /
 * bias may be NULL (1 / 0).  save [4C] = (mean, invstd, weight * invstd, bias)
 * is the backward's input.  backward: grad_x / grad_weight / grad_bias (each
 * NULLable).  Workspace: o3dml_batch_norm_workspace_size(n, c). */
size_t o3dml_batch_norm_workspace_size(int64_t n, int c);
int o3dml_batch_norm_forward(const float* x, int64_t n, int c, const float* weight, const float* bias,
                             float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum,
                             float eps, int training, int act, float slope, float* y, float* save, void* workspace,
                             size_t workspace_bytes, void* stream);
int o3dml_batch_norm_backward(const float* grad_y, const float* x, int64_t n, int c, const float* save, int training,
                              int act, float slope, float* grad_x, float* grad_weight, float* grad_bias,
                              void* workspace, size_t workspace_bytes, void* stream);

/* ---- PointPillars pillars (point_pillars.py:352-380,
 * 509-552, 567-601).
 * pillar_features: points f32 [n_points, cdim] (x, y, z, features...), the
 *   voxelize output (voxel_point_indices int64, voxel_point_row_splits int64
 *   [V+1], voxel_coords int32 [V,3] in x,y,z order) -> out f32
 *   [V, max_points, cdim + 5]: raw point, offset to the pillar mean (3),
 *   offset to the pillar centre ix*vx + x_offset, iy*vy + y_offset (2);
 *   padded slots zero.
 * pillar_scatter: features f32 [V, C], coords int32 [V, 4] (batch, z, y, x)
 *   -> canvas f32 [B, C, ny, nx] (zeroed by the caller) at [b, :, y, x].
 * pillar_gather: the adjoint (canvas -> features). */
int o3dml_pillar_features(const float* points, int64_t n_points, int cdim, const int64_t* voxel_point_indices,
                          const int64_t* voxel_point_row_splits, const int32_t* voxel_coords_xyz, int64_t n_voxels,
                          int max_points, float vx, float vy, float x_offset, float y_offset, float* out,
                          void* stream);
int o3dml_pillar_scatter(const float* features, const int32_t* coords_bzyx, int64_t n_voxels, int channels, int ny,
                         int nx, float* canvas, void* stream);
int o3dml_pillar_gather(const float* canvas, const int32_t* coords_bzyx, int64_t n_voxels, int channels, int ny,
                        int nx, float* features, void* stream);

/* ---- RandLA-Net neighbour gathers (ml3d/torch/models/
 * randlanet.py).  Channels-last: coords f32 [N,3], neighbour indices int32
 * [N,K], per-pair tensors [N,K,C], per-point [N,C].
 * relative_encoding: LocalSpatialEncoding's geometric input (randlanet.py:
 *   593-606) [|c-p|, c-p, c, p] -> out [N,K,10];
 * attentive_pool: AttentivePooling's softmax over K + weighted sum
 *   (randlanet.py:632-650): x, logits [N,K,C] -> out [N,C];
 * gather_max: random_sample (randlanet.py:306-331): out[m,c] = max_k
 *   feat[idx[m,k], c] -> [M,C]. ------------------------------------------- */
int o3dml_randla_relative_encoding(const float* coords, int64_t n, const int32_t* neighbors, int k, float* out,
                                   void* stream);
int o3dml_randla_attentive_pool(const float* x, const float* logits, int64_t n, int k, int c, float* out,
                                void* stream);
/* concat_rows: out[r] = [a[ia[r]] (da floats), b[ib[r]] (db floats)] for r <
 * rows; ia / ib nullable (identity), int32 or int64 per *_bits. */
int o3dml_concat_rows(const float* a, int da, const void* ia, int ia_bits, const float* b, int db, const void* ib,
                      int ib_bits, int64_t rows, float* out, void* stream);
/* att_pool: fused LocalSpatialEncoding + AttentivePooling (randlanet.py:
 * 540-650) for k == 16 neighbours and width d in {16, 32, 64, 128, 256}:
 * rel_j = leaky_0.2(Wr r_j + br) with r_j the 10-value relative encoding of
 * (n, neighbors[n, j]) (rel_in null) or rel_in [N, k, d/2];
 * F_j = [x[neighbors[n, j]] (x [N, d/2]), rel_j]; s_j = Ws F_j + bs;
 * out[n] = sum_j softmax_j(s_j) * F_j -> out [N, d].  Weights transposed:
 * wr_t [in][d/2], ws_t [d][d] (in-major).  rel_out [N, k, d/2] nullable. */
int o3dml_randla_att_pool(const float* coords, const float* x, const int32_t* neighbors, int64_t n, int k, int d,
                          const float* rel_in, const float* wr_t, const float* br, const float* ws_t,
                          const float* bs, float* rel_out, float* out, void* stream);
int o3dml_randla_gather_max(const float* feat, int c, const int32_t* idx, int64_t m, int k, float* out,
                            void* stream);

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

/* ---- stable key sort -----------------------------------------------------
 * The stable LSD radix sort behind every order the ops define (bins, voxels,
 * grid cells, tile orders): (keys, vals) sorted by key, ties in input order,
 * for keys < 2^end_bit (the passes cover only those bits); vals_in NULL =
 * element index.  key_bytes 4 or 8;
 * small_kind picks the one-workgroup sort used for n <= 8,192 (-1 default,
 * 0 LSD radix, 1 bitonic).  No reference entry point: Open3D sorts inside
 * its C++ ops (e.g. std::stable_sort in the voxelize / grid CPU kernels). */
size_t o3dml_sort_pairs_workspace_size(int64_t n, int key_bytes);
int o3dml_sort_pairs(const void* keys_in, const uint32_t* vals_in, void* keys_out, uint32_t* vals_out, int64_t n,
                     int key_bytes, int end_bit, int small_kind, void* workspace, size_t workspace_bytes,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* O3DML_AMD_H */
