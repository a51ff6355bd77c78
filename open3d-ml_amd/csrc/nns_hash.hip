// nns_hash.hip — spatial hash table build + fixed-radius neighbour search
// (Open3D ops.build_spatial_hash_table / ops.fixed_radius_search /
// layers.FixedRadiusSearch).
//
// HBM layout
//   points            f32 [N,3]  (caller, row-split batched)
//   hash_table_index  u32 [N]    point ids sorted by (bin, id)  — stable LSD radix
//   cell_splits       u32 [T+1]  CSR over bins, T = sum_b table_size_b
//   pts_sorted        f32x4 [N]  workspace: (x,y,z,id) in bin order, so a bin
//                                scan is one contiguous 16-B-per-point stream
// Search: one lane per query; with query_order = hash_table_index (self
// search) the 64 queries of a wave sit in the same / adjacent cells and hit
// the same bins in L1/L2.  Neighbour order per query = ascending bin, then
// ascending point id (the canonical order of oracle/o3d_oracle.c).
#include "primitives.hpp"

namespace o3dml {

// Open3D SpatialHash: 32-bit int products XOR-ed, converted to size_t (sign
// extension), reduced modulo the table size.
__device__ __forceinline__ uint32_t spatial_bin(int32_t x, int32_t y, int32_t z, uint32_t tsize) {
    const uint32_t h = (static_cast<uint32_t>(x) * 73856096u) ^ (static_cast<uint32_t>(y) * 193649663u) ^
                       (static_cast<uint32_t>(z) * 83492791u);
    const uint64_t u = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(h)));
    return static_cast<uint32_t>(u % tsize);
}

__device__ __forceinline__ uint32_t point_bin(float x, float y, float z, float inv, uint32_t tsize) {
    return spatial_bin(static_cast<int32_t>(floorf(x * inv)), static_cast<int32_t>(floorf(y * inv)),
                       static_cast<int32_t>(floorf(z * inv)), tsize);
}

__global__ void hash_points_kernel(const float* __restrict__ points, int64_t n, float inv, int n_batch,
                                   const int64_t* __restrict__ prs, const uint32_t* __restrict__ hts,
                                   uint32_t* __restrict__ bins) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(i, prs, n_batch);
        const uint32_t first = hts[b];
        const uint32_t tsize = hts[b + 1] - first;
        bins[i] = first + point_bin(points[3 * i], points[3 * i + 1], points[3 * i + 2], inv, tsize);
    }
}

// cell_splits[b] = first position of bin b in the sorted key array.
__global__ void bin_boundaries_kernel(const uint32_t* __restrict__ skeys, int64_t n, int64_t total_bins,
                                      uint32_t* __restrict__ cell_splits) {
    if (n == 0) {
        for (int64_t b = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; b <= total_bins;
             b += static_cast<int64_t>(gridDim.x) * blockDim.x)
            cell_splits[b] = 0;
        return;
    }
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = skeys[j];
        const int64_t kp = j == 0 ? -1 : static_cast<int64_t>(skeys[j - 1]);
        for (int64_t b = kp + 1; b <= k; ++b) cell_splits[b] = static_cast<uint32_t>(j);
        if (j == n - 1)
            for (int64_t b = k + 1; b <= total_bins; ++b) cell_splits[b] = static_cast<uint32_t>(n);
    }
}

__global__ void gather_sorted_points_kernel(const float* __restrict__ points, const uint32_t* __restrict__ index,
                                            int64_t n, float4* __restrict__ out) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t i = index[j];
        out[j] = make_float4(points[3 * static_cast<int64_t>(i)], points[3 * static_cast<int64_t>(i) + 1],
                             points[3 * static_cast<int64_t>(i) + 2], __uint_as_float(i));
    }
}

__device__ __forceinline__ void cswap(uint32_t& a, uint32_t& b) {
    const uint32_t lo = a < b ? a : b;
    const uint32_t hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// The 9 bins a query visits (own voxel + the 8 corners q ± r), sorted
// ascending; duplicates are skipped by the caller (bins[k] == bins[k-1]).
struct QueryBins {
    uint32_t b[9];
};

__device__ __forceinline__ QueryBins query_bins(float qx, float qy, float qz, float r, float inv, uint32_t first,
                                                uint32_t tsize) {
    QueryBins s;
    s.b[0] = point_bin(qx, qy, qz, inv, tsize);
    const float xs[2] = {qx - r, qx + r};
    const float ys[2] = {qy - r, qy + r};
    const float zs[2] = {qz - r, qz + r};
#pragma unroll
    for (int c = 0; c < 8; ++c) s.b[1 + c] = point_bin(xs[c & 1], ys[(c >> 1) & 1], zs[c >> 2], inv, tsize);
    // odd-even transposition network, 9 stages -> fully sorted
#pragma unroll
    for (int st = 0; st < 9; ++st) {
#pragma unroll
        for (int i = (st & 1); i + 1 < 9; i += 2) cswap(s.b[i], s.b[i + 1]);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) s.b[i] += first;
    return s;
}

template <int METRIC, bool IGNORE, bool FILL, class TIdx>
__global__ void __launch_bounds__(256) frs_kernel(const float4* __restrict__ pts_sorted, const float* __restrict__ queries,
                                                  int64_t n_queries, const uint32_t* __restrict__ qorder, float r,
                                                  float inv, float thr, int n_batch,
                                                  const int64_t* __restrict__ qrs, const uint32_t* __restrict__ hts,
                                                  const uint32_t* __restrict__ cs, int64_t* __restrict__ row_splits,
                                                  TIdx* __restrict__ out_idx, float* __restrict__ out_dist) {
    for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < n_queries;
         t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = qorder ? static_cast<int64_t>(qorder[t]) : t;
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        const int b = batch_of(q, qrs, n_batch);
        const uint32_t first = hts[b];
        const QueryBins bins = query_bins(qx, qy, qz, r, inv, first, hts[b + 1] - first);
        int64_t cnt = 0;
        int64_t o = 0;
        if constexpr (FILL) o = row_splits[q];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if (k > 0 && bins.b[k] == bins.b[k - 1]) continue;
            const uint32_t s = cs[bins.b[k]], e = cs[bins.b[k] + 1];
            for (uint32_t j = s; j < e; ++j) {
                const float4 p = pts_sorted[j];
                if (IGNORE && p.x == qx && p.y == qy && p.z == qz) continue;
                const float d = dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz);
                if (d <= thr) {
                    if constexpr (FILL) {
                        out_idx[o] = static_cast<TIdx>(__float_as_uint(p.w));
                        if (out_dist) out_dist[o] = d;
                        ++o;
                    } else {
                        ++cnt;
                    }
                }
            }
        }
        if constexpr (!FILL) row_splits[q + 1] = cnt;
    }
}

template <bool FILL, class TIdx>
static void launch_frs(int metric, bool ignore, unsigned grid, hipStream_t st, const float4* pts,
                       const float* queries, int64_t m, const uint32_t* qorder, float r, float inv, float thr,
                       int nb, const int64_t* qrs, const uint32_t* hts, const uint32_t* cs, int64_t* rs, TIdx* idx,
                       float* dist) {
#define O3DML_FRS(M, I) \
    frs_kernel<M, I, FILL, TIdx><<<grid, 256, 0, st>>>(pts, queries, m, qorder, r, inv, thr, nb, qrs, hts, cs, rs, idx, dist)
    if (metric == kL2) {
        if (ignore) O3DML_FRS(kL2, true); else O3DML_FRS(kL2, false);
    } else if (metric == kL1) {
        if (ignore) O3DML_FRS(kL1, true); else O3DML_FRS(kL1, false);
    } else {
        if (ignore) O3DML_FRS(kLinf, true); else O3DML_FRS(kLinf, false);
    }
#undef O3DML_FRS
    O3DML_LAUNCH_CHECK();
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int64_t o3dml_hash_table_splits(int64_t n_batch, const int64_t* points_row_splits_host,
                                          double hash_table_size_factor, int64_t max_hash_table_size,
                                          uint32_t* hash_table_splits_host) {
    hash_table_splits_host[0] = 0;
    for (int64_t b = 0; b < n_batch; ++b) {
        const int64_t nb = points_row_splits_host[b + 1] - points_row_splits_host[b];
        int64_t t = static_cast<int64_t>(hash_table_size_factor * static_cast<double>(nb));
        if (t < 1) t = 1;
        if (t > max_hash_table_size) t = max_hash_table_size;
        hash_table_splits_host[b + 1] = hash_table_splits_host[b] + static_cast<uint32_t>(t);
    }
    return hash_table_splits_host[n_batch];
}

O3DML_API size_t o3dml_build_spatial_hash_table_workspace_size(int64_t n_points, int64_t total_bins) {
    (void)total_bins;
    return ws_bytes<uint32_t>(n_points) * 2 + prim::radix_sort_workspace_bytes<uint32_t>(n_points);
}

O3DML_API int o3dml_build_spatial_hash_table(const float* points, int64_t n_points, float radius, int64_t n_batch,
                                             const int64_t* points_row_splits, const uint32_t* hash_table_splits,
                                             int64_t total_bins, uint32_t* hash_table_index,
                                             uint32_t* hash_table_cell_splits, void* workspace,
                                             size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(radius > 0.f, "radius must be > 0");
    O3DML_REQUIRE(n_batch >= 1, "need at least one batch item");
    O3DML_REQUIRE(total_bins >= n_batch && total_bins < (int64_t(1) << 32), "invalid hash table size %lld",
                  (long long)total_bins);
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const float inv = 1.0f / (2.0f * radius);
    uint32_t* bins = ws.take<uint32_t>(n_points);
    uint32_t* skeys = ws.take<uint32_t>(n_points);
    if (n_points > 0) {
        hash_points_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(points, n_points, inv, (int)n_batch,
                                                                      points_row_splits, hash_table_splits, bins);
        O3DML_LAUNCH_CHECK();
        prim::radix_sort_pairs<uint32_t>(bins, nullptr, skeys, hash_table_index, n_points,
                                         prim::bits_needed(static_cast<uint64_t>(total_bins - 1)), ws, st);
    }
    bin_boundaries_kernel<<<stream_grid(n_points > 0 ? n_points : total_bins + 1, 256), 256, 0, st>>>(
            skeys, n_points, total_bins, hash_table_cell_splits);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_fixed_radius_search_workspace_size(int64_t n_points, int64_t n_queries) {
    return ws_bytes<float4>(n_points) + prim::scan_workspace_bytes(n_queries);
}

O3DML_API int o3dml_fixed_radius_search_count(const float* points, int64_t n_points, const float* queries,
                                              int64_t n_queries, float radius, int64_t n_batch,
                                              const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                              const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                              const uint32_t* hash_table_cell_splits, const uint32_t* query_order,
                                              int metric, int ignore_query_point, int64_t* neighbors_row_splits,
                                              void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    (void)points_row_splits;
    O3DML_REQUIRE(metric >= 0 && metric <= 2, "metric must be L1(0), L2(1) or Linf(2)");
    O3DML_REQUIRE(radius > 0.f, "radius must be > 0");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    float4* pts = ws.take<float4>(n_points);
    O3DML_CHECK_HIP(hipMemsetAsync(neighbors_row_splits, 0, sizeof(int64_t), st));
    if (n_queries == 0) return 0;
    if (n_points == 0) {
        O3DML_CHECK_HIP(hipMemsetAsync(neighbors_row_splits, 0, sizeof(int64_t) * (n_queries + 1), st));
        return 0;
    }
    gather_sorted_points_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(points, hash_table_index, n_points, pts);
    O3DML_LAUNCH_CHECK();
    const float inv = 1.0f / (2.0f * radius);
    const float thr = metric == kL2 ? radius * radius : radius;
    launch_frs<false, int32_t>(metric, ignore_query_point != 0, stream_grid(n_queries, 256, 1 << 20), st, pts,
                               queries, n_queries, query_order, radius, inv, thr, (int)n_batch, queries_row_splits,
                               hash_table_splits, hash_table_cell_splits, neighbors_row_splits, nullptr, nullptr);
    prim::scan<int64_t, int64_t>(neighbors_row_splits + 1, neighbors_row_splits + 1, n_queries, true, ws, st);
    O3DML_GUARD_END
}

O3DML_API int o3dml_fixed_radius_search_fill(const float* points, int64_t n_points, const float* queries,
                                             int64_t n_queries, float radius, int64_t n_batch,
                                             const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                             const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                             const uint32_t* hash_table_cell_splits, const uint32_t* query_order,
                                             int metric, int ignore_query_point,
                                             const int64_t* neighbors_row_splits, int index_bits,
                                             void* neighbors_index, float* neighbors_distance, void* workspace,
                                             size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    (void)points;
    (void)points_row_splits;
    (void)hash_table_index;
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n_queries == 0 || n_points == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const float4* pts = ws.take<float4>(n_points);  // filled by _count (same workspace)
    const float inv = 1.0f / (2.0f * radius);
    const float thr = metric == kL2 ? radius * radius : radius;
    const unsigned grid = stream_grid(n_queries, 256, 1 << 20);
    int64_t* rs = const_cast<int64_t*>(neighbors_row_splits);
    if (index_bits == 32)
        launch_frs<true, int32_t>(metric, ignore_query_point != 0, grid, st, pts, queries, n_queries, query_order,
                                  radius, inv, thr, (int)n_batch, queries_row_splits, hash_table_splits,
                                  hash_table_cell_splits, rs, static_cast<int32_t*>(neighbors_index),
                                  neighbors_distance);
    else
        launch_frs<true, int64_t>(metric, ignore_query_point != 0, grid, st, pts, queries, n_queries, query_order,
                                  radius, inv, thr, (int)n_batch, queries_row_splits, hash_table_splits,
                                  hash_table_cell_splits, rs, static_cast<int64_t*>(neighbors_index),
                                  neighbors_distance);
    O3DML_GUARD_END
}
