// nns_hash.hip — spatial hash table build (Open3D ops.build_spatial_hash_table,
// used by layers.FixedRadiusSearch).  The search lives in
// nns_frs.hip.
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
#include <algorithm>

#include "primitives.hpp"
#include "spatial_hash.hpp"

namespace o3dml {

// Bucket of every point.  The row splits and, per batch item, the table
// offset / size / 2^64 mod size are staged in LDS, so a point costs one LDS
// binary search and a 32-bit modulo (no 64-bit division, no global search).
__global__ void __launch_bounds__(256) hash_points_kernel(const float* __restrict__ points, int64_t n, float inv,
                                                          int n_batch, const int64_t* __restrict__ prs,
                                                          const uint32_t* __restrict__ hts,
                                                          uint32_t* __restrict__ bins) {
    __shared__ int64_t s_rs[kLdsSplits];
    __shared__ uint32_t s_tab[kLdsSplits][3];  // first, size, 2^64 mod size
    const int64_t* rsp = stage_splits(s_rs, prs, n_batch);
    const bool tab = n_batch <= kLdsSplits;
    if (tab) {
        for (int b = threadIdx.x; b < n_batch; b += blockDim.x) {
            const uint32_t first = hts[b], tsize = hts[b + 1] - first;
            s_tab[b][0] = first;
            s_tab[b][1] = tsize;
            s_tab[b][2] = pow64_mod(tsize);
        }
        __syncthreads();
    }
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(i, rsp, n_batch);
        const uint32_t first = tab ? s_tab[b][0] : hts[b];
        const uint32_t tsize = tab ? s_tab[b][1] : hts[b + 1] - first;
        const uint32_t k64 = tab ? s_tab[b][2] : pow64_mod(tsize);
        bins[i] = first + point_bin_k(points[3 * i], points[3 * i + 1], points[3 * i + 2], inv, tsize, k64);
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

