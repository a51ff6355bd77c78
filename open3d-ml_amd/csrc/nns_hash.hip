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
#include <cstdlib>

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

// ---------------------------------------------------------------------------
// Small-table path (every batch item has <= kSmallTable bins): a stable
// counting sort per batch item, split into chunks of kHashChunk points so the
// whole GPU works on it — no radix passes.
//   plan:    chunk_start[b] (chunks of items < b, at least one per item) and
//            hist_off[b] (offset of item b's chunk histograms);
//   hist:    per chunk, the bin of every point (kept for the scatter) and the
//            chunk's bin histogram (LDS atomics: order-free);
//   scan:    per item, each bin's column of chunk counts -> the chunks'
//            first slots (bin start inside the item + earlier chunks), and
//            the item's cell_splits;
//   scatter: per chunk, the points ranked stably inside the chunk (ballot
//            peers, per-wave counts in LDS), ids written to their slots.
// ---------------------------------------------------------------------------
constexpr int kSmallTable = 4096;
// points per chunk = 4 waves x 16 rows of 64; calls with few points take
// chunks of 1024 (4 rows per wave) so more workgroups share the work (one
// 65,536-point scene: 16 -> 64 workgroups)
constexpr int kHashChunk = 4096;
constexpr int kHashChunkSmall = 1024;
constexpr int kHashWaves = 4;

// The plan, computed by one 256-thread workgroup into cs / ho (global or LDS):
// chunk_start[b] (chunks of items < b, at least one per item) and
// hist_off[b] (offset of item b's chunk histograms), [nb] the totals.
__device__ __forceinline__ void hash_plan_block(const int64_t* __restrict__ prs, int nb,
                                                const uint32_t* __restrict__ hts, int chunk, int64_t* cs,
                                                int64_t* ho) {
    __shared__ int64_t wsum[2][4];
    int64_t carry_c = 0, carry_h = 0;
    for (int b0 = 0; b0 < nb; b0 += 256) {
        const int b = b0 + threadIdx.x;
        int64_t c = 0, h = 0;
        if (b < nb) {
            const int64_t n = prs[b + 1] - prs[b];
            c = n > chunk ? ceil_div(n, chunk) : 1;
            h = c * static_cast<int64_t>(hts[b + 1] - hts[b]);
        }
        const int64_t ic = wave_inclusive_scan(c), ih = wave_inclusive_scan(h);
        if (lane_id() == 63) {
            wsum[0][wave_id()] = ic;
            wsum[1][wave_id()] = ih;
        }
        __syncthreads();
        int64_t bc = carry_c, bh = carry_h, tc = 0, th = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wave_id()) {
                bc += wsum[0][w];
                bh += wsum[1][w];
            }
            tc += wsum[0][w];
            th += wsum[1][w];
        }
        if (b < nb) {
            cs[b] = bc + ic - c;
            ho[b] = bh + ih - h;
        }
        carry_c += tc;
        carry_h += th;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cs[nb] = carry_c;
        ho[nb] = carry_h;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) hash_plan_kernel(const int64_t* __restrict__ prs, int nb,
                                                        const uint32_t* __restrict__ hts,
                                                        int64_t* __restrict__ chunk_start,
                                                        int64_t* __restrict__ hist_off, int chunk) {
    hash_plan_block(prs, nb, hts, chunk, chunk_start, hist_off);
}

// Batches of up to kPlanLds - 1 items: every histogram workgroup computes the
// plan itself in LDS (a few hundred cycles) and workgroup 0 publishes it for
// the later kernels — no plan launch
constexpr int kPlanLds = 512;

// Batch item and chunk of workgroup blockIdx.x (false: past the last chunk).
__device__ __forceinline__ bool hash_chunk_of(const int64_t* __restrict__ chunk_start, int nb, int& b, int64_t& c) {
    const int64_t w = blockIdx.x;
    if (w >= chunk_start[nb]) return false;
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (chunk_start[mid] <= w) lo = mid; else hi = mid - 1;
    }
    b = lo;
    c = w - chunk_start[lo];
    return true;
}

template <bool PLAN>
__global__ void __launch_bounds__(256) hash_chunk_hist_kernel(const float* __restrict__ points, float inv, int nb,
                                                              const int64_t* __restrict__ prs,
                                                              const uint32_t* __restrict__ hts,
                                                              int64_t* __restrict__ chunk_start,
                                                              int64_t* __restrict__ hist_off,
                                                              uint32_t* __restrict__ bins, uint32_t* __restrict__ hist,
                                                              int chunk) {
    extern __shared__ uint32_t h[];  // [max bins per item]
    __shared__ int64_t s_plan[PLAN ? 2 * kPlanLds : 1];
    const int64_t* cs = chunk_start;
    const int64_t* ho = hist_off;
    if constexpr (PLAN) {  // nb < kPlanLds: the plan in LDS, published by workgroup 0
        hash_plan_block(prs, nb, hts, chunk, s_plan, s_plan + kPlanLds);
        if (blockIdx.x == 0)
            for (int i = threadIdx.x; i <= nb; i += 256) {
                chunk_start[i] = s_plan[i];
                hist_off[i] = s_plan[kPlanLds + i];
            }
        cs = s_plan;
        ho = s_plan + kPlanLds;
    }
    int b;
    int64_t c;
    if (!hash_chunk_of(cs, nb, b, c)) return;
    const int64_t* hist_off_ = ho;
    const uint32_t tsize = hts[b + 1] - hts[b];
    const uint32_t k64 = pow64_mod(tsize);
    for (uint32_t i = threadIdx.x; i < tsize; i += 256) h[i] = 0;
    __syncthreads();
    const int64_t p0 = prs[b] + c * chunk, p1 = min(prs[b + 1], p0 + chunk);
    // 8 points per thread loaded before any is binned and stored (clamped to
    // p0 < p1, unconditional): one point per iteration had each load wait for
    // the previous iteration's bins store (vmcnt counts stores)
    constexpr int U = 8;
    for (int64_t i0 = p0 + threadIdx.x; i0 < p1; i0 += 256 * U) {
        float px[U], py[U], pz[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + 256 * u;
            const int64_t j = i < p1 ? i : p0;
            px[u] = points[3 * j];
            py[u] = points[3 * j + 1];
            pz[u] = points[3 * j + 2];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + 256 * u;
            if (i < p1) {
                const uint32_t bin = point_bin_k(px[u], py[u], pz[u], inv, tsize, k64);
                bins[i] = bin;
                atomicAdd(&h[bin], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t* out = hist + hist_off_[b] + c * tsize;
    for (uint32_t i = threadIdx.x; i < tsize; i += 256) out[i] = h[i];
}

// Per (batch item, slice of 64 bins), 4 waves: every bin's column of chunk
// counts becomes each chunk's first slot of that bin relative to the bin's
// start inside the item (exclusive scan over the chunks: wave q scans a
// quarter of the chunks, the quarters' sums meet in LDS), and the bin's total
// goes to bin_tot — the scan over the bins is done by the scatter kernel.
// (One workgroup per item scanned the columns before: a single 65,536-point
// item of 64 chunks took 11 us in one workgroup.)
constexpr int kColBins = 64;
__global__ void __launch_bounds__(256) hash_hist_colscan_kernel(int nslices, const uint32_t* __restrict__ hts,
                                                                const int64_t* __restrict__ chunk_start,
                                                                const int64_t* __restrict__ hist_off,
                                                                uint32_t* __restrict__ hist,
                                                                uint32_t* __restrict__ bin_tot) {
    __shared__ uint32_t qsum[4][kColBins];
    const int b = blockIdx.x / nslices, s = blockIdx.x % nslices;
    const int q = wave_id(), lane = lane_id();
    const uint32_t first = hts[b], tsize = hts[b + 1] - first;
    const uint32_t bin = static_cast<uint32_t>(s * kColBins + lane);
    if (static_cast<uint32_t>(s * kColBins) >= tsize) return;  // whole workgroup
    const bool valid = bin < tsize;
    const int64_t nchunks = chunk_start[b + 1] - chunk_start[b];
    const int64_t c0 = nchunks * q / 4, c1 = nchunks * (q + 1) / 4;
    uint32_t* H = hist + hist_off[b] + bin;
    uint32_t sum = 0;
    if (valid) {
        int64_t cc = c0;
        for (; cc + 8 <= c1; cc += 8) {  // independent loads in flight
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = H[(cc + u) * tsize];
            sum += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
        }
        for (; cc < c1; ++cc) sum += H[cc * tsize];
    }
    qsum[q][lane] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int k = 0; k < q; ++k) run += qsum[k][lane];
    if (valid) {
        if (q == 3) bin_tot[first + bin] = run + sum;
        int64_t cc = c0;
        for (; cc + 8 <= c1; cc += 8) {  // 8 loads in flight, then the 8 bases
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = H[(cc + u) * tsize];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                H[(cc + u) * tsize] = run;
                run += v[u];
            }
        }
        for (; cc < c1; ++cc) {
            const uint32_t v = H[cc * tsize];
            H[cc * tsize] = run;
            run += v;
        }
    }
}

// Per chunk: ranks the chunk's points stably and writes their ids; the chunk's
// first slot per bin = the bin's start inside the item (exclusive scan of the
// item's bin totals, done here in LDS; chunk 0 also writes the item's
// cell_splits) + the chunk's offset from hash_hist_colscan_kernel.
// NWV waves per chunk (4, or 8: half the rows per wave, so half the
// ranking chain per wave for the same chunk)
template <int CHUNK, int NWV = kHashWaves>
__global__ void __launch_bounds__(NWV * 64) hash_chunk_scatter_kernel(int nb, const int64_t* __restrict__ prs,
                                                                 const uint32_t* __restrict__ hts,
                                                                 const int64_t* __restrict__ chunk_start,
                                                                 const int64_t* __restrict__ hist_off,
                                                                 const uint32_t* __restrict__ bins,
                                                                 const uint32_t* __restrict__ hist,
                                                                 const uint32_t* __restrict__ bin_tot,
                                                                 uint32_t* __restrict__ cell_splits,
                                                                 uint32_t* __restrict__ hti, int max_bins) {
    constexpr int kRows = CHUNK / 64 / NWV;  // rows of 64 per wave
    // [NWV][max_bins]: counts, then bases; then [max_bins] bin starts
    extern __shared__ uint32_t wc_all[];
    __shared__ uint32_t wsum[NWV];
    int b;
    int64_t c;
    if (!hash_chunk_of(chunk_start, nb, b, c)) return;
    const int t = threadIdx.x, w = wave_id(), lane = lane_id();
    const uint32_t first = hts[b], tsize = hts[b + 1] - first;
    const int64_t item0 = prs[b], item_end = prs[b + 1];
    const uint32_t* base = hist + hist_off[b] + c * tsize;
    uint32_t* wc = wc_all + w * max_bins;
    uint32_t* bstart = wc_all + NWV * max_bins;
    for (uint32_t i = t; i < tsize; i += NWV * 64)
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) wc_all[ww * max_bins + i] = 0;
    {  // bin starts: exclusive scan of the item's bin totals, (NWV * 64)-bin rounds
        uint32_t carry = 0;
        for (uint32_t b0 = 0; b0 < tsize; b0 += NWV * 64) {
            const uint32_t i = b0 + t;
            const uint32_t v = i < tsize ? bin_tot[first + i] : 0u;
            const uint32_t inc = wave_inclusive_scan(v);
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t st = carry + inc - v, all = 0;
#pragma unroll
            for (int ww = 0; ww < NWV; ++ww) {
                st += ww < w ? wsum[ww] : 0u;
                all += wsum[ww];
            }
            if (i < tsize) {
                bstart[i] = st;
                if (c == 0) cell_splits[first + i] = static_cast<uint32_t>(item0 + st);
            }
            carry += all;
            __syncthreads();
        }
        if (c == 0 && b == nb - 1 && t == 0) cell_splits[first + tsize] = static_cast<uint32_t>(prs[nb]);
    }
    __syncthreads();  // the zeroed counts (tsize >= 1: the loop above has barriers too)
    // each wave ranks its contiguous rows in order (peers = same bin, found
    // with one ballot per bin bit), running per-bin counts in LDS — LDS
    // operations of one wave execute in order, no barrier between rows
    const int64_t p0 = item0 + c * CHUNK;
    const int64_t pend = min(item_end, p0 + CHUNK);
    const int nbits = tsize > 1 ? 32 - __builtin_clz(tsize - 1) : 0;
    const uint64_t lt = lanemask_lt();
    uint32_t dig[kRows], loff[kRows];
    // every row's bin loaded up front (clamped to p0 < pend, unconditional):
    // a load under `valid` compiled to one wait per row
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int64_t i = p0 + (static_cast<int64_t>(w) * kRows + r) * 64 + lane;
        dig[r] = bins[i < pend ? i : p0];
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int64_t i = p0 + (static_cast<int64_t>(w) * kRows + r) * 64 + lane;
        const bool valid = i < pend;
        const uint32_t d = valid ? dig[r] : 0u;
        dig[r] = d;
        uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
        for (int bit = 0; bit < nbits; ++bit) {
            const bool on = (d >> bit) & 1u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(on);
            peers &= on ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t before = valid ? wc[d] : 0u;
        loff[r] = before + rank;
        if (valid && rank == 0) wc[d] = before + static_cast<uint32_t>(__popcll(peers));
    }
    __syncthreads();
    // per-wave bases: chunk base + counts of the earlier waves (stable)
    for (uint32_t i = t; i < tsize; i += NWV * 64) {
        uint32_t a = bstart[i] + base[i];
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) {
            const uint32_t cw = wc_all[ww * max_bins + i];
            wc_all[ww * max_bins + i] = a;
            a += cw;
        }
    }
    __syncthreads();
    // ids to their slots (scattered inside the item's range)
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int64_t i = p0 + (static_cast<int64_t>(w) * kRows + r) * 64 + lane;
        if (i < pend) hti[item0 + wc[dig[r]] + loff[r]] = static_cast<uint32_t>(i);
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
    // radix path: bins + sorted keys + sort scratch; small-table path: bins,
    // chunk histograms (<= n_points + total_bins entries when every table has
    // <= kSmallTable bins: sum_b chunks_b T_b <= sum_b (N_b / chunk + 1) T_b)
    // and the plan — the larger of the two
    const size_t radix = ws_bytes<uint32_t>(n_points) * 2 + prim::radix_sort_workspace_bytes<uint32_t>(n_points);
    // chunks of 1024 (small calls): sum_b (N_b / 1024 + 1) T_b <= 4 N + T
    const int64_t nb_ub = total_bins;  // every batch item has >= 1 bin
    const int64_t hist_ub = 4 * n_points + total_bins;  // chunks of 1024 at most 4x the 4096 ones
    const size_t small = ws_bytes<uint32_t>(n_points) + ws_bytes<uint32_t>(hist_ub) +
                         ws_bytes<uint32_t>(total_bins) + 2 * ws_bytes<int64_t>(nb_ub + 1);
    return std::max(radix, small);
}

O3DML_API int o3dml_build_spatial_hash_table(const float* points, int64_t n_points, float radius, int64_t n_batch,
                                             const int64_t* points_row_splits, const uint32_t* hash_table_splits,
                                             const uint32_t* hash_table_splits_host, int64_t total_bins,
                                             uint32_t* hash_table_index, uint32_t* hash_table_cell_splits,
                                             void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(radius > 0.f, "radius must be > 0");
    O3DML_REQUIRE(n_batch >= 1, "need at least one batch item");
    O3DML_REQUIRE(total_bins >= n_batch && total_bins < (int64_t(1) << 32), "invalid hash table size %lld",
                  (long long)total_bins);
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const float inv = 1.0f / (2.0f * radius);
    bool small = hash_table_splits_host != nullptr && n_points > 0;
    uint32_t max_bins = 1;
    for (int64_t b = 0; small && b < n_batch; ++b) {
        const uint32_t tb = hash_table_splits_host[b + 1] - hash_table_splits_host[b];
        max_bins = std::max(max_bins, tb);
        small = tb <= static_cast<uint32_t>(kSmallTable);
    }
    if (small) {
        uint32_t* bins = ws.take<uint32_t>(n_points);
        // small calls (fewer than 512 chunks of 4096) take chunks of 1024;
        // O3DML_HASH_CHUNK (1024, 2048, 4096) forces one size (A/B)
        static const int forced = [] {
            const char* e = std::getenv("O3DML_HASH_CHUNK");
            const int v = e ? std::atoi(e) : 0;
            return (v == 1024 || v == 2048 || v == 4096) ? v : 0;
        }();
        const int chunk = forced ? forced : (ceil_div(n_points, kHashChunk) < 512 ? kHashChunkSmall : kHashChunk);
        uint32_t* hist = ws.take<uint32_t>((kHashChunk / chunk) * n_points + total_bins);
        uint32_t* bin_tot = ws.take<uint32_t>(total_bins);
        int64_t* chunk_start = ws.take<int64_t>(n_batch + 1);
        int64_t* hist_off = ws.take<int64_t>(n_batch + 1);
        const unsigned grid = static_cast<unsigned>(ceil_div(n_points, chunk) + n_batch);  // >= chunk count
        if (n_batch < kPlanLds) {  // the plan inside the histogram kernel
            hash_chunk_hist_kernel<true><<<grid, 256, sizeof(uint32_t) * max_bins, st>>>(
                    points, inv, (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins,
                    hist, chunk);
        } else {
            hash_plan_kernel<<<1, 256, 0, st>>>(points_row_splits, (int)n_batch, hash_table_splits, chunk_start,
                                                hist_off, chunk);
            O3DML_LAUNCH_CHECK();
            hash_chunk_hist_kernel<false><<<grid, 256, sizeof(uint32_t) * max_bins, st>>>(
                    points, inv, (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins,
                    hist, chunk);
        }
        O3DML_LAUNCH_CHECK();
        const int nslices = static_cast<int>(ceil_div(max_bins, kColBins));
        hash_hist_colscan_kernel<<<static_cast<unsigned>(n_batch * nslices), 256, 0, st>>>(
                nslices, hash_table_splits, chunk_start, hist_off, hist, bin_tot);
        O3DML_LAUNCH_CHECK();
        const size_t lds = sizeof(uint32_t) * (kHashWaves + 1) * max_bins;
        // 8 waves per 4,096-point chunk (O3DML_HASH_WAVES=8) while their LDS fits 64 KiB
        static const int hw = [] {
            const char* e = std::getenv("O3DML_HASH_WAVES");
            return e ? std::atoi(e) : 4;
        }();
        const size_t lds8 = sizeof(uint32_t) * 9 * max_bins;
        if (chunk == kHashChunkSmall)
            hash_chunk_scatter_kernel<kHashChunkSmall><<<grid, 256, lds, st>>>(
                    (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins, hist, bin_tot,
                    hash_table_cell_splits, hash_table_index, static_cast<int>(max_bins));
        else if (chunk == 2048)
            hash_chunk_scatter_kernel<2048><<<grid, 256, lds, st>>>(
                    (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins, hist, bin_tot,
                    hash_table_cell_splits, hash_table_index, static_cast<int>(max_bins));
        else if (hw == 8 && lds8 <= 65536)
            hash_chunk_scatter_kernel<kHashChunk, 8><<<grid, 512, lds8, st>>>(
                    (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins, hist, bin_tot,
                    hash_table_cell_splits, hash_table_index, static_cast<int>(max_bins));
        else
            hash_chunk_scatter_kernel<kHashChunk><<<grid, 256, lds, st>>>(
                    (int)n_batch, points_row_splits, hash_table_splits, chunk_start, hist_off, bins, hist, bin_tot,
                    hash_table_cell_splits, hash_table_index, static_cast<int>(max_bins));
        O3DML_LAUNCH_CHECK();
        return 0;
    }
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
