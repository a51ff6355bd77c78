// nns_knn.hip — exact k-nearest-neighbour search (Open3D ops.knn_search /
// layers.KNNSearch and core.nns.NearestNeighborSearch.knn_search; reference
// callers ml3d/datasets/utils/dataprocessing.py:87-103 <- randlanet.py:218-229,
// point_transformer.py:724-729).
//
// k <= 64: dense per-batch grid (grid.hpp, ~k/2 points per cell); one lane per
// query walks Chebyshev rings of cells around its cell, keeping the k best
// (distance, id) pairs sorted in registers, and stops once the k-th distance
// is strictly below a conservative lower bound on every unvisited point.
// Queries are processed in cell order (self search: the grid order itself),
// so the lanes of a wave scan overlapping cells through L1/L2.
// k > 64 (the sampler's single-centre patch crop): all distances
// of the query's batch item + stable radix sort on the distance bits.
// Result order per query: ascending (distance, index) — exact ties by index.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "grid.hpp"

namespace o3dml {

__device__ __forceinline__ bool lex_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && ia < ib);
}

// (distance, index) as one 64-bit key: distances are >= +0 (squared L2, L1,
// Linf of fabsf terms), whose float bits order as unsigned ints, so the
// lexicographic (distance, index) order is the unsigned order of
// (bits(d) << 32 | index) — one 64-bit compare instead of three float/int
// compares, one 64-bit select per move.  NaN distances (bits above +inf) sort
// after every finite one and after the empty entry's +inf, as lex_less never
// admits them either.
__device__ __forceinline__ uint64_t knn_key(float d, uint32_t id) {
    return (static_cast<uint64_t>(__float_as_uint(d)) << 32) | id;
}
constexpr uint64_t kKnnEmpty = (static_cast<uint64_t>(0x7f800000u) << 32) | 0xffffffffull;  // (+inf, ~0)

template <int K, int METRIC, bool IGNORE>
__global__ void __launch_bounds__(256) knn_grid_kernel(const float4* __restrict__ sorted, const uint32_t* __restrict__ splits,
                                                       const GridBatch* __restrict__ grids, const float* __restrict__ queries,
                                                       int64_t m, const uint32_t* __restrict__ qorder,
                                                       const int64_t* __restrict__ qrs, int nb, int k,
                                                       int32_t* __restrict__ out_idx, float* __restrict__ out_dist,
                                                       int64_t* __restrict__ counts) {
    for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < m;
         t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = qorder ? static_cast<int64_t>(qorder[t]) : t;
        const GridBatch g = grids[batch_of(q, qrs, nb)];
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        const int cx = grid_axis(qx, g.ox, g.inv_h, g.dx);
        const int cy = grid_axis(qy, g.oy, g.inv_h, g.dy);
        const int cz = grid_axis(qz, g.oz, g.inv_h, g.dz);
        uint64_t bk[K];  // sorted top-K keys (knn_key)
#pragma unroll
        for (int j = 0; j < K; ++j) bk[j] = kKnnEmpty;
        uint64_t kk = kKnnEmpty;
        int cnt = 0;
        auto consider = [&](const float4& p) {
            if (IGNORE && p.x == qx && p.y == qy && p.z == qz) return;
            const float d = dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz);
            const uint64_t key = knn_key(d, __float_as_uint(p.w));
            if (!(key < kk)) return;
            ++cnt;
#pragma unroll
            for (int r = K - 1; r >= 0; --r) {
                const bool lt_prev = r > 0 && key < bk[r > 0 ? r - 1 : 0];
                const bool lt_cur = key < bk[r];
                bk[r] = lt_prev ? bk[r > 0 ? r - 1 : 0] : (lt_cur ? key : bk[r]);
            }
            if (cnt >= k) {
#pragma unroll
                for (int r = 0; r < K; ++r)
                    if (r == k - 1) kk = bk[r];
            }
        };
        auto visit = [&](int xa, int xb, int y, int z) {  // cells xa..xb of a row: one contiguous run
            const uint32_t c = g.offset + static_cast<uint32_t>(g.dx * (y + g.dy * z));
            const uint32_t s = splits[c + xa], e = splits[c + xb + 1];
            uint32_t j = s;
            for (; j + 8 <= e; j += 8) {  // 8 loads in flight per lane
                float4 p[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) p[u] = sorted[j + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) consider(p[u]);
            }
            for (; j < e; ++j) consider(sorted[j]);
        };
        for (int R = 0;; ++R) {
            const int x0 = cx - R, x1 = cx + R, y0 = cy - R, y1 = cy + R, z0 = cz - R, z1 = cz + R;
            const int za = max(z0, 0), zb = min(z1, g.dz - 1);
            const int ya = max(y0, 0), yb = min(y1, g.dy - 1);
            const int xa = max(x0, 0), xb = min(x1, g.dx - 1);
            for (int z = za; z <= zb; ++z) {
                for (int y = ya; y <= yb; ++y) {
                    if (z == z0 || z == z1 || y == y0 || y == y1) {
                        visit(xa, xb, y, z);
                    } else {
                        if (x0 >= 0) visit(x0, x0, y, z);
                        if (x1 < g.dx) visit(x1, x1, y, z);
                    }
                }
            }
            const bool lo_x = x0 <= 0, hi_x = x1 >= g.dx - 1, lo_y = y0 <= 0, hi_y = y1 >= g.dy - 1;
            const bool lo_z = z0 <= 0, hi_z = z1 >= g.dz - 1;
            if (lo_x && hi_x && lo_y && hi_y && lo_z && hi_z) break;  // every cell visited
            if (cnt >= k) {
                // distance from q to the unvisited region (faces not on the grid boundary)
                float lb = INFINITY;
                if (!lo_x) lb = fminf(lb, qx - (g.ox + static_cast<float>(x0) * g.h));
                if (!hi_x) lb = fminf(lb, (g.ox + static_cast<float>(x1 + 1) * g.h) - qx);
                if (!lo_y) lb = fminf(lb, qy - (g.oy + static_cast<float>(y0) * g.h));
                if (!hi_y) lb = fminf(lb, (g.oy + static_cast<float>(y1 + 1) * g.h) - qy);
                if (!lo_z) lb = fminf(lb, qz - (g.oz + static_cast<float>(z0) * g.h));
                if (!hi_z) lb = fminf(lb, (g.oz + static_cast<float>(z1 + 1) * g.h) - qz);
                // conservative against float cell-assignment rounding
                lb = lb - 1e-3f * g.h - 1e-6f * (fabsf(qx) + fabsf(qy) + fabsf(qz));
                if (lb > 0.f) {
                    const float bound = METRIC == kL2 ? lb * lb : lb;
                    if (__uint_as_float(static_cast<uint32_t>(kk >> 32)) < bound) break;
                }
            }
        }
        const int c = cnt < k ? cnt : k;
        counts[q] = c;
        int32_t* oi = out_idx + q * static_cast<int64_t>(k);
        float* od = out_dist + q * static_cast<int64_t>(k);
#pragma unroll
        for (int r = 0; r < K; ++r) {
            if (r < c) {
                oi[r] = static_cast<int32_t>(static_cast<uint32_t>(bk[r]));
                od[r] = __uint_as_float(static_cast<uint32_t>(bk[r] >> 32));
            }
        }
    }
}


// ---------------------------------------------------------------------------
// k <= 16: G lanes per query (64 / G queries per wave; G = 8 by default,
// O3DML_KNN_G = 4 / 8 / 16).  A lane-per-query walk leaves the chip nearly
// idle on the sizes RandLA-Net searches (60 k queries = < 1 wave per SIMD,
// each lane a chain of dependent loads); here the group walks the same rings
// together, lanes taking every G-th point of each cell into their own sorted
// top-K.  After each ring the group merges its lists with a butterfly: per
// round a lane takes the K smallest of its list and its partner's as
// min(a[i], b[K-1-i]) — a bitonic sequence — and sorts it with a register
// bitonic network; after the last round every lane holds the group's exact
// top-K, whose k-th entry both prunes the next ring and decides termination.
// Lane 0 keeps the merged list, the others restart empty, so no entry is
// counted twice.  Order: (distance, index) ascending.
//
// Keys as doubles (O3DML_KNN_F64, default): the 64-bit key (bits(d) << 32 |
// index) of a distance d >= +0 whose bits are clamped to <= 0x7FC00000 (every
// NaN becomes the canonical one, which still sorts after +inf and the empty
// entry) is, read as an IEEE double, a finite non-negative double whose order
// is the key's unsigned order (exponent field <= 0x7FC, never 0x7FF; f64
// denormals are kept: the kernel's f64 denormal mode is IEEE).  So a
// compare-exchange is v_min_f64 + v_max_f64 — no VOPC into an SGPR mask (a
// 4-cycle issue, then a hazard nop before the v_cndmask pair that reads it) —
// and an insertion is branch-free in the list:
//   new[0] = min(key, old[0]),  new[r] = min(max(key, old[r-1]), old[r]),
// every position from the old list at once (no carried chain).  The butterfly
// partners are DPP lane moves (quad_perm 1,0,3,2 / 2,3,0,1, row_half_mirror,
// row_mirror: partner i^1, i^2, 7-i, 15-i — each pairs the two halves of the
// next larger group, which is all a butterfly needs) instead of ds_bpermute.
// ---------------------------------------------------------------------------
#ifndef O3DML_KNN_F64
#define O3DML_KNN_F64 1
#endif

struct KnnKey {
#if O3DML_KNN_F64
    double v;
    __device__ __forceinline__ static KnnKey from_bits(uint64_t b) { return {__builtin_bit_cast(double, b)}; }
    __device__ __forceinline__ uint64_t bits() const { return __builtin_bit_cast(uint64_t, v); }
    // plain v_min_f64 / v_max_f64: fmin / fmax would first canonicalise both
    // operands (one v_max_f64 x, x each: the signalling-NaN rule), and these
    // keys are never NaN
    __device__ __forceinline__ friend KnnKey kmin(KnnKey a, KnnKey b) {
        double r;
        asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a.v), "v"(b.v));
        return {r};
    }
    __device__ __forceinline__ friend KnnKey kmax(KnnKey a, KnnKey b) {
        double r;
        asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a.v), "v"(b.v));
        return {r};
    }
    __device__ __forceinline__ friend bool operator<(KnnKey a, KnnKey b) { return a.v < b.v; }
#else
    uint64_t v;
    __device__ __forceinline__ static KnnKey from_bits(uint64_t b) { return {b}; }
    __device__ __forceinline__ uint64_t bits() const { return v; }
    __device__ __forceinline__ friend KnnKey kmin(KnnKey a, KnnKey b) { return {b.v < a.v ? b.v : a.v}; }
    __device__ __forceinline__ friend KnnKey kmax(KnnKey a, KnnKey b) { return {b.v < a.v ? a.v : b.v}; }
    __device__ __forceinline__ friend bool operator<(KnnKey a, KnnKey b) { return a.v < b.v; }
#endif
};

__device__ __forceinline__ KnnKey knn_key_g(float d, uint32_t id) {
    const uint32_t db = min(__float_as_uint(d), 0x7fc00000u);  // every NaN -> the canonical one (see above)
    return KnnKey::from_bits((static_cast<uint64_t>(db) << 32) | id);
}

// partner of round `round` of the butterfly (see above), as a DPP control
template <int ROUND>
__device__ __forceinline__ uint32_t dpp_partner(uint32_t v) {
    constexpr int ctrl = ROUND == 0 ? 0xB1 : ROUND == 1 ? 0x4E : ROUND == 2 ? 0x141 : 0x140;
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), ctrl, 0xF, 0xF, false));
}

template <int ROUND>
__device__ __forceinline__ KnnKey dpp_partner_key(KnnKey k) {
    const uint64_t b = k.bits();
    const uint32_t lo = dpp_partner<ROUND>(static_cast<uint32_t>(b));
    const uint32_t hi = dpp_partner<ROUND>(static_cast<uint32_t>(b >> 32));
    return KnnKey::from_bits((static_cast<uint64_t>(hi) << 32) | lo);
}

template <int K>
__device__ __forceinline__ void cas_kkey(KnnKey (&a)[K], int i, int j) {
    const KnnKey lo = kmin(a[i], a[j]), hi = kmax(a[i], a[j]);
    a[i] = lo;
    a[j] = hi;
}

template <int K, int G, int ROUND = 0>
__device__ __forceinline__ void group_merge_g(KnnKey (&a)[K]) {
    if constexpr ((1 << ROUND) < G) {
        // a[i] = min(a[i], partner[K-1-i]): the K smallest of both lists,
        // bitonic; in place, pair (i, K-1-i) at a time (both partner entries
        // fetched before either is overwritten)
#pragma unroll
        for (int i = 0; i < K / 2; ++i) {
            const KnnKey p_hi = dpp_partner_key<ROUND>(a[K - 1 - i]);
            const KnnKey p_lo = dpp_partner_key<ROUND>(a[i]);
            a[i] = kmin(a[i], p_hi);
            a[K - 1 - i] = kmin(a[K - 1 - i], p_lo);
        }
        if constexpr (K == 1) a[0] = kmin(a[0], dpp_partner_key<ROUND>(a[0]));
#pragma unroll
        for (int st = K / 2; st >= 1; st >>= 1) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if ((i & st) == 0) cas_kkey<K>(a, i, i + st);
        }
        group_merge_g<K, G, ROUND + 1>(a);
    }
}

template <int G, int ROUND = 0>
__device__ __forceinline__ uint32_t group_sum_g(uint32_t v) {
    if constexpr ((1 << ROUND) < G) return group_sum_g<G, ROUND + 1>(v + dpp_partner<ROUND>(v));
    return v;
}

// waves per SIMD asked of the register allocator (A/B builds; 0 = the
// compiler's choice: 89 VGPRs -> 5 waves)
#ifndef O3DML_KNN_WAVES
#define O3DML_KNN_WAVES 0
#endif
#if O3DML_KNN_WAVES
#define O3DML_KNN_ATTR __attribute__((amdgpu_waves_per_eu(O3DML_KNN_WAVES, 8)))
#else
#define O3DML_KNN_ATTR
#endif
template <int K, int G, int METRIC, bool IGNORE>
__global__ void __launch_bounds__(256) O3DML_KNN_ATTR knn_group_kernel(const float4* __restrict__ sorted,
                                                        const uint32_t* __restrict__ splits,
                                                        const GridBatch* __restrict__ grids,
                                                        const float* __restrict__ queries, int64_t m,
                                                        const uint32_t* __restrict__ qorder,
                                                        const int64_t* __restrict__ qrs, int nb, int k,
                                                        int32_t* __restrict__ out_idx, float* __restrict__ out_dist,
                                                        int64_t* __restrict__ counts) {
    static_assert(G == 4 || G == 8 || G == 16, "group of 4, 8 or 16 lanes (DPP partners within a row)");
    const int gl = threadIdx.x & (G - 1);
    const KnnKey empty = KnnKey::from_bits(kKnnEmpty);
    const int64_t groups = static_cast<int64_t>(gridDim.x) * (blockDim.x / G);
    for (int64_t t = (blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x) / G; t < m + 0;
         t += groups) {
        const int64_t q = qorder ? static_cast<int64_t>(qorder[t]) : t;
        const GridBatch g = grids[batch_of(q, qrs, nb)];
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        const int cx = grid_axis(qx, g.ox, g.inv_h, g.dx);
        const int cy = grid_axis(qy, g.oy, g.inv_h, g.dy);
        const int cz = grid_axis(qz, g.oz, g.inv_h, g.dz);
        KnnKey bk[K];  // this lane's sorted top-K keys
#pragma unroll
        for (int j = 0; j < K; ++j) bk[j] = empty;
        KnnKey kk = empty;  // group k-th best after the last merge (pruning bound)
        KnnKey thr = empty;  // min(kk, bk[K-1]): a candidate enters only below it
        bool full = false;
        auto consider = [&](const float4& p) {
            if (IGNORE && p.x == qx && p.y == qy && p.z == qz) return;
            const float d = dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz);
            const KnnKey key = knn_key_g(d, __float_as_uint(p.w));
            if (!(key < thr)) return;
            // branch-free insertion, every position from the old list; in
            // place from the top (position r reads old r - 1 and old r)
#pragma unroll
            for (int r = K - 1; r >= 1; --r) bk[r] = kmin(kmax(key, bk[r - 1]), bk[r]);
            bk[0] = kmin(key, bk[0]);
            thr = kmin(kk, bk[K - 1]);
        };
        // cells xa..xb of one (y, z) row are adjacent in the cell order (x
        // fastest), so their points are one contiguous run of `sorted`: one
        // pair of split loads and one stream per run instead of per cell (the
        // chain of dependent split -> point loads per cell bounded this kernel)
        auto visit = [&](int xa, int xb, int y, int z) {
            const uint32_t c = g.offset + static_cast<uint32_t>(g.dx * (y + g.dy * z));
            const uint32_t s = splits[c + xa], e = splits[c + xb + 1];
            uint32_t j = s + gl;
            for (; j + G < e; j += 2 * G) {  // two loads in flight per lane
                const float4 p0 = sorted[j], p1 = sorted[j + G];
                consider(p0);
                consider(p1);
            }
            if (j < e) consider(sorted[j]);
        };
        for (int R = 0;; ++R) {
            const int x0 = cx - R, x1 = cx + R, y0 = cy - R, y1 = cy + R, z0 = cz - R, z1 = cz + R;
            const int za = max(z0, 0), zb = min(z1, g.dz - 1);
            const int ya = max(y0, 0), yb = min(y1, g.dy - 1);
            const int xa = max(x0, 0), xb = min(x1, g.dx - 1);
            for (int z = za; z <= zb; ++z) {
                for (int y = ya; y <= yb; ++y) {
                    if (z == z0 || z == z1 || y == y0 || y == y1) {
                        visit(xa, xb, y, z);
                    } else {
                        if (x0 >= 0) visit(x0, x0, y, z);
                        if (x1 < g.dx) visit(x1, x1, y, z);
                    }
                }
            }
            // merging only pays once the group holds k candidates (it can then
            // prune and terminate); before that the lists keep accumulating
            uint32_t have = 0;
#pragma unroll
            for (int r = 0; r < K; ++r) have += static_cast<uint32_t>(bk[r].bits()) != 0xffffffffu ? 1u : 0u;
            have = group_sum_g<G>(have);
            const bool last_ring = x0 <= 0 && x1 >= g.dx - 1 && y0 <= 0 && y1 >= g.dy - 1 && z0 <= 0 &&
                                   z1 >= g.dz - 1;
            if (have < static_cast<uint32_t>(k) && !last_ring) continue;
            group_merge_g<K, G>(bk);
#pragma unroll
            for (int r = 0; r < K; ++r)
                if (r == k - 1) kk = bk[r];
            full = static_cast<uint32_t>(kk.bits()) != 0xffffffffu;
            const float kd = __uint_as_float(static_cast<uint32_t>(kk.bits() >> 32));
            const bool lo_x = x0 <= 0, hi_x = x1 >= g.dx - 1, lo_y = y0 <= 0, hi_y = y1 >= g.dy - 1;
            const bool lo_z = z0 <= 0, hi_z = z1 >= g.dz - 1;
            if (lo_x && hi_x && lo_y && hi_y && lo_z && hi_z) break;  // every cell visited
            if (full) {
                float lb = INFINITY;
                if (!lo_x) lb = fminf(lb, qx - (g.ox + static_cast<float>(x0) * g.h));
                if (!hi_x) lb = fminf(lb, (g.ox + static_cast<float>(x1 + 1) * g.h) - qx);
                if (!lo_y) lb = fminf(lb, qy - (g.oy + static_cast<float>(y0) * g.h));
                if (!hi_y) lb = fminf(lb, (g.oy + static_cast<float>(y1 + 1) * g.h) - qy);
                if (!lo_z) lb = fminf(lb, qz - (g.oz + static_cast<float>(z0) * g.h));
                if (!hi_z) lb = fminf(lb, (g.oz + static_cast<float>(z1 + 1) * g.h) - qz);
                lb = lb - 1e-3f * g.h - 1e-6f * (fabsf(qx) + fabsf(qy) + fabsf(qz));
                if (lb > 0.f) {
                    const float bound = METRIC == kL2 ? lb * lb : lb;
                    if (kd < bound) break;
                }
            }
            if (gl != 0) {  // lane 0 carries the merged list into the next ring
#pragma unroll
                for (int j = 0; j < K; ++j) bk[j] = empty;
            }
            thr = kmin(kk, bk[K - 1]);
        }
        int c = 0;
#pragma unroll
        for (int r = 0; r < K; ++r) c += (r < k && static_cast<uint32_t>(bk[r].bits()) != 0xffffffffu) ? 1 : 0;
        if (gl == 0) counts[q] = c;
        int32_t* oi = out_idx + q * static_cast<int64_t>(k);
        float* od = out_dist + q * static_cast<int64_t>(k);
#pragma unroll
        for (int r = 0; r < K; ++r) {
            if (r < c && (r & (G - 1)) == gl) {
                const uint64_t b = bk[r].bits();
                oi[r] = static_cast<int32_t>(static_cast<uint32_t>(b));
                od[r] = __uint_as_float(static_cast<uint32_t>(b >> 32));
            }
        }
    }
}

// lanes per query of the group kernel (A/B knob O3DML_KNN_G: 4, 8 or 16)
static int knn_group_lanes() {
    static const int g = [] {
        const char* e = std::getenv("O3DML_KNN_G");
        const int v = e ? std::atoi(e) : 8;
        return v == 4 || v == 16 ? v : 8;
    }();
    return g;
}

template <int K>
static void launch_knn_k(int metric, bool ignore, unsigned grid, hipStream_t st, const GridIndex& gi, const float* q,
                         int64_t m, const uint32_t* qorder, const int64_t* qrs, int nb, int k, int32_t* oi, float* od,
                         int64_t* counts) {
#define O3DML_KNN_G(M, I, G)                                                                                     \
    knn_group_kernel<K, G, M, I><<<stream_grid(m * G, 256, 1 << 20), 256, 0, st>>>(                              \
            gi.sorted, gi.splits, gi.params, q, m, qorder, qrs, nb, k, oi, od, counts)
#define O3DML_KNN(M, I)                                                                                          \
    do {                                                                                                         \
        if constexpr (K <= 16) {                                                                                 \
            const int G = knn_group_lanes();                                                                     \
            if (G == 4) O3DML_KNN_G(M, I, 4);                                                                    \
            else if (G == 16) O3DML_KNN_G(M, I, 16);                                                             \
            else O3DML_KNN_G(M, I, 8);                                                                           \
        } else                                                                                                   \
            knn_grid_kernel<K, M, I><<<grid, 256, 0, st>>>(gi.sorted, gi.splits, gi.params, q, m, qorder, qrs, nb, \
                                                           k, oi, od, counts);                                   \
    } while (0)
    if (metric == kL2) {
        if (ignore) O3DML_KNN(kL2, true); else O3DML_KNN(kL2, false);
    } else if (metric == kL1) {
        if (ignore) O3DML_KNN(kL1, true); else O3DML_KNN(kL1, false);
    } else {
        if (ignore) O3DML_KNN(kLinf, true); else O3DML_KNN(kLinf, false);
    }
#undef O3DML_KNN
#undef O3DML_KNN_G
    O3DML_LAUNCH_CHECK();
}

__global__ void compact_rows_kernel(const int32_t* __restrict__ si, const float* __restrict__ sd, int64_t m, int k,
                                    const int64_t* __restrict__ rs, int bits, void* __restrict__ out_idx,
                                    float* __restrict__ out_dist) {
    const int64_t total = m * k;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = e / k;
        const int64_t j = e - q * k;
        const int64_t s = rs[q];
        if (s + j < rs[q + 1]) {
            if (bits == 32)
                static_cast<int32_t*>(out_idx)[s + j] = si[e];
            else
                static_cast<int64_t*>(out_idx)[s + j] = si[e];
            if (out_dist) out_dist[s + j] = sd[e];
        }
    }
}

// ---- k > kManyKnnMaxK (and the overflow queries of nns_many.hip): one query
// at a time, every distance of its batch item + a stable radix sort ----
__global__ void bigk_counts_kernel(const int64_t* __restrict__ prs, const int64_t* __restrict__ qrs, int nb,
                                   int64_t m, int64_t k, int64_t* __restrict__ counts) {
    for (int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; q < m;
         q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(q, qrs, nb);
        const int64_t nbp = prs[b + 1] - prs[b];
        counts[q] = nbp < k ? nbp : k;
    }
}

// ignore_query_point: min(k, N_b - points at the query's exact position), one
// workgroup per query over its batch item
__global__ void __launch_bounds__(256) bigk_counts_ignore_kernel(const float* __restrict__ pts,
                                                                 const float* __restrict__ queries,
                                                                 const int64_t* __restrict__ prs,
                                                                 const int64_t* __restrict__ qrs, int nb, int64_t m,
                                                                 int64_t k, int64_t* __restrict__ counts) {
    __shared__ uint32_t s_same;
    for (int64_t q = blockIdx.x; q < m; q += gridDim.x) {
        if (threadIdx.x == 0) s_same = 0;
        __syncthreads();
        const int b = batch_of(q, qrs, nb);
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        uint32_t same = 0;
        for (int64_t i = prs[b] + threadIdx.x; i < prs[b + 1]; i += blockDim.x)
            same += (pts[3 * i] == qx && pts[3 * i + 1] == qy && pts[3 * i + 2] == qz) ? 1u : 0u;
        same = wave_sum(same);
        if ((threadIdx.x & 63) == 0 && same) atomicAdd(&s_same, same);
        __syncthreads();
        if (threadIdx.x == 0) {
            const int64_t n = prs[b + 1] - prs[b] - s_same;
            counts[q] = n < k ? n : k;
        }
        __syncthreads();
    }
}

// nns_many.hip: batched 64 < k <= kManyKnnMaxK
constexpr int64_t kManyKnnMaxK = 2048;
size_t knn_many_workspace_bytes(int64_t n, int64_t m, int64_t k, int64_t nb);
void knn_many_count(const float* pts, int64_t n, const float* queries, int64_t m, int64_t k, int nb,
                    const int64_t* prs, const int64_t* qrs, int ignore, int64_t* rs, Workspace ws, hipStream_t st);
void knn_many_fill(const float* pts, int64_t n, const float* queries, int64_t m, int64_t k, int nb,
                   const int64_t* qrs, int metric, int ignore, const int64_t* rs, int bits, void* oi, float* od,
                   Workspace ws, hipStream_t st);
// nns_topk.hip: k > kManyKnnMaxK, one query by radix selection + a sort of the k selected
size_t topk_bigk_workspace_bytes(int64_t n_points, int64_t k);
void topk_bigk_one(const float* pts, int64_t ps, int64_t pn, const float* queries, int64_t q, int64_t k,
                   int metric, int ignore, const int64_t* rs, int bits, void* oi, float* od, Workspace ws,
                   hipStream_t st);

}  // namespace o3dml

using namespace o3dml;

static int knn_bucket(int64_t k) {
    if (k <= 1) return 1;
    if (k <= 4) return 4;
    if (k <= 8) return 8;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    if (k <= 64) return 64;
    return 0;
}

// cells per point at most (grid_cells_cap): O3DML_KNN_CAP (A/B), default 2
static double knn_cap_factor() {
    static const double v = [] {
        const char* e = std::getenv("O3DML_KNN_CAP");
        const double x = e ? std::atof(e) : 2.0;
        return x > 0.0 ? x : 2.0;
    }();
    return v;
}
// points per cell of the uniform-fill grid plan = max(min_target, k * factor)
static double knn_target_factor() {
    const char* e = std::getenv("O3DML_KNN_TARGET");
    return e ? std::atof(e) : 0.25;  // ~4 points per cell: measured best on RandLA patches
}
static double knn_min_target() {
    const char* e = std::getenv("O3DML_KNN_MIN_TARGET");
    return e ? std::atof(e) : 2.0;
}

O3DML_API size_t o3dml_knn_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t k, int64_t n_batch) {
    if (knn_bucket(k) == 0) {
        if (k <= kManyKnnMaxK) return knn_many_workspace_bytes(n_points, n_queries, k, n_batch);
        return std::max(topk_bigk_workspace_bytes(n_points, k),
                        ws_bytes<int64_t>(n_queries) + prim::scan_workspace_bytes(n_queries));
    }
    return grid_workspace_bytes(n_points, static_cast<int>(n_batch), knn_cap_factor()) +
           3 * ws_bytes<uint32_t>(n_queries) + prim::radix_sort_workspace_bytes<uint32_t>(n_queries) +
           ws_bytes<int32_t>(n_queries * k) + ws_bytes<float>(n_queries * k) + ws_bytes<int64_t>(n_queries) +
           prim::scan_workspace_bytes(n_queries);
}


// Phase 1: search; writes neighbors_row_splits [M+1] (device) and keeps the
// per-query results in the workspace for o3dml_knn_search_fill.
// Row-split arrays: *_host copies are needed to plan the grid.
O3DML_API int o3dml_knn_search_count(const float* points, int64_t n_points, const float* queries, int64_t n_queries,
                                     int64_t k, int64_t n_batch, const int64_t* points_row_splits,
                                     const int64_t* queries_row_splits, const int64_t* points_row_splits_host,
                                     const int64_t* queries_row_splits_host, int metric, int ignore_query_point,
                                     int self_search, int64_t* neighbors_row_splits, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k >= 1, "k must be >= 1");
    O3DML_REQUIRE(metric >= 0 && metric <= 2, "metric must be L1(0), L2(1) or Linf(2)");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    const int K = knn_bucket(k);
    if (K == 0) {
        // rows: min(k, eligible points) per query, on the device (no host round trip)
        (void)points_row_splits_host;
        (void)queries_row_splits_host;
        if (k <= kManyKnnMaxK) {  // batched (nns_many.hip): grid + eligible counts
            knn_many_count(points, n_points, queries, n_queries, k, nb, points_row_splits, queries_row_splits,
                           ignore_query_point, neighbors_row_splits, ws, st);
            return 0;
        }
        fill_async(neighbors_row_splits, 0, sizeof(int64_t), st);
        if (n_queries == 0) return 0;
        int64_t* cnt = ws.take<int64_t>(n_queries);
        if (ignore_query_point)
            bigk_counts_ignore_kernel<<<static_cast<unsigned>(std::min<int64_t>(n_queries, 1 << 16)), 256, 0, st>>>(
                    points, queries, points_row_splits, queries_row_splits, nb, n_queries, k, cnt);
        else
            bigk_counts_kernel<<<stream_grid(n_queries, 256), 256, 0, st>>>(points_row_splits, queries_row_splits,
                                                                           nb, n_queries, k, cnt);
        O3DML_LAUNCH_CHECK();
        prim::scan<int64_t, int64_t>(cnt, neighbors_row_splits + 1, n_queries, true, ws, st);
        return 0;
    }
    // per-query results first: o3dml_knn_search_fill finds them at the same offsets
    int32_t* si = ws.take<int32_t>(n_queries * k);
    float* sd = ws.take<float>(n_queries * k);
    int64_t* counts = ws.take<int64_t>(n_queries);
    GridIndex gi = build_grid(points, n_points, points_row_splits, nb, std::max(knn_min_target(), k * knn_target_factor()),
                              knn_cap_factor(), ws, st);
    uint32_t* qkeys = ws.take<uint32_t>(n_queries);
    uint32_t* qskeys = ws.take<uint32_t>(n_queries);
    uint32_t* qorder = ws.take<uint32_t>(n_queries);
    fill_async(neighbors_row_splits, 0, sizeof(int64_t), st);
    if (n_queries == 0) return 0;
    const uint32_t* order = nullptr;
    if (self_search) {
        order = gi.order;
    } else if (n_points > 0) {
        // process queries in cell order for wave coherence
        grid_key_kernel<<<stream_grid(n_queries, 256), 256, 0, st>>>(queries, n_queries, queries_row_splits, nb,
                                                                    gi.params, qkeys);
        O3DML_LAUNCH_CHECK();
        Workspace sws = ws;
        prim::radix_sort_pairs<uint32_t>(qkeys, nullptr, qskeys, qorder, n_queries,
                                         prim::bits_needed(static_cast<uint64_t>(std::max<int64_t>(gi.cells - 1, 0))),
                                         sws, st);
        order = qorder;
    }
    const unsigned grid = stream_grid(n_queries, 256, 1 << 20);
    const bool ig = ignore_query_point != 0;
    TimedRegion tr("knn_search", st);  // the search kernel alone (bench op roofline)
    switch (K) {
        case 1: launch_knn_k<1>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
        case 4: launch_knn_k<4>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
        case 8: launch_knn_k<8>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
        case 16: launch_knn_k<16>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
        case 32: launch_knn_k<32>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
        default: launch_knn_k<64>(metric, ig, grid, st, gi, queries, n_queries, order, queries_row_splits, nb, (int)k, si, sd, counts); break;
    }
    tr.end();
    prim::scan<int64_t, int64_t>(counts, neighbors_row_splits + 1, n_queries, true, ws, st);
    O3DML_GUARD_END
}

O3DML_API int o3dml_knn_search_fill(const float* points, int64_t n_points, const float* queries, int64_t n_queries,
                                    int64_t k, int64_t n_batch, const int64_t* queries_row_splits,
                                    const int64_t* points_row_splits_host, const int64_t* queries_row_splits_host,
                                    int metric, int ignore_query_point, const int64_t* neighbors_row_splits, int index_bits, void* neighbors_index,
                                    float* neighbors_distance, void* workspace, size_t workspace_bytes,
                                    void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    const int K = knn_bucket(k);
    if (n_queries == 0) return 0;
    if (K == 0) {
        if (k <= kManyKnnMaxK) {  // batched; overflowing queries by radix selection on the device
            knn_many_fill(points, n_points, queries, n_queries, k, nb, queries_row_splits, metric,
                          ignore_query_point, neighbors_row_splits, index_bits, neighbors_index, neighbors_distance,
                          ws, st);
            return 0;
        }
        // k > 2048: per query a radix selection + a sort of the k selected,
        // queued without any host synchronisation
        int b = 0;
        for (int64_t q = 0; q < n_queries; ++q) {
            while (b + 1 < nb && queries_row_splits_host[b + 1] <= q) ++b;
            const int64_t ps = points_row_splits_host[b], pn = points_row_splits_host[b + 1] - ps;
            topk_bigk_one(points, ps, pn, queries, q, k, metric, ignore_query_point, neighbors_row_splits,
                          index_bits, neighbors_index, neighbors_distance, ws, st);
        }
        return 0;
    }
    // same workspace layout as _count (results at the front)
    (void)points;
    (void)queries;
    (void)metric;
    const int32_t* si = ws.take<int32_t>(n_queries * k);
    const float* sd = ws.take<float>(n_queries * k);
    compact_rows_kernel<<<stream_grid(n_queries * k, 256), 256, 0, st>>>(si, sd, n_queries, (int)k,
                                                                        neighbors_row_splits, index_bits,
                                                                        neighbors_index, neighbors_distance);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
