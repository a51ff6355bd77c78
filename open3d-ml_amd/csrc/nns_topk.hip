// nns_topk.hip — exact kNN of single queries over WHOLE batch items by radix
// selection, entirely on the device (no host round trip, graph-capturable):
//   * k > 2048 (ops.knn_search / core.nns with huge k — the RandLA patch crop,
//     semseg_spatially_regular.py:94-95 / randlanet.py, k = num_points =
//     45,056 over the ~90k sub-cloud): select + a radix sort of the k
//     selected (distance, index) pairs, instead of a full sort of the item;
//   * the crop of the captured RandLA patch step (o3dml_knn_select): the
//     selected SET in index order, no sort at all (the patch is shuffled
//     right after, semseg_spatially_regular.py:100);
//     both over many workgroups (sel_* kernels below);
//   * the overflow queries of the batched 64 < k <= 2048 path (nns_many.hip:
//     candidate lists past its LDS capacity): one workgroup per listed query,
//     the overflow count read on the device (it replaced a host read and a
//     stream synchronisation per call).
//
// The order is the canonical kNN order of oracle/o3d_oracle.c (distance,
// then point index): a key is the float bits of the distance (monotone for
// distances >= +0; ignore_query_point makes the query's own position
// 0xffffffff, past every real key).  The kk-th smallest key T is found MSB
// first with three histogram passes (11/11/10-bit digits, LDS histogram of
// 2,048 bins, the first pass wave-aggregated: distances share few exponent
// bins); the selected set = keys < T plus the first (in index order) keys == T
// needed to make kk — written in index order by an order-preserving compaction
// (waves own contiguous ranges: a count pass, a 16-entry scan, a write pass
// ranked by ballot), so (distance, index) order needs only a stable sort of
// the k selected by distance.
#include <algorithm>

#include "primitives.hpp"

namespace o3dml {

constexpr int kTopkThreads = 1024;
constexpr int kTopkWaves = kTopkThreads / 64;
constexpr int kTopkBins = 2048;
constexpr int kTopkSortMax = 2048;  // selected sets sorted in LDS (overflow path)

struct TopkShared {
    uint32_t hist[kTopkBins];
    uint32_t wsum[2 * kTopkWaves];
    uint32_t sel[4];
};

template <int METRIC>
__device__ __forceinline__ uint32_t topk_key(const float* __restrict__ pts, int64_t i, float qx, float qy, float qz,
                                             bool ignore) {
    const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
    if (ignore && px == qx && py == qy && pz == qz) return 0xffffffffu;
    return __float_as_uint(dist_metric<METRIC>(px, py, pz, qx, qy, qz));
}

// The kk-th smallest (1-based) of key(j), j < n (key(j, pass): pass 0 may
// compute and store, later passes re-read): T and how many keys == T the
// selection takes (>= 1).  Every thread of the workgroup calls it.
template <class KeyFn>
__device__ void topk_radix_select(KeyFn key, int64_t n, uint32_t kk, TopkShared& s, uint32_t& T,
                                  uint32_t& take_eq) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t prefix = 0, hmask = 0, rem = kk;
    constexpr int kShift[3] = {21, 10, 0};
    constexpr uint32_t kWidth[3] = {0x7ffu, 0x7ffu, 0x3ffu};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int sh = kShift[d];
        const uint32_t wm = kWidth[d];
        for (int i = tid; i < kTopkBins; i += kTopkThreads) s.hist[i] = 0;
        __syncthreads();
        for (int64_t j0 = 0; j0 < n; j0 += kTopkThreads) {
            const int64_t j = j0 + tid;
            const bool live = j < n;
            const uint32_t k = live ? key(j, d) : 0u;
            const bool in = live && (k & hmask) == prefix;
            const uint32_t bin = (k >> sh) & wm;
            if (d == 0) {
                // few distinct exponent bins per wave: one atomic per distinct bin
                uint64_t todo = __builtin_amdgcn_ballot_w64(in);
                while (todo) {
                    const int leader = __builtin_ctzll(todo);
                    const uint32_t lb = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bin), leader));
                    const uint64_t same = __builtin_amdgcn_ballot_w64(in && bin == lb);
                    if (lane == leader) atomicAdd(&s.hist[lb], static_cast<uint32_t>(__popcll(same)));
                    todo &= ~same;
                }
            } else if (in) {
                atomicAdd(&s.hist[bin], 1u);
            }
        }
        __syncthreads();
        // the bin holding the rem-th key: thread t owns bins 2t, 2t + 1
        const uint32_t h0 = s.hist[2 * tid], h1 = s.hist[2 * tid + 1];
        const uint32_t v = h0 + h1;
        const uint32_t incl = wave_inclusive_scan(v);
        if (lane == 63) s.wsum[wv] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (int w = 0; w < wv; ++w) base += s.wsum[w];
        const uint32_t before = base + incl - v;
        if (before < rem && rem <= before + v) {
            const bool first = rem <= before + h0;
            s.sel[0] = first ? 2u * tid : 2u * tid + 1u;
            s.sel[1] = rem - (first ? before : before + h0);
        }
        __syncthreads();
        prefix |= s.sel[0] << sh;
        hmask |= wm << sh;
        rem = s.sel[1];
        __syncthreads();
    }
    T = prefix;
    take_eq = rem;
}

// Order-preserving compaction of the selection: sink(pos, j, key) for every
// selected j, pos = its rank in index order.  Wave w owns the contiguous
// range [w * chunk, (w + 1) * chunk).
template <class KeyFn, class Sink>
__device__ void topk_compact(KeyFn key, int64_t n, uint32_t T, uint32_t take_eq, TopkShared& s, Sink sink) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t chunk = ((n + kTopkWaves - 1) / kTopkWaves + 63) & ~int64_t(63);
    const int64_t a = min(n, static_cast<int64_t>(wv) * chunk), b = min(n, a + chunk);
    uint32_t lt = 0, eq = 0;
    for (int64_t j0 = a; j0 < b; j0 += 64) {
        const int64_t j = j0 + lane;
        const uint32_t k = j < b ? key(j, 3) : 0xffffffffu;
        lt += static_cast<uint32_t>(__popcll(__builtin_amdgcn_ballot_w64(j < b && k < T)));
        eq += static_cast<uint32_t>(__popcll(__builtin_amdgcn_ballot_w64(j < b && k == T)));
    }
    if (lane == 0) {
        s.wsum[wv] = lt;
        s.wsum[kTopkWaves + wv] = eq;
    }
    __syncthreads();
    uint32_t lt_base = 0, eq_base = 0;
    for (int w = 0; w < wv; ++w) {
        lt_base += s.wsum[w];
        eq_base += s.wsum[kTopkWaves + w];
    }
    __syncthreads();  // wsum reused by the caller
    uint32_t pos = lt_base + min(eq_base, take_eq), eqr = eq_base;
    const uint64_t below = lanemask_lt();
    for (int64_t j0 = a; j0 < b; j0 += 64) {
        const int64_t j = j0 + lane;
        const uint32_t k = j < b ? key(j, 4) : 0xffffffffu;
        const bool is_eq = j < b && k == T;
        const uint64_t em = __builtin_amdgcn_ballot_w64(is_eq);
        const bool take = (j < b && k < T) || (is_eq && eqr + __popcll(em & below) < take_eq);
        const uint64_t tm = __builtin_amdgcn_ballot_w64(take);
        if (take) sink(pos + static_cast<uint32_t>(__popcll(tm & below)), j, k);
        pos += static_cast<uint32_t>(__popcll(tm));
        eqr += static_cast<uint32_t>(__popcll(em));
    }
}

// ---------------------------------------------------------------------------
// one query over a whole item (the RandLA crop, k > 2048 rows): the same
// selection spread over up to 256 workgroups, each owning a contiguous chunk
// of the item: three histogram launches (11/11/10-bit digits; each workgroup
// re-derives the digits chosen so far from the global histograms, 8 bins per
// thread), a count launch (per-workgroup keys < T and == T) and an ordered
// write launch (workgroup bases from the counts, tile ranks by ballot).  A
// single workgroup walking a ~100k-point item five times took ~0.1 ms per
// patch; this is a few microseconds per launch.
// ---------------------------------------------------------------------------
constexpr int kSelThreads = 256;
constexpr int kSelMaxWgs = 256;
constexpr int kSelChunkMin = 4096;  // histogram passes: keys per workgroup at least (fewer global atomics)
constexpr int kSelChunkOut = 1024;  // count / ordered write: keys per workgroup at least (tiles walked in order)

struct SelGlobal {
    uint32_t hist[3][kTopkBins];  // zeroed per call (one memset)
    uint32_t cnt[2][kSelMaxWgs];  // per workgroup: keys < T, keys == T
};

struct SelShared {
    uint32_t h[kTopkBins];
    uint32_t wsum[2][kSelThreads / 64];
    uint32_t sel[2];
};

__device__ __forceinline__ int sel_shift(int d) { return d == 0 ? 21 : (d == 1 ? 10 : 0); }
__device__ __forceinline__ uint32_t sel_width(int d) { return d == 2 ? 0x3ffu : 0x7ffu; }

// the bin of histogram h holding the rem-th key (every thread of the
// workgroup calls it; thread t owns bins 8t .. 8t + 7): bin and the rank
// within it, through LDS
__device__ void sel_find(const uint32_t* __restrict__ h, uint32_t rem, SelShared& s, uint32_t& bin,
                         uint32_t& rem_out) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint4 a = reinterpret_cast<const uint4*>(h)[2 * tid], b = reinterpret_cast<const uint4*>(h)[2 * tid + 1];
    const uint32_t hv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += hv[i];
    const uint32_t incl = wave_inclusive_scan(v);
    if (lane == 63) s.wsum[0][wv] = incl;
    __syncthreads();
    uint32_t before = incl - v;
    for (int w = 0; w < wv; ++w) before += s.wsum[0][w];
    if (before < rem && rem <= before + v) {
        uint32_t acc = before;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (rem <= acc + hv[i]) {
                s.sel[0] = 8u * tid + i;
                s.sel[1] = rem - acc;
                break;
            }
            acc += hv[i];
        }
    }
    __syncthreads();
    bin = s.sel[0];
    rem_out = s.sel[1];
    __syncthreads();
}

// digits 0 .. npass-1 of the kk-th smallest key from the global histograms
__device__ void sel_resolve(const SelGlobal* __restrict__ g, uint32_t kk, int npass, SelShared& s, uint32_t& prefix,
                            uint32_t& hmask, uint32_t& rem) {
    prefix = 0;
    hmask = 0;
    rem = kk;
    for (int d = 0; d < npass; ++d) {
        uint32_t bin;
        sel_find(g->hist[d], rem, s, bin, rem);
        prefix |= bin << sel_shift(d);
        hmask |= sel_width(d) << sel_shift(d);
    }
}

__device__ __forceinline__ uint32_t sel_kk(const int64_t* rs, int64_t q, int64_t k) {
    return static_cast<uint32_t>(rs ? rs[q + 1] - rs[q] : k);
}

template <int METRIC, int PASS>
__global__ void __launch_bounds__(kSelThreads) sel_hist_kernel(const float* __restrict__ pts, int64_t n,
                                                               const float* __restrict__ query, int ignore,
                                                               const int64_t* __restrict__ rs, int64_t q, int64_t k,
                                                               int64_t chunk, uint32_t* __restrict__ keys,
                                                               SelGlobal* __restrict__ g) {
    __shared__ SelShared s;
    const uint32_t kk = sel_kk(rs, q, k);
    if (kk == 0) return;
    const int tid = threadIdx.x;
    uint32_t prefix = 0, hmask = 0, rem;
    if (PASS > 0) sel_resolve(g, kk, PASS, s, prefix, hmask, rem);
    for (int i = tid; i < kTopkBins; i += kSelThreads) s.h[i] = 0;
    __syncthreads();
    const float qx = query[0], qy = query[1], qz = query[2];
    const int64_t a = static_cast<int64_t>(blockIdx.x) * chunk, b = min(n, a + chunk);
    constexpr int sh = PASS == 0 ? 21 : (PASS == 1 ? 10 : 0);
    constexpr uint32_t wm = PASS == 2 ? 0x3ffu : 0x7ffu;
    constexpr int U = 4;  // keys per thread in flight
    for (int64_t j0 = a; j0 < b; j0 += U * kSelThreads) {
        uint32_t kv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * kSelThreads + tid;
            kv[u] = 0;
            if (j < b) {
                if (PASS == 0) {
                    kv[u] = topk_key<METRIC>(pts, j, qx, qy, qz, ignore != 0);
                    keys[j] = kv[u];
                } else {
                    kv[u] = keys[j];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = j0 + u * kSelThreads + tid < b && (kv[u] & hmask) == prefix;
            if (in) atomicAdd(&s.h[(kv[u] >> sh) & wm], 1u);
        }
    }
    __syncthreads();
    for (int i = tid; i < kTopkBins; i += kSelThreads)
        if (s.h[i]) atomicAdd(&g->hist[PASS][i], s.h[i]);
}

// per workgroup: keys < T and keys == T in its chunk
__global__ void __launch_bounds__(kSelThreads) sel_count_kernel(int64_t n, const int64_t* __restrict__ rs, int64_t q,
                                                                int64_t k, int64_t chunk,
                                                                const uint32_t* __restrict__ keys,
                                                                SelGlobal* __restrict__ g) {
    __shared__ SelShared s;
    const uint32_t kk = sel_kk(rs, q, k);
    if (kk == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t T, hmask, take;
    sel_resolve(g, kk, 3, s, T, hmask, take);
    const int64_t a = static_cast<int64_t>(blockIdx.x) * chunk, b = min(n, a + chunk);
    uint32_t lt = 0, eq = 0;
    for (int64_t j = a + tid; j < b; j += kSelThreads) {
        const uint32_t kv = keys[j];
        lt += kv < T;
        eq += kv == T;
    }
    // block sums (lane 63 of the inclusive scans)
    lt = wave_inclusive_scan(lt);
    eq = wave_inclusive_scan(eq);
    if (lane == 63) {
        s.wsum[0][wv] = lt;
        s.wsum[1][wv] = eq;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t tl = 0, te = 0;
        for (int w = 0; w < kSelThreads / 64; ++w) {
            tl += s.wsum[0][w];
            te += s.wsum[1][w];
        }
        g->cnt[0][blockIdx.x] = tl;
        g->cnt[1][blockIdx.x] = te;
    }
}

// the selection in index order: pos of every selected j; SINK 0 = int64 ids
// (+ base), 1 = (key, local index) pairs padded with ~0 up to kcap
template <int SINK>
__global__ void __launch_bounds__(kSelThreads) sel_write_kernel(int64_t n, const int64_t* __restrict__ rs, int64_t q,
                                                                int64_t k, int64_t chunk,
                                                                const uint32_t* __restrict__ keys,
                                                                const SelGlobal* __restrict__ g,
                                                                int64_t* __restrict__ out_ids, int64_t kcap,
                                                                uint32_t* __restrict__ sel_key,
                                                                uint32_t* __restrict__ sel_idx) {
    __shared__ SelShared s;
    __shared__ uint32_t wcnt[2][2][kSelThreads / 64];  // [tile parity][eq, take][wave]
    const uint32_t kk = sel_kk(rs, q, k);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (SINK == 1) {
        for (int64_t i = kk + static_cast<int64_t>(blockIdx.x) * kSelThreads + tid; i < kcap;
             i += static_cast<int64_t>(gridDim.x) * kSelThreads) {
            sel_key[i] = 0xffffffffu;
            sel_idx[i] = 0xffffffffu;
        }
    }
    if (kk == 0) return;
    uint32_t T, hmask, take_eq;
    sel_resolve(g, kk, 3, s, T, hmask, take_eq);
    // bases: the counts of the workgroups before this one
    uint32_t lt = tid < static_cast<int>(blockIdx.x) ? g->cnt[0][tid] : 0u;
    uint32_t eq = tid < static_cast<int>(blockIdx.x) ? g->cnt[1][tid] : 0u;
    lt = wave_inclusive_scan(lt);
    eq = wave_inclusive_scan(eq);
    if (lane == 63) {
        s.wsum[0][wv] = lt;
        s.wsum[1][wv] = eq;
    }
    __syncthreads();
    uint32_t lt_base = 0, eq_base = 0;
    for (int w = 0; w < kSelThreads / 64; ++w) {
        lt_base += s.wsum[0][w];
        eq_base += s.wsum[1][w];
    }
    uint32_t pos = lt_base + min(eq_base, take_eq), eqr = eq_base;
    const uint64_t below = lanemask_lt();
    const int64_t a = static_cast<int64_t>(blockIdx.x) * chunk, b = min(n, a + chunk);
    int par = 0;
    for (int64_t j0 = a; j0 < b; j0 += kSelThreads, par ^= 1) {
        const int64_t j = j0 + tid;
        const uint32_t kv = j < b ? keys[j] : 0xffffffffu;
        const bool is_lt = j < b && kv < T, is_eq = j < b && kv == T;
        const uint64_t em = __builtin_amdgcn_ballot_w64(is_eq);
        if (lane == 0) wcnt[par][0][wv] = static_cast<uint32_t>(__popcll(em));
        __syncthreads();
        uint32_t eq_before = eqr, eq_tile = 0;
        for (int w = 0; w < kSelThreads / 64; ++w) {
            const uint32_t c = wcnt[par][0][w];
            if (w < wv) eq_before += c;
            eq_tile += c;
        }
        const bool take = is_lt || (is_eq && eq_before + __popcll(em & below) < take_eq);
        const uint64_t tm = __builtin_amdgcn_ballot_w64(take);
        if (lane == 0) wcnt[par][1][wv] = static_cast<uint32_t>(__popcll(tm));
        __syncthreads();
        uint32_t t_before = pos, t_tile = 0;
        for (int w = 0; w < kSelThreads / 64; ++w) {
            const uint32_t c = wcnt[par][1][w];
            if (w < wv) t_before += c;
            t_tile += c;
        }
        if (take) {
            const uint32_t p = t_before + static_cast<uint32_t>(__popcll(tm & below));
            if (p < kk) {  // always (T exact); bounds the store regardless
                if (SINK == 0) {
                    out_ids[p] = j;
                } else {
                    sel_key[p] = kv;
                    sel_idx[p] = static_cast<uint32_t>(j);
                }
            }
        }
        pos += t_tile;
        eqr += eq_tile;
    }
}

__global__ void __launch_bounds__(kSelThreads) sel_zero_kernel(SelGlobal* __restrict__ g) {
    uint32_t* h = &g->hist[0][0];
    for (int i = threadIdx.x; i < 3 * kTopkBins; i += kSelThreads) h[i] = 0;
}

size_t sel_workspace_bytes(int64_t n) { return ws_bytes<uint32_t>(n) + ws_bytes<SelGlobal>(1); }

// the launches of one selection (zero + 3 histograms + count + write; the
// histograms are cleared by a kernel, not a memset node, in captured graphs)
template <int SINK>
static void sel_run(const float* pts, int64_t n, const float* query, int metric, int ignore, const int64_t* rs,
                    int64_t q, int64_t k, int64_t* out_ids, int64_t kcap, uint32_t* sel_key, uint32_t* sel_idx,
                    Workspace& ws, hipStream_t st) {
    uint32_t* keys = ws.take<uint32_t>(n);
    SelGlobal* g = ws.take<SelGlobal>(1);
    sel_zero_kernel<<<1, kSelThreads, 0, st>>>(g);
    const int64_t G = std::max<int64_t>(1, std::min<int64_t>(kSelMaxWgs, ceil_div(n, kSelChunkMin)));
    const int64_t chunk = ceil_div(n, G);
    const unsigned grid = static_cast<unsigned>(G);
    // the count / write launches walk their chunk tile by tile (two barriers
    // per 256 keys): smaller chunks, more workgroups
    const int64_t Gw = std::max<int64_t>(1, std::min<int64_t>(kSelMaxWgs, ceil_div(n, kSelChunkOut)));
    const int64_t chunk_w = ceil_div(n, Gw);
    const unsigned grid_w = static_cast<unsigned>(ceil_div(n, chunk_w));
#define O3DML_SELH(M, P) \
    sel_hist_kernel<M, P><<<grid, kSelThreads, 0, st>>>(pts, n, query, ignore, rs, q, k, chunk, keys, g)
#define O3DML_SELH3(M) \
    do {                  \
        O3DML_SELH(M, 0); \
        O3DML_SELH(M, 1); \
        O3DML_SELH(M, 2); \
    } while (0)
    if (metric == kL2) O3DML_SELH3(kL2); else if (metric == kL1) O3DML_SELH3(kL1); else O3DML_SELH3(kLinf);
#undef O3DML_SELH3
#undef O3DML_SELH
    O3DML_LAUNCH_CHECK();
    sel_count_kernel<<<grid_w, kSelThreads, 0, st>>>(n, rs, q, k, chunk_w, keys, g);
    O3DML_LAUNCH_CHECK();
    sel_write_kernel<SINK><<<grid_w, kSelThreads, 0, st>>>(n, rs, q, k, chunk_w, keys, g, out_ids, kcap, sel_key,
                                                           sel_idx);
    O3DML_LAUNCH_CHECK();
}

// the overflow queries of the batched path (64 < k <= 2048): one workgroup
// per listed query (grid-stride over the device count), keys recomputed from
// the points on every pass (no per-query buffer), the selection sorted in LDS
// by (distance, index) and written to the row at rs[q]
__device__ __forceinline__ void topk_lds_bitonic(uint64_t* v, int N) {
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < N; i += kTopkThreads) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = v[i], b = v[ixj];
                    if ((a > b) == ((i & k) == 0)) {
                        v[i] = b;
                        v[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

template <int METRIC>
__global__ void __launch_bounds__(kTopkThreads) topk_overflow_kernel(
        const float* __restrict__ pts, const float* __restrict__ queries, const int64_t* __restrict__ prs,
        const int64_t* __restrict__ qrs, int nb, int ignore, const uint32_t* __restrict__ over,
        const int64_t* __restrict__ n_over, const int64_t* __restrict__ rs, int bits, void* __restrict__ out_idx,
        float* __restrict__ out_dist) {
    __shared__ TopkShared s;
    __shared__ uint64_t buf[kTopkSortMax];
    const int64_t cnt = *n_over;
    for (int64_t t = blockIdx.x; t < cnt; t += gridDim.x) {
        const int64_t q = over[t];
        const int b = batch_of(q, qrs, nb);
        const int64_t ps = prs[b], pn = prs[b + 1] - ps;
        const uint32_t kk = static_cast<uint32_t>(rs[q + 1] - rs[q]);  // <= kTopkSortMax (k <= 2048)
        if (kk == 0) continue;
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        auto key = [&](int64_t j, int) { return topk_key<METRIC>(pts, ps + j, qx, qy, qz, ignore != 0); };
        uint32_t T, take;
        topk_radix_select(key, pn, kk, s, T, take);
        topk_compact(key, pn, T, take, s, [&](uint32_t pos, int64_t j, uint32_t k) {
            buf[pos] = (static_cast<uint64_t>(k) << 32) | static_cast<uint32_t>(ps + j);
        });
        int N = 1;
        while (N < static_cast<int>(kk)) N <<= 1;
        for (int i = kk + threadIdx.x; i < N; i += kTopkThreads) buf[i] = ~0ull;
        __syncthreads();
        topk_lds_bitonic(buf, N);
        const int64_t o = rs[q];
        for (int i = threadIdx.x; i < static_cast<int>(kk); i += kTopkThreads) {
            const uint64_t v = buf[i];
            const uint32_t id = static_cast<uint32_t>(v);
            if (bits == 32)
                static_cast<int32_t*>(out_idx)[o + i] = static_cast<int32_t>(id);
            else
                static_cast<int64_t*>(out_idx)[o + i] = static_cast<int64_t>(id);
            if (out_dist) out_dist[o + i] = __uint_as_float(static_cast<uint32_t>(v >> 32));
        }
        __syncthreads();  // buf / s reused by the next query
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
void topk_overflow(const float* pts, const float* queries, const int64_t* prs, const int64_t* qrs, int nb,
                   int metric, int ignore, const uint32_t* over, const int64_t* n_over, const int64_t* rs, int bits,
                   void* oi, float* od, int64_t max_over, hipStream_t st) {
    if (max_over <= 0) return;
    // a fixed grid: the count stays on the device (usually 0 — the waves exit)
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(max_over, 64));
#define O3DML_TOV(M) \
    topk_overflow_kernel<M><<<g, kTopkThreads, 0, st>>>(pts, queries, prs, qrs, nb, ignore, over, n_over, rs, bits, oi, od)
    if (metric == kL2) O3DML_TOV(kL2); else if (metric == kL1) O3DML_TOV(kL1); else O3DML_TOV(kLinf);
#undef O3DML_TOV
    O3DML_LAUNCH_CHECK();
}

size_t topk_bigk_workspace_bytes(int64_t n_points, int64_t k) {
    const int64_t kc = std::min(k, n_points);
    return sel_workspace_bytes(n_points) + 4 * ws_bytes<uint32_t>(kc) + prim::radix_sort_workspace_bytes<uint32_t>(kc);
}

__global__ void write_topk_rows_kernel(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ sidx,
                                       const int64_t* __restrict__ rs, int64_t q, int64_t base_id, int bits,
                                       void* __restrict__ out_idx, float* __restrict__ out_dist) {
    const int64_t out_off = rs[q], cnt = rs[q + 1] - out_off;
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < cnt;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t id = base_id + sidx[j];
        if (bits == 32)
            static_cast<int32_t*>(out_idx)[out_off + j] = static_cast<int32_t>(id);
        else
            static_cast<int64_t*>(out_idx)[out_off + j] = id;
        if (out_dist) out_dist[out_off + j] = __uint_as_float(skeys[j]);
    }
}

// one query of the k > 2048 path: select, stable sort of the selected by
// distance (index order kept among equal distances), write the row
void topk_bigk_one(const float* pts, int64_t ps, int64_t pn, const float* queries, int64_t q, int64_t k,
                   int metric, int ignore, const int64_t* rs, int bits, void* oi, float* od, Workspace ws,
                   hipStream_t st) {
    if (pn == 0) return;
    const int64_t kc = std::min(k, pn);
    uint32_t* k_in = ws.take<uint32_t>(kc);
    uint32_t* i_in = ws.take<uint32_t>(kc);
    uint32_t* k_out = ws.take<uint32_t>(kc);
    uint32_t* i_out = ws.take<uint32_t>(kc);
    sel_run<1>(pts + 3 * ps, pn, queries + 3 * q, metric, ignore, rs, q, 0, nullptr, kc, k_in, i_in, ws, st);
    prim::radix_sort_pairs<uint32_t>(k_in, i_in, k_out, i_out, kc, 32, ws, st);
    write_topk_rows_kernel<<<stream_grid(kc, 256), 256, 0, st>>>(k_out, i_out, rs, q, ps, bits, oi, od);
    O3DML_LAUNCH_CHECK();
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_knn_select_workspace_size(int64_t n_points) { return sel_workspace_bytes(n_points); }

O3DML_API int o3dml_knn_select(const float* points, int64_t n_points, const float* center, int64_t k, int metric,
                               int64_t* out_index, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k >= 1 && k <= n_points, "knn_select: need 1 <= k <= n_points");
    O3DML_REQUIRE(n_points < (int64_t(1) << 31), "too many points");
    O3DML_REQUIRE(metric >= 0 && metric <= 2, "metric must be L1(0), L2(1) or Linf(2)");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    sel_run<0>(points, n_points, center, metric, 0, nullptr, 0, k, out_index, 0, nullptr, nullptr, ws, st);
    O3DML_GUARD_END
}
