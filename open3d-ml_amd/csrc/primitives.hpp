// primitives.hpp — device-wide building blocks used by the hot-path kernels:
//   * scan():            tiled reduce-then-scan (deterministic, in-place safe)
//   * radix_sort_pairs(): stable LSD radix sort (8-bit digits) of u32/u64 keys
//                         with u32 payloads; stability is what gives the
//                         canonical "ascending point id within a bin / voxel"
//                         order the oracle defines.
// Header-only templates, instantiated per translation unit (no -fgpu-rdc).
#pragma once

#include <cstdlib>

#include <type_traits>

#include "common.hpp"

namespace o3dml {
namespace prim {

constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;  // 2048 elements per workgroup

template <class TIn>
__global__ void __launch_bounds__(kScanBlock) scan_tile_sums(const TIn* __restrict__ in, int64_t n,
                                                             int64_t* __restrict__ sums) {
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + k * kScanBlock + threadIdx.x;
        if (i < n) s += static_cast<int64_t>(in[i]);
    }
    s = wave_sum(s);
    __shared__ int64_t ws[kScanBlock / 64];
    if (lane_id() == 0) ws[wave_id()] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
#pragma unroll
        for (int w = 0; w < kScanBlock / 64; ++w) t += ws[w];
        sums[blockIdx.x] = t;
    }
}

// Scan one tile (striped coalesced load -> LDS -> blocked per-thread scan).
// offsets (nullable): exclusive carry-in per tile.
// raw_sums (nullable): the tiles' plain sums — the tile adds up its
// predecessors itself (no separate scan of the sums: one launch fewer).
// tail (nullable, e.g. pinned host memory): the last tile writes the total
// to tail[0] and, with tail_src, tail_src[0] to tail[1].
template <class TIn, class TOut>
__global__ void __launch_bounds__(kScanBlock) scan_tile_apply(const TIn* in, TOut* out, int64_t n,
                                                              const int64_t* __restrict__ offsets,
                                                              int inclusive,
                                                              const int64_t* __restrict__ raw_sums = nullptr,
                                                              int64_t* tail = nullptr,
                                                              const int64_t* tail_src = nullptr) {
    // +1 pad per 8 elements keeps the blocked LDS reads off one bank
    __shared__ int64_t tile[kScanTile + kScanTile / 8];
    __shared__ int64_t wsum[kScanBlock / 64];
    __shared__ int64_t carry_in[kScanBlock / 64];
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
    const int t = threadIdx.x;
    if (raw_sums) {  // (uniform branch) carry = sum of the earlier tiles' sums, 4 loads in flight
        int64_t c = 0;
        const int64_t nb = blockIdx.x;
        int64_t j = t;
        for (; j + 3 * kScanBlock < nb; j += 4 * kScanBlock)
            c += (raw_sums[j] + raw_sums[j + kScanBlock]) + (raw_sums[j + 2 * kScanBlock] + raw_sums[j + 3 * kScanBlock]);
        for (; j < nb; j += kScanBlock) c += raw_sums[j];
        c = wave_sum(c);
        if (lane_id() == 0) carry_in[wave_id()] = c;
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int e = k * kScanBlock + t;
        const int64_t i = base + e;
        tile[e + (e >> 3)] = i < n ? static_cast<int64_t>(in[i]) : 0;
    }
    __syncthreads();
    int64_t v[kScanItems];
    int64_t acc = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        const int e = t * kScanItems + j;
        v[j] = tile[e + (e >> 3)];
        acc += v[j];
    }
    const int64_t incl = wave_inclusive_scan(acc);
    if (lane_id() == 63) wsum[wave_id()] = incl;
    __syncthreads();
    int64_t run = incl - acc + (offsets ? offsets[blockIdx.x] : 0);
    if (raw_sums)
        for (int w = 0; w < kScanBlock / 64; ++w) run += carry_in[w];
    for (int w = 0; w < wave_id(); ++w) run += wsum[w];
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        const int e = t * kScanItems + j;
        const int64_t x = v[j];
        tile[e + (e >> 3)] = inclusive ? run + x : run;
        run += x;
    }
    if (tail && blockIdx.x == gridDim.x - 1 && t == kScanBlock - 1) {  // run = the inclusive total
        tail[0] = run;
        if (tail_src) tail[1] = tail_src[0];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int e = k * kScanBlock + t;
        const int64_t i = base + e;
        if (i < n) out[i] = static_cast<TOut>(tile[e + (e >> 3)]);
    }
}

inline size_t scan_workspace_bytes(int64_t n) {
    size_t b = 0;
    int64_t tiles = ceil_div(n, kScanTile);
    while (tiles > 1) {
        b += ws_bytes<int64_t>(tiles);
        tiles = ceil_div(tiles, kScanTile);
    }
    return b;
}

// Tiles up to which every tile sums its predecessors' sums itself (two
// launches: sums, apply); more tiles scan the sums recursively (three+).
constexpr int64_t kScanDirectTiles = 4096;

// out[i] = sum_{j<=i} in[j] (inclusive) or sum_{j<i} in[j] (exclusive).
// in == out is allowed.  tail (nullable): total -> tail[0] (and tail_src[0]
// -> tail[1]) written by the last tile, e.g. into pinned host memory.
template <class TIn, class TOut>
void scan(const TIn* in, TOut* out, int64_t n, bool inclusive, Workspace& ws, hipStream_t st,
          int64_t* tail = nullptr, const int64_t* tail_src = nullptr) {
    if (n <= 0) return;
    const int64_t tiles = ceil_div(n, kScanTile);
    if (tiles == 1) {
        scan_tile_apply<TIn, TOut><<<1, kScanBlock, 0, st>>>(in, out, n, nullptr, inclusive, nullptr, tail,
                                                             tail_src);
        O3DML_LAUNCH_CHECK();
        return;
    }
    int64_t* sums = ws.take<int64_t>(tiles);
    scan_tile_sums<TIn><<<static_cast<unsigned>(tiles), kScanBlock, 0, st>>>(in, n, sums);
    O3DML_LAUNCH_CHECK();
    if (tiles <= kScanDirectTiles) {
        scan_tile_apply<TIn, TOut><<<static_cast<unsigned>(tiles), kScanBlock, 0, st>>>(in, out, n, nullptr,
                                                                                       inclusive, sums, tail,
                                                                                       tail_src);
        O3DML_LAUNCH_CHECK();
        return;
    }
    scan<int64_t, int64_t>(sums, sums, tiles, false, ws, st);
    scan_tile_apply<TIn, TOut><<<static_cast<unsigned>(tiles), kScanBlock, 0, st>>>(in, out, n, sums,
                                                                                   inclusive, nullptr, tail,
                                                                                   tail_src);
    O3DML_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits, 2048-key tiles.
// ---------------------------------------------------------------------------
constexpr int kRsBlock = 256;
#ifndef O3DML_RS_ITEMS
#define O3DML_RS_ITEMS 8
#endif
constexpr int kRsItems = O3DML_RS_ITEMS;
constexpr int kRsTile = kRsBlock * kRsItems;
constexpr int kRsWaves = kRsBlock / 64;

// offs[d * tiles + j] = number of digit-d keys in tiles < j, dtot[d] = all
// digit-d keys: one block per digit scans its row of the tile histogram (the
// digits' global bases are a 256-entry scan the scatter kernel does itself).
static __global__ void __launch_bounds__(kRsBlock) radix_digit_scan(const uint32_t* __restrict__ hist, int64_t tiles,
                                                             uint32_t* __restrict__ offs,
                                                             uint32_t* __restrict__ dtot,
                                                             const uint64_t* __restrict__ or_and = nullptr,
                                                             int pass = 0) {
    if (or_and && pass > 0 && ((((or_and[0] & or_and[1]) >> (8 * pass)) & 255u) == 0)) return;  // skipped pass
    __shared__ uint32_t wsum[kRsWaves];
    const int64_t row = static_cast<int64_t>(blockIdx.x) * tiles;
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < tiles; c0 += kRsBlock * 8) {
        uint32_t v[8];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // blocked: thread t owns entries t*8 .. t*8+7 of the chunk
            const int64_t j = c0 + threadIdx.x * 8 + k;
            v[k] = j < tiles ? hist[row + j] : 0u;
            acc += v[k];
        }
        const uint32_t inc = wave_inclusive_scan(acc);
        if (lane_id() == 63) wsum[wave_id()] = inc;
        __syncthreads();
        uint32_t run = carry + inc - acc, tot = 0;
#pragma unroll
        for (int w = 0; w < kRsWaves; ++w) {
            run += w < wave_id() ? wsum[w] : 0u;
            tot += wsum[w];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t j = c0 + threadIdx.x * 8 + k;
            if (j < tiles) offs[row + j] = run;
            run += v[k];
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) dtot[blockIdx.x] = carry;
}

// Device-planned passes (radix_sort_pairs with or_and != nullptr): or_and[0]
// = OR of all keys, or_and[1] = OR of their complements (both start at 0),
// so the bits that vary among the keys are or_and[0] & or_and[1] and
// only passes whose 8-bit digit varies run (pass 0 always: it also moves
// the keys when none varies); the others return at once.  The i-th of the A
// running passes reads the input (i = 0) or the previous pass's output and
// writes out when A - 1 - i is even, tmp otherwise, so the last running pass
// lands in out.  Returns false for a skipped pass.
template <class K>
struct PassPlan {
    const K* src;
    K* dst;
    const uint32_t* vsrc;
    uint32_t* vdst;
};

template <class K>
__device__ __forceinline__ bool device_pass(const uint64_t* or_and, int p, int passes, const K* kin,
                                            const uint32_t* vin, K* ktmp, uint32_t* vtmp, K* kout, uint32_t* vout,
                                            PassPlan<K>& plan) {
    const uint64_t vary = or_and[0] & or_and[1];
    auto act = [&](int q) { return q == 0 || ((vary >> (8 * q)) & 255u) != 0; };
    if (!act(p)) return false;
    int A = 0, i = 0;
    for (int q = 0; q < passes; ++q) {
        const bool a = act(q);
        A += a;
        i += a && q < p;
    }
    auto dst_out = [&](int j) { return ((A - 1 - j) & 1) == 0; };
    plan.src = i == 0 ? kin : (dst_out(i - 1) ? kout : ktmp);
    plan.vsrc = i == 0 ? vin : (dst_out(i - 1) ? vout : vtmp);
    plan.dst = dst_out(i) ? kout : ktmp;
    plan.vdst = dst_out(i) ? vout : vtmp;
    return true;
}

template <class K>
__global__ void __launch_bounds__(kRsBlock) radix_hist(const K* __restrict__ keys, int64_t n, int shift,
                                                       uint32_t* __restrict__ hist, int64_t tiles,
                                                       const uint64_t* __restrict__ or_and = nullptr,
                                                       int passes = 0, const K* kalt = nullptr,
                                                       const K* kout = nullptr) {
    if (or_and) {  // device-planned: skip, or read this pass's source (keys = the input)
        PassPlan<K> pl;
        if (!device_pass<K>(or_and, shift / 8, passes, keys, nullptr, const_cast<K*>(kalt), nullptr,
                            const_cast<K*>(kout), nullptr, pl))
            return;
        keys = pl.src;
    }
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile;
#pragma unroll
    for (int k = 0; k < kRsItems; ++k) {
        const int64_t i = base + k * kRsBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[static_cast<uint32_t>(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[static_cast<int64_t>(threadIdx.x) * tiles + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter.  Each wave ranks its own contiguous 512 keys of the tile,
// row by row (64 keys; peers with the same digit found with eight 64-bit
// ballots), keeping its running per-digit counts in LDS — LDS operations of
// one wave execute in order, so no barrier is needed between rows.  One
// block scan then turns (digit, wave) counts into tile-local bases (tile
// digit offset + counts of earlier waves: stable), the keys are placed in
// LDS in tile-local digit order and written out so that consecutive threads
// write consecutive addresses of each digit run (coalesced).  Four barriers
// per tile.
template <class K>
__global__ void __launch_bounds__(kRsBlock) radix_scatter(const K* kin, const uint32_t* vin, K* kout, uint32_t* vout,
                                                          int64_t n, int shift,
                                                          const uint32_t* __restrict__ offsets,
                                                          const uint32_t* __restrict__ dtot,
                                                          const uint32_t* __restrict__ hist, int64_t tiles,
                                                          const uint64_t* __restrict__ or_and = nullptr,
                                                          int passes = 0, K* ktmp = nullptr,
                                                          uint32_t* vtmp = nullptr, K* kfinal = nullptr,
                                                          uint32_t* vfinal = nullptr) {
    if (or_and) {  // device-planned: kin / vin = the sort's input, kfinal / vfinal its output
        PassPlan<K> pl;
        if (!device_pass<K>(or_and, shift / 8, passes, kin, vin, ktmp, vtmp, kfinal, vfinal, pl)) return;
        kin = pl.src;
        vin = pl.vsrc;
        kout = pl.dst;
        vout = pl.vdst;
    }
    constexpr int kRowsPerWave = kRsItems * kRsBlock / 64 / kRsWaves;  // = kRsItems
    __shared__ uint32_t wcnt[kRsWaves][256];
    __shared__ uint32_t wsum[kRsWaves], dsum[kRsWaves];
    __shared__ uint32_t toff[256];
    __shared__ int64_t goff[256];
    __shared__ K lkey[kRsTile];
    __shared__ uint32_t lval[kRsTile];
    const int t = threadIdx.x;
    const int w = wave_id();
    const int lane = lane_id();
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile;
    const int tile_n = static_cast<int>(n - base < kRsTile ? n - base : kRsTile);
    {
        // tile digit offsets: exclusive scan of this tile's histogram
        const uint32_t c = hist[static_cast<int64_t>(t) * tiles + blockIdx.x];
        const uint32_t inc = wave_inclusive_scan(c);
        // digit total and this tile's base within its digit: from
        // radix_digit_scan, or (offsets == nullptr: few tiles) summed here
        // over the digit's histogram row — the same counts, one launch fewer
        uint32_t dt, tbase;
        if (offsets) {
            dt = dtot[t];
            tbase = offsets[static_cast<int64_t>(t) * tiles + blockIdx.x];
        } else {
            dt = 0u;
            tbase = 0u;
            const uint32_t* hr = hist + static_cast<int64_t>(t) * tiles;
            for (int64_t j = 0; j < tiles; ++j) {
                const uint32_t v = hr[j];
                dt += v;
                tbase += j < static_cast<int64_t>(blockIdx.x) ? v : 0u;
            }
        }
        const uint32_t dinc = wave_inclusive_scan(dt);  // digit bases: scan of the digit totals
        if (lane == 63) {
            wsum[w] = inc;
            dsum[w] = dinc;
        }
#pragma unroll
        for (int ww = 0; ww < kRsWaves; ++ww) wcnt[ww][t] = 0;
        __syncthreads();
        uint32_t before = 0, dbefore = 0;
        for (int ww = 0; ww < w; ++ww) {
            before += wsum[ww];
            dbefore += dsum[ww];
        }
        toff[t] = before + inc - c;
        goff[t] = static_cast<int64_t>(dbefore + dinc - dt) + tbase;
    }
    // phase 1: each wave ranks its rows in order, counts per digit in LDS
    const uint64_t lt = lanemask_lt();
    K key[kRowsPerWave];
    uint32_t val[kRowsPerWave], loff[kRowsPerWave];
    uint32_t dig[kRowsPerWave];
#pragma unroll
    for (int r = 0; r < kRowsPerWave; ++r) {
        const int64_t i = base + (static_cast<int64_t>(w) * kRowsPerWave + r) * 64 + lane;
        const bool valid = i < n;
        key[r] = valid ? kin[i] : K(0);
        val[r] = valid ? (vin ? vin[i] : static_cast<uint32_t>(i)) : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRowsPerWave; ++r) {
        const int64_t i = base + (static_cast<int64_t>(w) * kRowsPerWave + r) * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = static_cast<uint32_t>(key[r] >> shift) & 255u;
        dig[r] = d;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t before = valid ? wcnt[w][d] : 0u;
        loff[r] = before + rank;
        if (valid && rank == 0) wcnt[w][d] = before + static_cast<uint32_t>(__popcll(peers));
    }
    __syncthreads();
    // phase 2: (digit, wave) counts -> tile-local bases
    {
        uint32_t acc = toff[t];
#pragma unroll
        for (int ww = 0; ww < kRsWaves; ++ww) {
            const uint32_t c = wcnt[ww][t];
            wcnt[ww][t] = acc;
            acc += c;
        }
    }
    __syncthreads();
    // phase 3: place in tile-local digit order
#pragma unroll
    for (int r = 0; r < kRowsPerWave; ++r) {
        const int64_t i = base + (static_cast<int64_t>(w) * kRowsPerWave + r) * 64 + lane;
        if (i < n) {
            const uint32_t lp = wcnt[w][dig[r]] + loff[r];
            lkey[lp] = key[r];
            lval[lp] = val[r];
        }
    }
    __syncthreads();
    // phase 4: coalesced runs out
    for (int j = t; j < tile_n; j += kRsBlock) {
        const K k2 = lkey[j];
        const uint32_t d = static_cast<uint32_t>(k2 >> shift) & 255u;
        const int64_t pos = goff[d] + (j - static_cast<int64_t>(toff[d]));
        kout[pos] = k2;
        vout[pos] = lval[j];
    }
}

template <class K>
__global__ void copy_pairs(const K* __restrict__ kin, const uint32_t* __restrict__ vin, K* __restrict__ kout,
                           uint32_t* __restrict__ vout, int64_t n) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        kout[i] = kin[i];
        vout[i] = vin ? vin[i] : static_cast<uint32_t>(i);
    }
}

// Small sorts (n <= kBsMax, e.g. the deep SparseConvUnet levels) in ONE
// workgroup: bitonic network over (key & mask, input position) in LDS, so the
// result is the stable LSD order without the 3-4 launches per radix pass.
constexpr int kBsMax = 8192;
constexpr int kBsThreads = 1024;

// Element i lives in thread i % 1024, register slot i / 1024, so a
// compare-exchange partner i ^ j is the same thread's other slot for
// j >= 1024 (register swap), another lane of the same wave for j < 64
// (__shfl_xor), and only for 64 <= j < 1024 another wave (through LDS, two
// barriers): 22 of the 91 stages of an 8192-element network touch LDS.
template <class K, int S>
__global__ void __launch_bounds__(kBsThreads) block_sort_pairs(const K* __restrict__ kin,
                                                               const uint32_t* __restrict__ vin,
                                                               K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                               int n, K mask) {
    constexpr int N = S * kBsThreads;
    __shared__ K sk[N];
    __shared__ uint32_t sp[N];
    const int t = threadIdx.x;
    K key[S];
    uint32_t pos[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int i = s * kBsThreads + t;
        key[s] = i < n ? (kin[i] & mask) : ~K(0);
        pos[s] = i < n ? static_cast<uint32_t>(i) : 0xffffffffu;
    }
    // the element of slot s takes its partner's (ok, op) or keeps its own
    auto settle = [&](int s, int i, int j, int k, K ok, uint32_t op) {
        const bool mine_gt = key[s] > ok || (key[s] == ok && pos[s] > op);
        const bool lower = (i & j) == 0, asc = (i & k) == 0;
        const bool keep = (lower == asc) ? !mine_gt : mine_gt;
        if (!keep) {
            key[s] = ok;
            pos[s] = op;
        }
    };
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= kBsThreads) {  // same thread, slots s and s ^ (j / 1024)
                // slot distance as a compile-time constant: the register
                // arrays are never indexed dynamically (that would spill them)
                auto slots = [&](auto js_c) {
                    constexpr int js = decltype(js_c)::value;
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        if ((s & js) || (s | js) >= S) continue;
                        const int s2 = s | js;
                        const int i = s * kBsThreads + t;
                        const bool gt = key[s] > key[s2] || (key[s] == key[s2] && pos[s] > pos[s2]);
                        if (gt == ((i & k) == 0)) {
                            const K tk = key[s];
                            key[s] = key[s2];
                            key[s2] = tk;
                            const uint32_t tp = pos[s];
                            pos[s] = pos[s2];
                            pos[s2] = tp;
                        }
                    }
                };
                const int js = j / kBsThreads;
                if (js == 1) slots(std::integral_constant<int, 1>{});
                else if (js == 2) slots(std::integral_constant<int, 2>{});
                else slots(std::integral_constant<int, 4>{});
            } else if (j < 64) {  // same wave
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const K ok = __shfl_xor(key[s], j, 64);
                    const uint32_t op = __shfl_xor(pos[s], j, 64);
                    settle(s, s * kBsThreads + t, j, k, ok, op);
                }
            } else {  // another wave of the workgroup
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    sk[s * kBsThreads + t] = key[s];
                    sp[s * kBsThreads + t] = pos[s];
                }
                __syncthreads();
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const int i = s * kBsThreads + t;
                    settle(s, i, j, k, sk[i ^ j], sp[i ^ j]);
                }
                __syncthreads();
            }
        }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int i = s * kBsThreads + t;
        if (i < n) {
            kout[i] = kin[pos[s]];
            vout[i] = vin ? vin[pos[s]] : pos[s];
        }
    }
}

// Small sorts by LSD radix in ONE workgroup (the default; O3DML_BS_KIND=1 runs
// the bitonic network above): 4-bit digits, and only the digits in which the
// keys differ (the OR of key ^ key[0] over the input) — the SparseConvUnet grid
// keys (three 20-bit fields, a few bits varying in each) take 6 passes, not 16.
// Each pass is a stable counting pass: digit counters in thread-private LDS
// columns (u16 pairs packed in a u32), a packed wave scan of the thread's 8
// counter words, wave totals through LDS, then the ranked scatter into the
// exchange buffer.  Element i lives in thread i / S, slot i % S (blocked), so
// counting a thread's slots in order keeps equal digits in input order.
// Padding slots (pos = ~0) take digit 15 in every pass: they start last and
// stay last.  N <= 8,192 keeps every rank and packed sum within 16 bits.
template <class K, int S>
__global__ void __launch_bounds__(kBsThreads) block_radix_sort_pairs(const K* __restrict__ kin,
                                                                     const uint32_t* __restrict__ vin,
                                                                     K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                                     int n, K mask) {
    constexpr int N = S * kBsThreads;
    constexpr int kWaves = kBsThreads / 64;
    static_assert(N <= 8192, "packed 16-bit counters");
    // exchange buffers padded by one slot per 32 (bpad): a thread's S
    // consecutive slots no longer start on the same few banks as its neighbours'
    __shared__ K xk[N + N / 32];
    __shared__ uint32_t xp[N + N / 32];
    auto bpad = [](int i) { return i + (i >> 5); };
    __shared__ uint32_t cnt[8 * kBsThreads];  // [digit pair][thread]
    __shared__ uint32_t wtot[kWaves][8];
    __shared__ K wor[kWaves];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int s = 0; s < S; ++s) {  // coalesced load, blocked read below
        const int i = s * kBsThreads + t;
        xk[bpad(i)] = i < n ? (kin[i] & mask) : K(0);
    }
    __syncthreads();
    const K k0 = xk[0];  // bpad(0) = 0
    K key[S];
    uint32_t pos[S];
    K vb = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int i = t * S + s;
        key[s] = xk[bpad(i)];
        pos[s] = i < n ? static_cast<uint32_t>(i) : 0xffffffffu;
        if (i < n) vb |= key[s] ^ k0;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) vb |= __shfl_xor(vb, d, 64);
    if (lane == 0) wor[w] = vb;
    __syncthreads();
    K vbits = 0;
#pragma unroll
    for (int v = 0; v < kWaves; ++v) vbits |= wor[v];
    for (int sh = 0; sh < static_cast<int>(8 * sizeof(K)); sh += 4) {
        if (((vbits >> sh) & K(15)) == 0) continue;  // uniform: this digit is the same everywhere
#pragma unroll
        for (int j = 0; j < 8; ++j) cnt[j * kBsThreads + t] = 0u;
        uint32_t dg[S], lr[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t d = pos[s] != 0xffffffffu ? static_cast<uint32_t>(key[s] >> sh) & 15u : 15u;
            dg[s] = d;
            const int a = static_cast<int>(d >> 1) * kBsThreads + t;
            const int hs = static_cast<int>(d & 1u) * 16;
            const uint32_t v = cnt[a];
            lr[s] = (v >> hs) & 0xffffu;
            cnt[a] = v + (1u << hs);
        }
        uint32_t c[8], x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c[j] = cnt[j * kBsThreads + t];
            x[j] = wave_inclusive_scan(c[j]);
        }
        if (lane == 63) {
#pragma unroll
            for (int j = 0; j < 8; ++j) wtot[w][j] = x[j];
        }
        __syncthreads();
        uint32_t base = 0;  // elements of all digits below 2j
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t wp = 0, tot = 0;
#pragma unroll
            for (int v = 0; v < kWaves; ++v) {
                const uint32_t y = wtot[v][j];
                wp += v < w ? y : 0u;
                tot += y;
            }
            const uint32_t ex = wp + x[j] - c[j];
            const uint32_t lo = tot & 0xffffu;
            const uint32_t p0 = (ex & 0xffffu) + base, p1 = (ex >> 16) + base + lo;
            cnt[j * kBsThreads + t] = p0 | (p1 << 16);
            base += lo + (tot >> 16);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t v = cnt[static_cast<int>(dg[s] >> 1) * kBsThreads + t];
            const uint32_t r = ((v >> ((dg[s] & 1u) * 16)) & 0xffffu) + lr[s];
            xk[bpad(static_cast<int>(r))] = key[s];
            xp[bpad(static_cast<int>(r))] = pos[s];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < S; ++s) {
            key[s] = xk[bpad(t * S + s)];
            pos[s] = xp[bpad(t * S + s)];
        }
        __syncthreads();  // exchange buffer and wave totals free for the next pass
    }
#pragma unroll
    for (int s = 0; s < S; ++s) xp[bpad(t * S + s)] = pos[s];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int i = s * kBsThreads + t;
        if (i < n) {
            const uint32_t p = xp[bpad(i)];
            kout[i] = kin[p];
            vout[i] = vin ? vin[p] : p;
        }
    }
}

// Small-sort kind: 0 = LSD radix in one workgroup (default), 1 = bitonic
// (O3DML_BS_KIND, A/B); a call may pick one (small_kind >= 0: o3dml_sort_pairs
// for the tests) — an argument, not process state, so concurrent host
// threads never see another call's choice
inline int block_sort_kind(int small_kind = -1) {
    static const int v = [] {
        const char* e = std::getenv("O3DML_BS_KIND");
        return e ? std::atoi(e) : 0;
    }();
    return small_kind >= 0 ? small_kind : v;
}

// Largest n sorted in one workgroup: O3DML_BS_MAX (A/B), default kBsMax
inline int64_t block_sort_max() {
    static const int64_t v = [] {
        const char* e = std::getenv("O3DML_BS_MAX");
        const int64_t x = e ? std::atoll(e) : kBsMax;
        return x < 0 ? 0 : (x > kBsMax ? kBsMax : x);
    }();
    return v;
}

// Largest tile count whose scatter sums its own digit bases (no
// radix_digit_scan launch): O3DML_RS_FUSED_TILES (A/B; 0 = never), default 64
// (n <= 131,072 keys: every block reads the 256 x tiles histogram, <= 64 KiB)
inline int64_t rs_fused_tiles() {
    static const int64_t v = [] {
        const char* e = std::getenv("O3DML_RS_FUSED_TILES");
        return e ? std::atoll(e) : 64;
    }();
    return v;
}

inline int bits_needed(uint64_t max_key) {
    int b = 0;
    while (b < 64 && (max_key >> b) != 0) ++b;
    return b;
}

template <class K>
size_t radix_sort_workspace_bytes(int64_t n) {
    const int64_t tiles = ceil_div(n > 0 ? n : 1, kRsTile);
    return ws_bytes<K>(n) + ws_bytes<uint32_t>(n) + 2 * ws_bytes<uint32_t>(256 * tiles) + ws_bytes<uint32_t>(256);
}

// Sorts (keys_in, vals_in) by key bits [0, end_bit) into (keys_out, vals_out).
// vals_in == nullptr means the payload is the element index (iota).
// keys_in must not alias keys_out.
// or_and (nullable, device [2]): OR of all n keys and OR of their
// complements (the bits that vary: both set) — the passes whose
// digit does not vary then return at once (device-planned, see device_pass):
// the launches stay, their work goes.  For keys of which the host knows only a
// generous bit width (packed coordinates).
template <class K>
void radix_sort_pairs(const K* keys_in, const uint32_t* vals_in, K* keys_out, uint32_t* vals_out,
                      int64_t n, int end_bit, Workspace& ws, hipStream_t st, int small_kind = -1,
                      const uint64_t* or_and = nullptr) {
    if (n <= 0) return;
    const int passes = (end_bit + 7) / 8;
    if (passes == 0 || n == 1) {
        copy_pairs<K><<<stream_grid(n, 256), 256, 0, st>>>(keys_in, vals_in, keys_out, vals_out, n);
        O3DML_LAUNCH_CHECK();
        return;
    }
    if (n <= block_sort_max()) {
        const K mask = end_bit >= static_cast<int>(8 * sizeof(K)) ? ~K(0) : ((K(1) << end_bit) - 1);
        // (a merge-path merge sort of packed (key, position) words measured
        // slower: 46 vs 37 us at ~4k keys — dependent LDS latency of the
        // per-round binary searches)
        const int ni = static_cast<int>(n);
        if (block_sort_kind(small_kind) == 0) {
            if (n <= kBsThreads)
                block_radix_sort_pairs<K, 1><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
            else if (n <= 2 * kBsThreads)
                block_radix_sort_pairs<K, 2><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
            else if (n <= 4 * kBsThreads)
                block_radix_sort_pairs<K, 4><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
            else
                block_radix_sort_pairs<K, 8><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
        } else if (n <= kBsThreads)
            block_sort_pairs<K, 1><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
        else if (n <= 2 * kBsThreads)
            block_sort_pairs<K, 2><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
        else if (n <= 4 * kBsThreads)
            block_sort_pairs<K, 4><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
        else
            block_sort_pairs<K, 8><<<1, kBsThreads, 0, st>>>(keys_in, vals_in, keys_out, vals_out, ni, mask);
        O3DML_LAUNCH_CHECK();
        return;
    }
    const int64_t tiles = ceil_div(n, kRsTile);
    // up to kRsFusedTiles tiles the scatter sums its digit bases from the
    // histogram itself (radix_digit_scan skipped: 2 launches per pass, not 3)
    const bool fused = tiles <= rs_fused_tiles();
    K* ktmp = ws.take<K>(n);
    uint32_t* vtmp = ws.take<uint32_t>(n);
    uint32_t* hist = ws.take<uint32_t>(256 * tiles);
    uint32_t* offs = ws.take<uint32_t>(256 * tiles);
    uint32_t* dtot = ws.take<uint32_t>(256);
    if (or_and) {
        for (int p = 0; p < passes; ++p) {
            const int shift = 8 * p;
            radix_hist<K><<<static_cast<unsigned>(tiles), kRsBlock, 0, st>>>(keys_in, n, shift, hist, tiles, or_and,
                                                                             passes, ktmp, keys_out);
            O3DML_LAUNCH_CHECK();
            if (!fused) {
                radix_digit_scan<<<256, kRsBlock, 0, st>>>(hist, tiles, offs, dtot, or_and, p);
                O3DML_LAUNCH_CHECK();
            }
            radix_scatter<K><<<static_cast<unsigned>(tiles), kRsBlock, 0, st>>>(
                    keys_in, vals_in, nullptr, nullptr, n, shift, fused ? nullptr : offs, dtot, hist, tiles, or_and,
                    passes, ktmp, vtmp, keys_out, vals_out);
            O3DML_LAUNCH_CHECK();
        }
        return;
    }
    const K* ksrc = keys_in;
    const uint32_t* vsrc = vals_in;
    for (int p = 0; p < passes; ++p) {
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        K* kdst = to_out ? keys_out : ktmp;
        uint32_t* vdst = to_out ? vals_out : vtmp;
        const int shift = 8 * p;
        radix_hist<K><<<static_cast<unsigned>(tiles), kRsBlock, 0, st>>>(ksrc, n, shift, hist, tiles);
        O3DML_LAUNCH_CHECK();
        if (!fused) {
            radix_digit_scan<<<256, kRsBlock, 0, st>>>(hist, tiles, offs, dtot);
            O3DML_LAUNCH_CHECK();
        }
        radix_scatter<K><<<static_cast<unsigned>(tiles), kRsBlock, 0, st>>>(ksrc, vsrc, kdst, vdst, n, shift,
                                                                          fused ? nullptr : offs, dtot, hist, tiles);
        O3DML_LAUNCH_CHECK();
        ksrc = kdst;
        vsrc = vdst;
    }
}

// Segment starts of a sorted key array: off[s] = first position whose key is
// >= s (lower bound), for s in [0, nseg]; keys >= nseg sort after every
// segment.  One thread per segment boundary (binary search).
template <class K>
__global__ void segment_offsets_kernel(const K* __restrict__ skeys, int64_t total, int64_t nseg,
                                       int64_t* __restrict__ off) {
    for (int64_t s = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; s <= nseg;
         s += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        int64_t lo = 0, hi = total;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (static_cast<int64_t>(skeys[mid]) < s) lo = mid + 1;
            else hi = mid;
        }
        off[s] = lo;
    }
}

// Inverse of a scatter: pairs whose destination is keys[p] (keys >= nseg are
// dropped) grouped by destination in ascending p (the sort is stable).  Lets a
// scatter-add become a fixed-order gather (run-to-run bitwise identical).
struct Inverse {
    const uint32_t* pairs;  // pair ids, grouped by destination
    const int64_t* off;     // [nseg + 1] group starts
};

inline size_t inverse_workspace_bytes(int64_t total, int64_t nseg) {
    return 3 * ws_bytes<uint32_t>(total) + ws_bytes<int64_t>(nseg + 1) + radix_sort_workspace_bytes<uint32_t>(total);
}

// keys: [total] destination per pair, in workspace-owned or caller memory
inline Inverse build_inverse(const uint32_t* keys, int64_t total, int64_t nseg, Workspace& ws, hipStream_t st) {
    O3DML_REQUIRE(total < (int64_t(1) << 32) && nseg < (int64_t(1) << 32) - 1,
                  "inverse: %lld pairs / %lld groups exceed 32-bit ids", (long long)total, (long long)nseg);
    uint32_t* skeys = ws.take<uint32_t>(total);
    uint32_t* pairs = ws.take<uint32_t>(total);
    int64_t* off = ws.take<int64_t>(nseg + 1);
    radix_sort_pairs<uint32_t>(keys, nullptr, skeys, pairs, total, bits_needed(static_cast<uint64_t>(nseg)), ws, st);
    segment_offsets_kernel<uint32_t><<<stream_grid(nseg + 1, 256), 256, 0, st>>>(skeys, total, nseg, off);
    O3DML_LAUNCH_CHECK();
    return Inverse{pairs, off};
}

}  // namespace prim
}  // namespace o3dml
