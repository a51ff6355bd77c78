// sparse_conv.hip — SparseConv / SparseConvTranspose gather-GEMM-scatter on
// MFMA, replacing open3d.ml.torch.ops.sparse_conv,
// sparse_conv_transpose and their gradients as bound by layers.SparseConv /
// layers.SparseConvTranspose (ml3d/torch/models/sparseconvnet.py:344-482).
//
// Data flow (all device):
//   CSR pairs (neighbors_index, neighbors_kernel_index, neighbors_row_splits)
//     -> dense kernel map  map[o*K + k] = input row or -1   (build_kernel_map)
//   forward  out[o,:] = oscale[o] * sum_k (src[map[o,k],:] * sscale[i] * pscale[o,k]) @ W[k] + bias
//            output-stationary implicit GEMM: a wave owns 32 output rows x 32
//            output channels, walks the K offsets its rows use and Cin in
//            32-channel stages, operands gathered straight into the
//            v_mfma_f32_32x32x2_f32 registers (exact fp32 FMA chains); when the
//            tiles cannot fill the chip the (offset, Cin) stages are split
//            across waves and the partials reduced in a fixed order.  No
//            atomics -> deterministic.  Optional eval prologue (folded
//            BatchNorm + ReLU on the gathered rows) and residual epilogue.
//   dIn      the same kernel on the inverse map inv[i*K+k] = o with W^T.
//   dW       per offset k the pair list (o, i) (k-major compaction of the map);
//            dW[k] = sum_j src[i_j]^T g[o_j], one wave per 32x32 tile and pair
//            chunk with the pairs as the MFMA reduction index (operands gathered
//            straight into registers), chunk slabs reduced in a fixed order.
// Roofline: MFMA fp32 (157 TF/s dense) for Cin*Cout >= ~64^2, gather/HBM bound
// below that.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <array>
#include <vector>

#include "counters.hpp"
#include "primitives.hpp"

namespace o3dml {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef O3DML_GEMM_THREADS
#define O3DML_GEMM_THREADS 256
#endif
constexpr int kGemmThreads = O3DML_GEMM_THREADS;  // 4 waves

// --------------------------------------------------------------------------
// kernel maps
// --------------------------------------------------------------------------
__global__ void build_kernel_map_kernel(const int32_t* __restrict__ nbr, const int32_t* __restrict__ kidx,
                                        const float* __restrict__ nimp, const int64_t* __restrict__ rs, int64_t n_out,
                                        int64_t n_in, int K, int32_t* __restrict__ map, float* __restrict__ pscale,
                                        float* __restrict__ norm, int* __restrict__ dup) {
    for (int64_t o = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; o < n_out;
         o += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float s = 0.f;
        for (int64_t e = rs[o], ee = rs[o + 1]; e < ee; ++e) {
            const int k = kidx[e];
            if (k < 0 || k >= K) {
                atomicOr(dup, 2);
                continue;
            }
            const int32_t nb = nbr[e];
            if (nb < 0 || nb >= n_in) {  // would address past the features (and the inverse map)
                atomicOr(dup, 8);
                continue;
            }
            int32_t* slot = map + o * K + k;
            if (*slot >= 0) {
                atomicOr(dup, 1);  // two pairs share (o, k): dense map impossible
                continue;
            }
            *slot = nb;
            const float w = nimp ? nimp[e] : 1.f;
            if (pscale) pscale[o * K + k] = w;
            s += w;
        }
        if (norm) norm[o] = s;
    }
}

// inv [n_in, K]: an entry i >= n_in (a map built for other sizes than the
// caller states, e.g. a transpose_map partner) is dropped and flagged as
// build_map does (status bit 8), never written past the inverse map
__global__ void build_inverse_map_kernel(const int32_t* __restrict__ map, const float* __restrict__ pscale,
                                         int64_t n_out, int K, int64_t n_in, int32_t* __restrict__ inv,
                                         float* __restrict__ ipscale, int* __restrict__ dup) {
    const int64_t total = n_out * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int32_t i = map[e];
        if (i < 0) continue;
        if (i >= n_in) {
            atomicOr(dup, 8);
            continue;
        }
        const int64_t o = e / K;
        const int k = static_cast<int>(e - o * K);
        const int32_t prev = atomicCAS(inv + static_cast<int64_t>(i) * K + k, -1, static_cast<int32_t>(o));
        if (prev != -1) atomicOr(dup, 1);
        if (ipscale && pscale) ipscale[static_cast<int64_t>(i) * K + k] = pscale[e];
    }
}

__global__ void recip_norm_kernel(const float* __restrict__ norm, const float* __restrict__ mul, int64_t n,
                                  float* __restrict__ out) {
    for (int64_t o = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; o < n;
         o += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float s = norm ? (norm[o] != 0.f ? 1.f / norm[o] : 1.f) : 1.f;
        if (mul) s *= mul[o];
        out[o] = s;
    }
}

// --------------------------------------------------------------------------
// tile order: the GEMM wave walks the UNION of the offsets its 32 rows use, so
// rows with different neighbour masks in one tile cost MFMA work on zero
// operands (C4 room voxels in voxelize order: 67 % useful).  The rows are
// stably sorted by a 16-bit hash of their offset mask once per map; tiles then
// take 32 consecutive rows of that order (98 % useful), spatial order kept
// within a mask class.  Absent offsets only ever added exact zeros, so the
// per-row sums are unchanged.
// --------------------------------------------------------------------------
constexpr int64_t kOrderMinRows = 2048;
// O3DML_TILE_ORDER=0: no tile orders (rows in map order; A/B)
static bool use_order(int64_t n, int K) {
    static const bool on = [] {
        const char* e = std::getenv("O3DML_TILE_ORDER");
        return !(e && e[0] == '0');
    }();
    return on && K > 8 && n >= kOrderMinRows;
}

// Grids of the GEMM kernels.  O3DML_GEMM_XCD=1: a multiple of 8 workgroups,
// so xcd_block() hands each XCD one contiguous range of tiles (the extra
// workgroups exit at once).  OFF by default: same-session A/B on the C4 room
// (tools/gemm_probe.py, with and without the chunked tile order below) was
// neutral to 4 % slower at 32->32, 64->32 and 128->128 — the gathers' L2
// locality is not what bounds these kernels.  Off: an odd grid, so
// xcd_block() keeps blockIdx.x.
static int64_t round8(int64_t g) {
    static const bool on = [] {
        const char* e = std::getenv("O3DML_GEMM_XCD");
        return e ? std::atoi(e) != 0 : false;
    }();
    if (!on) return g | 1;  // odd: xcd_block() falls back to blockIdx.x
    return (g + 7) & ~int64_t(7);
}

// Tile order: rows grouped by their offset mask, globally (default) or inside
// chunks of O3DML_ORDER_CHUNK consecutive rows (rows come in voxel order, so
// a chunk is a spatial slab that keeps a tile's or an XCD's gathers local).
// Chunks measured neutral (4,096 rows) to 10 % slower (1,024) — kept off.
static int order_chunk_log() {
    static const int v = [] {
        const char* e = std::getenv("O3DML_ORDER_CHUNK");
        const int c = e ? std::atoi(e) : 0;
        if (c <= 0) return 0;
        int l = 0;
        while ((1 << (l + 1)) <= c) ++l;
        return l;
    }();
    return v;
}

// key = (chunk, hb-bit hash of the offset mask): 16 bits in all while the
// chunks allow it (two radix passes), never fewer than 10 hash bits
__global__ void mask_keys_kernel(const int32_t* __restrict__ map, int64_t n, int K, int chunk_log, int hb,
                                 uint32_t* __restrict__ keys, int* __restrict__ flag) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *flag = 1;  // the sort below completes before any GEMM reads it
    for (int64_t o = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; o < n;
         o += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        uint32_t m = 0u;
        for (int k = 0; k < K; ++k) m |= (map[o * K + k] >= 0 ? 1u : 0u) << k;
        const uint32_t chunk = chunk_log ? static_cast<uint32_t>(o >> chunk_log) : 0u;
        keys[o] = (chunk << hb) | ((m * 0x9E3779B1u) >> (32 - hb));
    }
}

static size_t order_scratch_bytes(int64_t n) {
    return 2 * ws_bytes<uint32_t>(n) + prim::radix_sort_workspace_bytes<uint32_t>(n);
}

// The map rows in tile order, tmap[j] = map[order[j]], padded with -1 rows to
// whole 128-row blocks (the largest GEMM tile): a GEMM wave reads its tile's
// map rows as one contiguous block, issued at once with (not after) its read
// of the order.
constexpr int64_t kTileMapPad = 128;
// O3DML_GEMM_TILE_MAP=0: no tile-order map copy; tiles read the map through the order (A/B)
static bool use_tile_map() {
    static const bool on = [] {
        const char* e = std::getenv("O3DML_GEMM_TILE_MAP");
        return !(e && e[0] == '0');
    }();
    return on;
}
static int64_t tile_map_entries(int64_t n, int K) { return ((n + kTileMapPad - 1) & ~(kTileMapPad - 1)) * K; }
__global__ void tile_map_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ order, int64_t n, int K,
                                int32_t* __restrict__ tmap) {
    const int64_t tot = ((n + kTileMapPad - 1) & ~(kTileMapPad - 1)) * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < tot;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t j = e / K;
        tmap[e] = j < n ? map[static_cast<int64_t>(order[j]) * K + (e - j * K)] : -1;
    }
}

static void build_order(const int32_t* map, int64_t n, int K, int32_t* order, int32_t* tmap, int* flag,
                        Workspace scratch, hipStream_t st) {
    if (!use_order(n, K)) return;
    uint32_t* kin = scratch.take<uint32_t>(n);
    uint32_t* kout = scratch.take<uint32_t>(n);
    const int cl = order_chunk_log();
    const int cb = cl ? prim::bits_needed(static_cast<uint64_t>((n - 1) >> cl)) : 0;
    const int hb = std::max(10, 16 - cb);
    mask_keys_kernel<<<stream_grid(n, 256), 256, 0, st>>>(map, n, K, cl, hb, kin, flag);
    O3DML_LAUNCH_CHECK();
    const int bits = hb + cb;
    O3DML_REQUIRE(bits <= 32, "tile order: too many row chunks");
    prim::radix_sort_pairs<uint32_t>(kin, nullptr, kout, reinterpret_cast<uint32_t*>(order), n, bits, scratch, st);
    if (use_tile_map()) {
        tile_map_kernel<<<stream_grid(tile_map_entries(n, K), 256), 256, 0, st>>>(map, order, n, K, tmap);
        O3DML_LAUNCH_CHECK();
    }
}

// W [K][Cin][Cout] -> Wt [K][Cout][Cin]
__global__ void transpose_filters_kernel(const float* __restrict__ w, int K, int cin, int cout, float* __restrict__ wt) {
    const int64_t total = static_cast<int64_t>(K) * cin * cout;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = e / (static_cast<int64_t>(cin) * cout);
        const int64_t r = e - k * cin * cout;
        const int64_t a = r / cout, c = r - a * cout;
        wt[(k * cout + c) * cin + a] = w[e];
    }
}

// --------------------------------------------------------------------------
// implicit GEMM (forward / dIn): one wave owns 32 output rows x 32 output
// channels and walks the (offset, Cin-chunk) stages its rows use.  Operands go
// straight from global memory into registers in the MFMA layout — lane (i, h)
// gathers 16 consecutive channels [c0 + 16h, +16) of row i's input (4 x 16-B
// loads) and the matching 16 weights of column i — so no LDS and no barriers;
// the next stage's loads are issued before the current stage's 16
// v_mfma_f32_32x32x2_f32 (reduction index permuted consistently on A and B:
// step s pairs channels c0+s and c0+16+s), hiding the gather latency.
// --------------------------------------------------------------------------
struct GemmStage {
    float a[16], b[16];
    bf16x8 bs[6];  // filters split once per call (BS kernels): hi, mid, lo of channels 8t.. for t = 0, 1
    float s1, s2;  // row importance, pair scale (1 without them)
    float v;       // 1 for a present neighbour, 0 for a missing one
};

// Optional prologue on the gathered rows (eval-mode BatchNorm + ReLU of the
// layer input, folded to a per-channel affine): a = relu(x * ps[c] + pb[c]),
// staged once per workgroup in LDS.  Missing neighbours stay exactly 0
// (row factor 0), as the zero padding of the activated features.
struct GemmPrologue {
    const float* scale;  // [cin] or null
    const float* shift;  // [cin]
    // byte sizes of the gathered rows and of the filters: the num_records of
    // the buffer resources (BUF kernels), so a row index past the operand
    // reads zeros, never foreign memory (set by the launcher)
    uint32_t src_bytes = 0, w_bytes = 0;
    // the filters split into bf16 hi / mid / lo once per call (split_filters_kernel;
    // BS kernels) and the byte size of that copy
    const __bf16* wsplit = nullptr;
    uint32_t wsplit_bytes = 0;
    // the map rows in tile order (tile_map_kernel; valid with the order):
    // implicit_gemm_lds_kernel loads its tile's rows from here
    const int32_t* tmap = nullptr;
    // persistent grid (implicit_gemm_lds_kernel): the column blocks of the
    // work when the grid holds only the resident waves, each looping over
    // (tile, split, column block) items; 0 = one wave per item
    int pcols = 0;
};
constexpr int kPreMax = 1024;  // max cin with a prologue (LDS staging)

__device__ __forceinline__ float pre_act(float v, float s, float b) { return fmaxf(fmaf(v, s, b), 0.f); }

// Every load below is unconditional and its value is used unconditionally:
// lanes without data (missing neighbour, channel or column past the end) read
// from a zero page instead.  A select of "valid ? load : 0" lets the compiler
// sink the load into a branch with a vmcnt(0) wait per load, which serialises
// the stage's loads instead of keeping them in flight.  All arithmetic on the
// loaded values happens in gemm_finish, after the previous stage's MFMAs.
__device__ __attribute__((aligned(16))) float g_zero_page[16];
__device__ float g_one_page[1] = {1.f};

template <bool VEC4>
__device__ __forceinline__ void gemm_load(GemmStage& st, int32_t m, int K, int64_t o, int k, int c0, int h, int col,
                                          const float* __restrict__ src, const float* __restrict__ sscale,
                                          const float* __restrict__ pscale, const float* __restrict__ Wt, int cin,
                                          int cout, bool live = true) {
    const int cb = c0 + 16 * h;
    const bool valid = m >= 0;
    const int64_t mr = valid ? m : 0;
    // scales: pointer selects (no branch, so the waitcnt placement stays exact);
    // they are uniform per launch, the loads hit a one-word page without them
    st.s1 = *(sscale ? sscale + mr : g_one_page);
    st.s2 = *(pscale ? pscale + (valid ? o : 0) * K + k : g_one_page);
    st.v = valid ? 1.f : 0.f;
    const float* row = src + mr * cin;
    if (VEC4) {  // cin % 4 == 0: float4 granules
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cb + 4 * q;
            const float4 v = *reinterpret_cast<const float4*>((valid && c < cin) ? row + c : g_zero_page);
            st.a[4 * q] = v.x;
            st.a[4 * q + 1] = v.y;
            st.a[4 * q + 2] = v.z;
            st.a[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) st.a[s] = *((valid && cb + s < cin) ? row + cb + s : g_zero_page);
    }
    // B from the transposed filters Wt[k][col][c]: column col's 16 weights are
    // contiguous, so the same four 16-B loads as the A side
    const bool colv = live && col < cout;  // a dead stage reads only the zero page
    const float* wr = Wt + (static_cast<int64_t>(k) * cout + (colv ? col : 0)) * cin;
    if (VEC4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cb + 4 * q;
            const float4 v = *reinterpret_cast<const float4*>((colv && c < cin) ? wr + c : g_zero_page);
            st.b[4 * q] = v.x;
            st.b[4 * q + 1] = v.y;
            st.b[4 * q + 2] = v.z;
            st.b[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) st.b[s] = *((colv && cb + s < cin) ? wr + cb + s : g_zero_page);
    }
}

// Split s of nsplit owns the global stages (offset k, chunk c), g = k*nch + c,
// in [s*G/nsplit, (s+1)*G/nsplit) with G = K*nch — a partition of the
// (offset, Cin) reduction that does not depend on which rows share a tile, so
// every row's partial sums (and the fixed-order reduce) are the same for any
// tile order.  Returns the number of the wave's used stages before split s.
__device__ __forceinline__ int split_stage(unsigned used, int nch, int K, int s, int nsplit) {
    const int g = static_cast<int>(static_cast<int64_t>(s) * K * nch / nsplit);
    const int kk = g / nch, cc = g - kk * nch;
    const unsigned below = kk >= 32 ? used : (used & ((1u << kk) - 1u));
    const bool own = kk < 32 && ((used >> kk) & 1u);
    return __builtin_popcount(below) * nch + (own ? cc : 0);
}

template <bool PRE, bool SC = true>
__device__ __forceinline__ void gemm_finish(GemmStage& st, int c0, int h, const float* lps, const float* lpb) {
    // no prologue and no scales: the factor is 1, and a missing row was
    // gathered from the zero page already — nothing to do (same bits)
    if constexpr (!PRE && !SC) return;
    const int cb = c0 + 16 * h;
    const float sc = st.v != 0.f ? st.s1 * st.s2 : 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) st.a[s] = (PRE ? pre_act(st.a[s], lps[cb + s], lpb[cb + s]) : st.a[s]) * sc;
}

// Split-K store: the wave writes its raw 32 x 32 partial tile into slab s;
// with tile counters (counters.hpp) the LAST of the nsplit waves owning the
// tile then sums the slabs in split order and applies split_reduce_kernel's
// epilogue (same arithmetic, same bits) — no reduce launch.  orow32: the 32
// output rows of the tile (-1 = none).
__device__ __forceinline__ void split_store_finish(const f32x16& acc, const int32_t* orow32, int h, int col,
                                                   int lane, int s, int nsplit, int64_t n_out, int cout,
                                                   float* __restrict__ part, uint32_t* __restrict__ counters,
                                                   int64_t tile, const float* __restrict__ oscale,
                                                   const float* __restrict__ bias,
                                                   const float* __restrict__ residual, float* __restrict__ out) {
    const int64_t total = n_out * cout;
    float* P = part + static_cast<int64_t>(s) * total;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t orr = orow32[(r & 3) + 8 * (r >> 2) + 4 * h];
        if (orr >= 0 && col < cout) {
            if (counters)  // agent-scope store: written through to the device-coherent level
                __hip_atomic_store(P + orr * cout + col, acc[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                P[orr * cout + col] = acc[r];
        }
    }
    if (!counters) return;  // split_reduce_kernel finishes
    // arrival once the slab stores are complete (no device-scope fence: on the
    // 8-XCD part it writes back the whole L2 per wave); the last wave reads
    // the slabs with agent-scope loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t prev = 0;
    if (lane == 0) prev = atomicAdd(counters + tile, 1u);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev != static_cast<uint32_t>(nsplit - 1)) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t orr = orow32[(r & 3) + 8 * (r >> 2) + 4 * h];
        if (orr >= 0 && col < cout) {
            const int64_t e = orr * cout + col;
            float v = 0.f;
            for (int sp = 0; sp < nsplit; ++sp)
                v += __hip_atomic_load(part + sp * total + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (oscale) v *= oscale[orr];
            if (bias) v += bias[col];
            if (residual) v += residual[e];
            out[e] = v;
        }
    }
    if (lane == 0) atomicExch(counters + tile, 0u);  // ready for the next launch
}

// The map rows of a tile into LDS with every global load in flight at once:
// thread t of T takes the entries e = t + T * it (K <= 32 bounds their number
// at compile time), a dead entry's address is clamped to map[0] so that each
// load is unconditional, and the LDS stores follow.  (The plain loop over e
// waited for each load before issuing the next: 14 serialised map-load
// latencies per wave at 32 rows x 27 offsets, ahead of the first gather.)
template <int ROWS, int T>
__device__ __forceinline__ void load_map_tile(const int32_t* __restrict__ map, const int32_t* orow, int K, int t,
                                              int32_t* mtile) {
    constexpr int kIt = (ROWS * 32 + T - 1) / T;
    const int tot = ROWS * K;
    // e / K through a float reciprocal: exact here (e < 2,048, K <= 32, so
    // (e + 0.5) / K stays >= 1/64 away from an integer)
    const float invk = 1.0f / static_cast<float>(K);
    int32_t v[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int e = t + T * it;
        int rr = static_cast<int>((static_cast<float>(e) + 0.5f) * invk);
        rr = rr < ROWS ? rr : ROWS - 1;
        const int32_t orr = e < tot ? orow[rr] : -1;
        const int64_t a = orr >= 0 ? static_cast<int64_t>(orr) * K + (e - rr * K) : 0;
        const int32_t m = map[a];
        v[it] = orr >= 0 ? m : -1;
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int e = t + T * it;
        if (e < tot) mtile[e] = v[it];
    }
}

// A tile from the tile-order map copy (tile_map_kernel): its ROWS x K entries
// are contiguous at tm, so thread t of T issues all its loads at once without
// waiting for the order; into LDS as load_map_tile.  Returns the offsets the
// thread's entries use, OR-reduced over its wave: the same bits as a ballot
// over the LDS tile, without its LDS round trips.
template <int ROWS, int T>
struct MapTileRegs {
    int32_t v[(ROWS * 32 + T - 1) / T];
};
// the loads only (values land in registers; map_tile_commit stores them)
template <int ROWS, int T>
__device__ __forceinline__ void map_tile_fetch(const int32_t* __restrict__ tm, int K, int t, MapTileRegs<ROWS, T>& r) {
    constexpr int kIt = (ROWS * 32 + T - 1) / T;
    const int tot = ROWS * K;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int e = t + T * it;
        r.v[it] = tm[e < tot ? e : 0];
    }
}
template <int ROWS, int T>
__device__ __forceinline__ unsigned map_tile_commit(const MapTileRegs<ROWS, T>& r, int K, int t, int32_t* mtile) {
    constexpr int kIt = (ROWS * 32 + T - 1) / T;
    const int tot = ROWS * K;
    const float invk = 1.0f / static_cast<float>(K);  // e / K exact as in load_map_tile
    const int32_t* v = r.v;
    unsigned mask = 0u;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int e = t + T * it;
        if (e < tot) {
            mtile[e] = v[it];
            const int rr = static_cast<int>((static_cast<float>(e) + 0.5f) * invk);
            mask |= v[it] >= 0 ? 1u << (e - rr * K) : 0u;
        }
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) mask |= static_cast<unsigned>(__shfl_xor(static_cast<int>(mask), d));
    return __builtin_amdgcn_readfirstlane(mask);
}
template <int ROWS, int T>
__device__ __forceinline__ unsigned load_map_tile_direct(const int32_t* __restrict__ tm, int K, int t,
                                                         int32_t* mtile) {
    MapTileRegs<ROWS, T> r;
    map_tile_fetch<ROWS, T>(tm, K, t, r);
    return map_tile_commit<ROWS, T>(r, K, t, mtile);
}

template <bool VEC4, bool PRE>
__global__ void __launch_bounds__(kGemmThreads)
implicit_gemm_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ order, const int* order_flag,
                     int K, int64_t n_out,
                     const float* __restrict__ src,
                     const float* __restrict__ sscale, const float* __restrict__ pscale,
                     const float* __restrict__ Wt /*[K][cout][cin]*/, int cin, int cout,
                     const float* __restrict__ oscale, const float* __restrict__ bias, float* __restrict__ out,
                     int nsplit, float* __restrict__ part, GemmPrologue pre, const float* __restrict__ residual,
                     uint32_t* __restrict__ counters) {
    __shared__ float lpre[PRE ? 2 * (kPreMax + 32) : 1];
    float* lps = lpre;
    float* lpb = lpre + (PRE ? kPreMax + 32 : 0);
    if (PRE) {  // channels past cin stay 0 -> relu(0) * factor = 0
        for (int c = threadIdx.x; c < kPreMax + 32; c += kGemmThreads) {
            lps[c] = c < cin ? pre.scale[c] : 0.f;
            lpb[c] = c < cin ? pre.shift[c] : 0.f;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t o0 = (static_cast<int64_t>(blockIdx.x) * (kGemmThreads / 64) + (threadIdx.x >> 6)) * 32;
    if (o0 >= n_out) return;  // whole wave; no barriers below
    const int i = lane & 31, h = lane >> 5;
    const int col = blockIdx.y * 32 + i;
    // the wave's 32 rows: positions o0.. of the tile order (identity without
    // one); their output row ids and map rows -> LDS, offsets in use
    __shared__ int32_t mtile_all[kGemmThreads / 64][32 * 32];
    __shared__ int32_t orow_all[kGemmThreads / 64][32];
    int32_t* mtile = mtile_all[threadIdx.x >> 6];
    int32_t* orow = orow_all[threadIdx.x >> 6];
    if (order && *order_flag == 0) order = nullptr;  // map built without a tile order
    if (lane < 32) {
        const int64_t oo = o0 + lane;
        orow[lane] = oo < n_out ? (order ? order[oo] : static_cast<int32_t>(oo)) : -1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    load_map_tile<32, 64>(map, orow, K, lane, mtile);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    unsigned used = 0u;
    for (int k = h; k < K; k += 2) {  // lanes 0-31 test even k, lanes 32-63 odd k
        const uint64_t b = __ballot(mtile[i * K + k] >= 0);
        used |= ((h ? (b >> 32) : (b & 0xffffffffull)) != 0ull) ? (1u << k) : 0u;
    }
    used |= __builtin_amdgcn_readlane(used, 32) | __builtin_amdgcn_readlane(used, 0);
    const int64_t o = orow[i] >= 0 ? orow[i] : 0;  // this lane's output row (pair scales)
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // the wave's stage stream = (used offset, 32-channel chunk) in order; split
    // s of nsplit takes its stages in [j0, j1) (split_stage)
    const int nch = (cin + 31) >> 5;
    const int s = blockIdx.z;
    const int j0 = split_stage(used, nch, K, s, nsplit);
    const int j1 = split_stage(used, nch, K, s + 1, nsplit);
    if (j0 < j1) {
        unsigned u = used;
        for (int t = j0 / nch; t > 0; --t) u &= u - 1u;
        // two stage buffers in ping-pong (no register copy between stages, so
        // the loads of stage j+1 stay in flight under the MFMAs of stage j)
        auto advance = [&](int& kk, int& cc) {
            cc += 32;
            if (cc >= cin) {
                cc = 0;
                u &= u - 1u;
                kk = u ? __builtin_ctz(u) : 0;
            }
        };
        GemmStage sa, sb;
        int ka = __builtin_ctz(u), ca = (j0 % nch) * 32, kb = 0, cb = 0;
        gemm_load<VEC4>(sa, mtile[i * K + ka], K, o, ka, ca, h, col, src, sscale, pscale, Wt, cin, cout);
        for (int j = j0;; j += 2) {
            kb = ka;
            cb = ca;
            advance(kb, cb);
            // loads are issued unconditionally (a stage past the end reads the zero
            // page): a skipped load on one path makes the compiler's wait counts
            // conservative at the join and the MFMAs would wait for these loads
            const bool lb = j + 1 < j1;
            gemm_load<VEC4>(sb, lb ? mtile[i * K + kb] : -1, K, o, kb, cb, h, col, src, sscale, pscale, Wt, cin, cout,
                            lb);
            __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs
            gemm_finish<PRE>(sa, ca, h, lps, lpb);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sa.a[r], sa.b[r], acc, 0, 0, 0);
            if (j + 1 >= j1) break;
            ka = kb;
            ca = cb;
            advance(ka, ca);
            const bool la = j + 2 < j1;
            gemm_load<VEC4>(sa, la ? mtile[i * K + ka] : -1, K, o, ka, ca, h, col, src, sscale, pscale, Wt, cin, cout,
                            la);
            __builtin_amdgcn_sched_barrier(0);
            gemm_finish<PRE>(sb, cb, h, lps, lpb);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sb.a[r], sb.b[r], acc, 0, 0, 0);
            if (j + 2 >= j1) break;
        }
    }
    if (nsplit > 1) {  // raw partial sums; the tile's last wave (or split_reduce_kernel) finishes
        split_store_finish(acc, orow, h, col, lane, s, nsplit, n_out, cout, part, counters,
                           (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * (kGemmThreads / 64) +
                                   (threadIdx.x >> 6),
                           oscale, bias, residual, out);
        return;
    }
    // epilogue: C/D map row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t orr = orow[row];
        if (orr >= 0 && col < cout) {
            float v = acc[r];
            if (oscale) v *= oscale[orr];
            if (bias) v += bias[col];
            if (residual) v += residual[orr * cout + col];
            out[orr * cout + col] = v;
        }
    }
}

// --------------------------------------------------------------------------
// implicit GEMM, LDS-staged (cin % 4 == 0, the common case): the same tiles,
// stage order and MFMA reduction order as implicit_gemm_kernel (so the same
// fp32 sums bit for bit), but each stage's operands travel global -> LDS as
// full 128-B lines with global_load_lds_dwordx4 (8 lanes per row, 8 rows per
// instruction) instead of fragment-shaped 16-B loads (32 rows x 16 B per
// instruction, every line touched by 4 instructions): 4x fewer L1 accesses
// per stage, which bounded the register-staged kernel (PMC: 512 TCP accesses
// per 16-MFMA stage, MFMA pipes 34 % busy at 128 channels).
// LDS image per operand: [32 rows][8 pieces of 16 B], piece p of row r in slot
// p ^ (r & 7) — the swizzle sits on the global source address because the
// DMA's LDS destination is lane-linear — read back in the MFMA layout with
// ds_read_b128 (lane (i, h): pieces 4h .. 4h+3 of row i), conflict-free over
// any 8 consecutive rows.  One buffer per operand and wave: stage j is read
// into registers, then stage j+1's DMA is issued into the same buffer and
// runs under stage j's 16 MFMAs.
// --------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_void_ptr;

__device__ __forceinline__ void glds16(const float* g, float* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_ptr)(lds_wave_base), 16, 0, 0);
}

// DMA of one stage (offset k, channels [c0, c0+32)) into abuf / bbuf, plus the
// row factors of lane (i, h)'s row i into st.
// BREG: B (the filters, L2-resident) as fragment-shaped 16-B loads straight
// into st.b instead of through LDS — half the LDS per wave, so more waves.
// SC: row / pair scales present (importance, normalisation); without them the
// factors are 1 and no per-stage scale loads are issued
// BUF (cin % 32 == 0, operands < 2 GiB, no scales, BREG): the rows and the
// filters through buffer resources with 32-bit offsets — a missing row or
// column gets an offset past the resource's range, which the buffer unit
// answers with zeros (no zero-page select, no 64-bit address arithmetic:
// ~40 % of the loop's VALU went to addresses)
constexpr uint32_t kNoRow = 0x7FFFFFF0u;  // > num_records of every operand resource (its true byte size)
struct GemmRsrc {
    __amdgpu_buffer_rsrc_t src, w, wsp;
};
__device__ __forceinline__ GemmRsrc gemm_rsrc(const float* src, const float* Wt, const GemmPrologue& pre) {
    return {__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), static_cast<short>(0),
                                              static_cast<int>(pre.src_bytes), kBufferFlags),
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Wt), static_cast<short>(0),
                                              static_cast<int>(pre.w_bytes), kBufferFlags),
            __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(pre.wsplit), static_cast<short>(0),
                                              static_cast<int>(pre.wsplit_bytes), kBufferFlags)};
}

// O3DML_GEMM_DIAG (cost-split builds only, results invalid): 1 = the per-wave
// kernel's buffer path issues no filter loads, 2 = no row gathers
#ifndef O3DML_GEMM_DIAG
#define O3DML_GEMM_DIAG 0
#endif
// A stage's map entries from the LDS tile: the 4 gathered rows of this lane
// (rows 8 q + lane / 8) and its own row i; -1 on a dead stage.  The reads are
// unconditional and then selected: `live` is wave-uniform, and a read under
// it compiled to one branch per read, each read waited on alone (k stays a
// valid offset on a dead stage, so the reads are in bounds).
struct StageMap {
    int32_t mq[4];
    int32_t mi;
};
__device__ __forceinline__ StageMap lds_map(const int32_t* mtile, int K, int k, int lane, int i, bool live) {
    StageMap m;
#pragma unroll
    for (int q = 0; q < 4; ++q) m.mq[q] = mtile[(8 * q + (lane >> 3)) * K + k];
    m.mi = mtile[i * K + k];
#pragma unroll
    for (int q = 0; q < 4; ++q) m.mq[q] = live ? m.mq[q] : -1;
    m.mi = live ? m.mi : -1;
    return m;
}

template <bool BREG, bool SC = true, bool BUF = false, bool BS = false>
__device__ __forceinline__ void lds_issue_map(float* abuf, float* bbuf, const StageMap& sm, int k, int c0, int lane,
                                              int64_t o, int i, int col0, const float* __restrict__ src,
                                              const float* __restrict__ sscale, const float* __restrict__ pscale,
                                              const float* __restrict__ Wt, int K, int cin, int cout, bool live,
                                              GemmStage& st, const GemmRsrc* rs) {
    const int sl = lane & 7;
    const int32_t* mq = sm.mq;
    const int32_t mi = sm.mi;
    if constexpr (BUF) {
        static_assert(BREG && !SC, "buffer addressing: filters in registers, no scales");
        const uint32_t row_bytes = static_cast<uint32_t>(cin) * 4u;
#if O3DML_GEMM_DIAG != 2  // cost-split diagnostics: 2 = no row gathers
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = 8 * q + (lane >> 3);
            const uint32_t cb = static_cast<uint32_t>(c0 + 4 * (sl ^ (r & 7))) * 4u;
            // 24-bit multiply (full rate): the host admits the buffer path only when
            // every byte offset is < 2^31 with cin >= 32, so rows < 2^24
            const uint32_t off = mq[q] >= 0 ? __umul24(static_cast<uint32_t>(mq[q]), row_bytes) + cb : kNoRow;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs->src, (lds_void_ptr)(abuf + 256 * q), 16, off, 0, 0, 0);
        }
#else
        (void)row_bytes;
#endif
        const int col = col0 + i;
#if O3DML_GEMM_DIAG == 1  // cost-split diagnostics: 1 = no filter loads
        if constexpr (!BS) {
#pragma unroll
            for (int q = 0; q < 16; ++q) st.b[q] = 1.f;
            st.s1 = st.s2 = 1.f;
            st.v = mi >= 0 ? 1.f : 0.f;
            return;
        }
#endif
        if constexpr (BS) {  // the lane's 16 channels as two 8-channel blocks of 3 x 16 B
            const uint32_t soff = (live && col < cout)
                                          ? (static_cast<uint32_t>(k * cout + col) * static_cast<uint32_t>(cin) +
                                             static_cast<uint32_t>(c0 + 16 * (lane >> 5))) / 8u * 48u
                                          : kNoRow;
#pragma unroll
            for (int m = 0; m < 6; ++m)
                st.bs[m] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs->wsp, soff + 16u * m, 0, 0));
        } else {
            const uint32_t boff = (live && col < cout)
                                          ? (__umul24(static_cast<uint32_t>(k * cout + col), static_cast<uint32_t>(cin)) +
                                             static_cast<uint32_t>(c0 + 16 * (lane >> 5))) * 4u
                                          : kNoRow;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs->w, boff + 16u * q, 0, 0));
                st.b[4 * q] = v.x;
                st.b[4 * q + 1] = v.y;
                st.b[4 * q + 2] = v.z;
                st.b[4 * q + 3] = v.w;
            }
        }
        st.s1 = st.s2 = 1.f;
        st.v = mi >= 0 ? 1.f : 0.f;
        return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = 8 * q + (lane >> 3);
        const int c = c0 + 4 * (sl ^ (r & 7));
        const int32_t m = mq[q];
        const float* ga = (m >= 0 && c < cin) ? src + static_cast<int64_t>(m) * cin + c : g_zero_page;
        glds16(ga, abuf + 256 * q);
        if constexpr (!BREG) {
            const int cc = col0 + r;
            const float* gb = (live && cc < cout && c < cin) ? Wt + (static_cast<int64_t>(k) * cout + cc) * cin + c
                                                              : g_zero_page;
            glds16(gb, bbuf + 256 * q);
        }
    }
    if constexpr (BREG) {  // lane (i, h): channels [c0 + 16h, +16) of column col0 + i
        const int cb = c0 + 16 * (lane >> 5);
        const int col = col0 + i;
        const bool colv = live && col < cout;
        const float* wr = Wt + (static_cast<int64_t>(k) * cout + (colv ? col : 0)) * cin;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cb + 4 * q;
            const float4 v = *reinterpret_cast<const float4*>((colv && c < cin) ? wr + c : g_zero_page);
            st.b[4 * q] = v.x;
            st.b[4 * q + 1] = v.y;
            st.b[4 * q + 2] = v.z;
            st.b[4 * q + 3] = v.w;
        }
    }
    const bool valid = mi >= 0;
    if constexpr (SC) {
        st.s1 = *(sscale ? sscale + (valid ? mi : 0) : g_one_page);
        st.s2 = *(pscale ? pscale + (valid ? o : 0) * K + k : g_one_page);
    } else {
        st.s1 = st.s2 = 1.f;
    }
    st.v = valid ? 1.f : 0.f;
}

template <bool BREG, bool SC = true, bool BUF = false, bool BS = false>
__device__ __forceinline__ void lds_issue(float* abuf, float* bbuf, const int32_t* mtile, int K, int k, int c0,
                                          int lane, int64_t o, int i, int col0, const float* __restrict__ src,
                                          const float* __restrict__ sscale, const float* __restrict__ pscale,
                                          const float* __restrict__ Wt, int cin, int cout, bool live, GemmStage& st,
                                          const GemmRsrc* rs = nullptr) {
    // all LDS reads of the map first (a DMA in between would order after them)
    const StageMap sm = lds_map(mtile, K, k, lane, i, live);
    lds_issue_map<BREG, SC, BUF, BS>(abuf, bbuf, sm, k, c0, lane, o, i, col0, src, sscale, pscale, Wt, K, cin, cout,
                                     live, st, rs);
}

template <bool BREG>
__device__ __forceinline__ void lds_read(const float* abuf, const float* bbuf, int i, int h, GemmStage& st) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int slot = (4 * h + q) ^ (i & 7);
        const float4 va = *reinterpret_cast<const float4*>(abuf + 32 * i + 4 * slot);
        st.a[4 * q] = va.x;
        st.a[4 * q + 1] = va.y;
        st.a[4 * q + 2] = va.z;
        st.a[4 * q + 3] = va.w;
        if constexpr (!BREG) {
            const float4 vb = *reinterpret_cast<const float4*>(bbuf + 32 * i + 4 * slot);
            st.b[4 * q] = vb.x;
            st.b[4 * q + 1] = vb.y;
            st.b[4 * q + 2] = vb.z;
            st.b[4 * q + 3] = vb.w;
        }
    }
}

// f32 products on the bf16 MFMA pipe.  x = hi + mid + lo with hi =
// rne_bf16(x), mid = rne_bf16(x - hi), lo = rne_bf16(x - hi - mid): each
// rounding keeps 8 more significant bits, so the three terms hold all 24 bits
// of an f32 (exact up to the last rounding, <= 2^-25 |x|).  Each bf16 x bf16
// product is exact in the f32 accumulator.
//  * NT = 6 (default, "bf16x6"): a*b = hh + hm + mh + hl + lh + mm, dropping
//    terms <= 2^-24 |a*b| — the f32 rounding level, so the sums agree with the
//    exact f32-input MFMA to within its own rounding.  Six
//    v_mfma_f32_32x32x16_bf16 (32 cycles each) per 16 reduction steps instead
//    of eight v_mfma_f32_32x32x2_f32 (64 cycles each): 2.7x fewer MFMA cycles.
//  * NT = 3 ("bf16x3"): hh + hm + mh with x = hi + mid only (<= 2^-17
//    relative per product), 5.3x fewer MFMA cycles.
// Fragment of MFMA t (t = 0, 1) on lane (i, h): element j = stage register
// 8t + j (channel c0 + 16h + 8t + j in the forward GEMM) — the same map on A
// (row i) and B (column i), so any consistent permutation of the reduction.
template <int NT>
__device__ __forceinline__ void split_bf16x8(const float* v, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hi[j] = static_cast<__bf16>(v[j]);
        const float r1 = v[j] - static_cast<float>(hi[j]);
        mid[j] = static_cast<__bf16>(r1);
        if constexpr (NT == 6) lo[j] = static_cast<__bf16>(r1 - static_cast<float>(mid[j]));
    }
}

template <int NT, class Stage>
__device__ __forceinline__ void mfma_stage_split(const Stage& cu, f32x16& acc) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        bf16x8 ah, am, al, bh, bm, bl;
        split_bf16x8<NT>(cu.a + 8 * t, ah, am, al);
        split_bf16x8<NT>(cu.b + 8 * t, bh, bm, bl);
        if constexpr (NT == 6) {  // smallest terms first
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    }
}

// bf16x6 products with the B operand split once per call (BS): the same six
// MFMAs in the same order as mfma_stage_split<6> on the same bf16 terms, so
// the same bits; only A is split per stage
template <class Stage>
__device__ __forceinline__ void mfma_stage_bs(const Stage& cu, f32x16& acc) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        bf16x8 ah, am, al;
        split_bf16x8<6>(cu.a + 8 * t, ah, am, al);
        const bf16x8 bh = cu.bs[3 * t], bm = cu.bs[3 * t + 1], bl = cu.bs[3 * t + 2];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    }
}

// The filters Wt [K][cout][cin] (cin % 8 == 0) as 8-channel blocks of three
// bf16x8 (split_bf16x8<6>: hi, mid, lo) for the BS kernels
__global__ void split_filters_kernel(const float* __restrict__ wt, int64_t nblk, bf16x8* __restrict__ out) {
    for (int64_t b = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; b < nblk;
         b += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const float4 p = reinterpret_cast<const float4*>(wt)[2 * b];
        const float4 q = reinterpret_cast<const float4*>(wt)[2 * b + 1];
        const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
        bf16x8 hi, mid, lo;
        split_bf16x8<6>(v, hi, mid, lo);
        out[3 * b] = hi;
        out[3 * b + 1] = mid;
        out[3 * b + 2] = lo;
    }
}

// product precision of a GEMM instantiation: 0 = exact f32 MFMA, 3 / 6 = bf16 split
template <int NT, class Stage>
__device__ __forceinline__ void mfma_stage(const Stage& cu, f32x16& acc) {
    if constexpr (NT == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cu.a[r], cu.b[r], acc, 0, 0, 0);
    } else {
        mfma_stage_split<NT>(cu, acc);
    }
}

// Per-wave timeline of implicit_gemm_lds_kernel (diagnostic builds only:
// -DO3DML_GEMM_TRACE=1, tools/gemm_trace.py): 100-MHz real-time stamps of
// each wave's phases, read back with o3dml_gemm_trace_read.  Slots: 0 entry,
// 1 output rows in LDS, 2 map tile in LDS, 3 offset mask, 4..11 stage j's
// operands landed (first 8 stages), 12 stages done, 13 results stored,
// 14 stage count, 15 HW_ID | XCC_ID << 32.
#ifndef O3DML_GEMM_TRACE
#define O3DML_GEMM_TRACE 0
#endif
#if O3DML_GEMM_TRACE
constexpr int kTraceSlots = 16;
constexpr int64_t kTraceWaves = 1 << 16;
__device__ uint64_t g_gemm_trace[kTraceWaves * kTraceSlots];
#define O3DML_TRACE_AT(slot, v)                                                            \
    do {                                                                                   \
        if (trace_row >= 0 && lane == 0) g_gemm_trace[trace_row * kTraceSlots + (slot)] = (v); \
    } while (0)
#define O3DML_TRACE(slot) O3DML_TRACE_AT(slot, __builtin_amdgcn_s_memrealtime())
#else
#define O3DML_TRACE_AT(slot, v) do {} while (0)
#define O3DML_TRACE(slot) do {} while (0)
#endif

// DEPTH 2 (BUF only, O3DML_GEMM_DEPTH=2): two stages in flight per wave —
// stage j+2's DMA is issued while stage j is multiplied.  Off by default:
// 12 instead of 16 waves per CU (136 registers, 49 KiB LDS per workgroup), and
// same-session A/B 3-8 % slower at 32->32 / 64->32 (tools/gemm_probe.py)
template <bool PRE, bool BREG, int NT = 0, bool SC = true, bool BUF = false, int DEPTH = 1, bool BS = false>
__global__ void __launch_bounds__(kGemmThreads)
implicit_gemm_lds_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ order,
                         const int* order_flag, int K, int64_t n_out,
                         const float* __restrict__ src, const float* __restrict__ sscale,
                         const float* __restrict__ pscale, const float* __restrict__ Wt /*[K][cout][cin]*/, int cin,
                         int cout, const float* __restrict__ oscale, const float* __restrict__ bias,
                         float* __restrict__ out, int nsplit, float* __restrict__ part, GemmPrologue pre,
                         const float* __restrict__ residual, uint32_t* __restrict__ counters) {
    __shared__ float lpre[PRE ? 2 * (kPreMax + 32) : 1];
    __shared__ __attribute__((aligned(16))) float stage_all[kGemmThreads / 64][BREG && DEPTH == 1 ? 1 : 2][32 * 32];
    __shared__ int32_t mtile_all[kGemmThreads / 64][32 * 32];
    __shared__ int32_t orow_all[kGemmThreads / 64][32];
#if O3DML_GEMM_TRACE
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
#endif
    float* lps = lpre;
    float* lpb = lpre + (PRE ? kPreMax + 32 : 0);
    if (PRE) {
        for (int c = threadIdx.x; c < kPreMax + 32; c += kGemmThreads) {
            lps[c] = c < cin ? pre.scale[c] : 0.f;
            lpb[c] = c < cin ? pre.shift[c] : 0.f;
        }
        __syncthreads();
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: item decode in scalars
    int32_t* mtile = mtile_all[w];
    int32_t* orow = orow_all[w];
    float* abuf = stage_all[w][0];
    float* bbuf = stage_all[w][BREG ? 0 : 1];  // unused with BREG
    // Work items (32-row tile, column block, split).  Default: one wave per
    // item, the grid's (x, y, z).  Persistent grid (pre.pcols > 0): only as
    // many waves as are resident, each looping over items tile-major, so no
    // partial last round of waves idles most SIMDs (wave-lifetime tail).
    const bool pers = pre.pcols > 0;
    const int64_t ntw = (n_out + 31) >> 5;
    const int64_t per_tile = pers ? static_cast<int64_t>(pre.pcols) * nsplit : 1;
    const int64_t n_items = pers ? ntw * per_tile : 1;
    const int64_t it_step = static_cast<int64_t>(gridDim.x) * (kGemmThreads / 64);
    const int64_t it0 = pers ? static_cast<int64_t>(blockIdx.x) * (kGemmThreads / 64) + w : 0;
    // With the tile-order map copy, an item's map rows and output rows come
    // from registers loaded ahead: the wave's first tile before the order
    // flag is read (the map workspace holds the order and the copy whether
    // or not they were built, so the loads stay in bounds; their values are
    // dropped when the flag says no order), each next tile under the current
    // item's stages (persistent grid).
    MapTileRegs<32, 64> nxt;
    int32_t nrow = -1;
    bool have_next = false;
    if (order && pre.tmap && it0 < n_items) {
        const int64_t tw0 = pers ? it0 / per_tile : xcd_block() * (kGemmThreads / 64) + w;
        const int64_t f0 = tw0 * 32;
        if (f0 < n_out) {
            const int ln = threadIdx.x & 63;
            map_tile_fetch<32, 64>(pre.tmap + f0 * K, K, ln, nxt);
            nrow = ln < 32 && f0 + ln < n_out ? order[f0 + ln] : -1;
            have_next = true;
        }
    }
    if (order && *order_flag == 0) {  // map built without a tile order
        order = nullptr;
        have_next = false;
    }
    const bool prefetch = pers && order && pre.tmap;
#pragma clang loop unroll(disable)
    for (int64_t it = it0; it < n_items; it += it_step) {
    // the lane index made opaque per item: otherwise every lane-derived
    // address of the body is hoisted out of the item loop and held live
    // across it (72 -> 161 registers, half the waves)
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const int i = lane & 31, h = lane >> 5;
    int64_t tw;
    int cy, s;
    if (pers) {
        tw = it / per_tile;
        const int r = static_cast<int>(it - tw * per_tile);
        cy = r % pre.pcols;
        s = r / pre.pcols;
    } else {
        // XCD-contiguous tiles (grid a multiple of 8): XCD x takes one
        // contiguous eighth of the (spatially chunked) tile order, so its L2
        // holds the input rows that eighth gathers
        tw = xcd_block() * (kGemmThreads / 64) + w;
        cy = blockIdx.y;
        s = blockIdx.z;
    }
    const int64_t o0 = tw * 32;
    if (o0 >= n_out) continue;  // whole wave; no barriers below
    const int col0 = cy * 32;
    const int col = col0 + i;
#if O3DML_GEMM_TRACE
    const int64_t trace_wave = pers ? it
                                    : ((static_cast<int64_t>(blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x +
                                       blockIdx.x) * (kGemmThreads / 64) + w;
    const int64_t trace_row = trace_wave < kTraceWaves ? trace_wave : -1;
    O3DML_TRACE_AT(0, t_entry);
    O3DML_TRACE_AT(15, static_cast<uint64_t>(__builtin_amdgcn_s_getreg((31 << 11) | 4)) |
                           (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32));
#endif
    // the previous item's LDS reads (orow, mtile, stage) are done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    unsigned used = 0u;
    if (order && pre.tmap) {  // tile order with its map copy: map rows and output rows loaded together
        MapTileRegs<32, 64> cur;
        int32_t orv;
        if (have_next) {
            cur = nxt;
            orv = nrow;
        } else {
            map_tile_fetch<32, 64>(pre.tmap + o0 * K, K, lane, cur);
            orv = lane < 32 && o0 + lane < n_out ? order[o0 + lane] : -1;
        }
        if (lane < 32) orow[lane] = orv;
        used = map_tile_commit<32, 64>(cur, K, lane, mtile);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        O3DML_TRACE(1);
        O3DML_TRACE(2);
    } else {
        if (lane < 32) {
            const int64_t oo = o0 + lane;
            orow[lane] = oo < n_out ? (order ? order[oo] : static_cast<int32_t>(oo)) : -1;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        O3DML_TRACE(1);
        load_map_tile<32, 64>(map, orow, K, lane, mtile);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        O3DML_TRACE(2);
        for (int k = h; k < K; k += 2) {
            const uint64_t b = __ballot(mtile[i * K + k] >= 0);
            used |= ((h ? (b >> 32) : (b & 0xffffffffull)) != 0ull) ? (1u << k) : 0u;
        }
        used = __builtin_amdgcn_readlane(used, 32) | __builtin_amdgcn_readlane(used, 0);
    }
    O3DML_TRACE(3);
    const int64_t o = orow[i] >= 0 ? orow[i] : 0;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int nch = (cin + 31) >> 5;
    const int j0 = split_stage(used, nch, K, s, nsplit);
    const int j1 = split_stage(used, nch, K, s + 1, nsplit);
    O3DML_TRACE_AT(14, static_cast<uint64_t>(j1 - j0));
    have_next = false;
    if (prefetch && it + it_step < n_items) {  // in flight with stage 0's operands
        const int64_t no0 = (it + it_step) / per_tile * 32;
        map_tile_fetch<32, 64>(pre.tmap + no0 * K, K, lane, nxt);
        nrow = lane < 32 && no0 + lane < n_out ? order[no0 + lane] : -1;
        have_next = true;
    }
    if (DEPTH == 2 && j0 < j1) {
        static_assert(DEPTH == 1 || (BUF && BREG && !SC), "two stages in flight: buffer path only");
        unsigned u = used;
        for (int t = j0 / nch; t > 0; --t) u &= u - 1u;
        int k = __builtin_ctz(u), c0 = (j0 % nch) * 32;
        auto advance = [&]() {
            c0 += 32;
            if (c0 >= cin) {
                c0 = 0;
                u &= u - 1u;
                k = u ? __builtin_ctz(u) : 0;
            }
        };
        const GemmRsrc rs = gemm_rsrc(src, Wt, pre);
        float* buf1 = stage_all[w][1];
        GemmStage s0, s1, cu;
        int c00 = c0;
        lds_issue<true, false, true>(abuf, nullptr, mtile, K, k, c0, lane, o, i, col0, src, sscale, pscale, Wt, cin,
                                     cout, true, s0, &rs);
        advance();
        int c01 = c0;
        lds_issue<true, false, true>(buf1, nullptr, mtile, K, k, c0, lane, o, i, col0, src, sscale, pscale, Wt, cin,
                                     cout, j0 + 1 < j1, s1, &rs);
        advance();
        // every stage issues exactly 8 vector-memory ops (4 row DMAs, 4 filter
        // loads; dead stages read zeros), so vmcnt(8) = the older stage landed
        for (int j = j0; j < j1; j += 2) {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            lds_read<true>(abuf, nullptr, i, h, cu);
#pragma unroll
            for (int r = 0; r < 16; ++r) cu.b[r] = s0.b[r];
            cu.s1 = s0.s1;
            cu.s2 = s0.s2;
            cu.v = s0.v;  // the prologue zeroes a missing row (relu(0 * s + b) != 0)
            int cj = c00;
            c00 = c0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_issue<true, false, true>(abuf, nullptr, mtile, K, k, c0, lane, o, i, col0, src, sscale, pscale, Wt,
                                         cin, cout, j + 2 < j1, s0, &rs);
            advance();
            __builtin_amdgcn_sched_barrier(0);
            gemm_finish<PRE, false>(cu, cj, h, lps, lpb);
            mfma_stage<NT>(cu, acc);
            if (j + 1 >= j1) break;
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            lds_read<true>(buf1, nullptr, i, h, cu);
#pragma unroll
            for (int r = 0; r < 16; ++r) cu.b[r] = s1.b[r];
            cu.s1 = s1.s1;
            cu.s2 = s1.s2;
            cu.v = s1.v;  // the prologue zeroes a missing row (relu(0 * s + b) != 0)
            cj = c01;
            c01 = c0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_issue<true, false, true>(buf1, nullptr, mtile, K, k, c0, lane, o, i, col0, src, sscale, pscale, Wt,
                                         cin, cout, j + 3 < j1, s1, &rs);
            advance();
            __builtin_amdgcn_sched_barrier(0);
            gemm_finish<PRE, false>(cu, cj, h, lps, lpb);
            mfma_stage<NT>(cu, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dead DMAs have landed before the wave exits
    } else if (j0 < j1) {
        static_assert(!BS || (BUF && BREG && !SC && NT == 6 && DEPTH == 1), "split filters: bf16x6 buffer path");
        unsigned u = used;
        for (int t = j0 / nch; t > 0; --t) u &= u - 1u;
        int k = __builtin_ctz(u), c0 = (j0 % nch) * 32;
        GemmStage nx, cu;
        const GemmRsrc rs = gemm_rsrc(src, Wt, pre);
        lds_issue<BREG, SC, BUF, BS>(abuf, bbuf, mtile, K, k, c0, lane, o, i, col0, src, sscale, pscale, Wt, cin,
                                     cout, true, nx, &rs);
        for (int j = j0; j < j1; ++j) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage j in LDS, its row factors in nx
            if (j - j0 < 8) O3DML_TRACE(4 + j - j0);
            const int kj = k, cj = c0;
            c0 += 32;
            if (c0 >= cin) {
                c0 = 0;
                u &= u - 1u;
                k = u ? __builtin_ctz(u) : 0;
            }
            // the next stage's map entries are read beside this stage's rows
            // (different LDS arrays), so one LDS wait covers both
            const StageMap sm = lds_map(mtile, K, k, lane, i, j + 1 < j1);
            lds_read<BREG>(abuf, bbuf, i, h, cu);
            __builtin_amdgcn_sched_barrier(0);  // both read groups issued before any waits on them
            if constexpr (BS) {
#pragma unroll
                for (int m = 0; m < 6; ++m) cu.bs[m] = nx.bs[m];
            } else if constexpr (BREG) {
#pragma unroll
                for (int r = 0; r < 16; ++r) cu.b[r] = nx.b[r];
            }
            cu.s1 = nx.s1;
            cu.s2 = nx.s2;
            cu.v = nx.v;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // buffer read out before the next DMA
            lds_issue_map<BREG, SC, BUF, BS>(abuf, bbuf, sm, k, c0, lane, o, i, col0, src, sscale, pscale, Wt, K, cin,
                                             cout, j + 1 < j1, nx, &rs);
            __builtin_amdgcn_sched_barrier(0);
            (void)kj;
            gemm_finish<PRE, SC>(cu, cj, h, lps, lpb);
            if constexpr (BS) mfma_stage_bs(cu, acc);
            else mfma_stage<NT>(cu, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dead DMA has landed before the wave exits
    }
    O3DML_TRACE(12);
    if (nsplit > 1) {
        split_store_finish(acc, orow, h, col, lane, s, nsplit, n_out, cout, part, counters,
                           pers ? cy * ntw + tw
                                : (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * (kGemmThreads / 64) + w,
                           oscale, bias, residual, out);
        O3DML_TRACE(13);
        continue;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t orr = orow[(r & 3) + 8 * (r >> 2) + 4 * h];
        if (orr >= 0 && col < cout) {
            float v = acc[r];
            if (oscale) v *= oscale[orr];
            if (bias) v += bias[col];
            if (residual) v += residual[orr * cout + col];
            out[orr * cout + col] = v;
        }
    }
    O3DML_TRACE(13);
    }  // work items
}

#if O3DML_GEMM_TRACE
// diagnostic builds: copy the per-wave timeline out (kTraceWaves x kTraceSlots
// u64) after the GEMM of interest has run; o3dml_gemm_trace_clear zeroes it
O3DML_API int o3dml_gemm_trace_read(void* dst, size_t bytes) {
    bytes = std::min(bytes, sizeof(g_gemm_trace));
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gemm_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
O3DML_API int o3dml_gemm_trace_clear() {
    static std::vector<uint64_t> z(kTraceWaves * kTraceSlots, 0);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_trace), z.data(), sizeof(g_gemm_trace), 0, hipMemcpyHostToDevice) ==
                   hipSuccess ? 0 : -1;
}
#endif

// --------------------------------------------------------------------------
// implicit GEMM, A tile shared by the workgroup (cout >= 64): NW waves own the
// same 32 output rows and NW adjacent 32-column blocks, so the gathered rows
// of a stage (32 rows x 32 channels, the bytes that bound the per-wave kernel
// once its products run on the bf16 pipe) are fetched once per workgroup
// instead of once per column block: each wave DMAs 4/NW of the 4 row groups
// into a double-buffered LDS image, a barrier per stage publishes it, and
// every wave reads the whole tile in the MFMA layout.  B (filters) stays in
// registers per wave; stage order, split-K partition and reduction order per
// output are those of implicit_gemm_lds_kernel (same sums).
// --------------------------------------------------------------------------
// DMA of this wave's share of one stage: row groups q = w, w + NW, ... of the
// tile's 4*RB groups of 8 rows (lane-linear LDS destination, swizzled source
// as in lds_issue)
template <int NW, int RB, bool BUF = false>
__device__ __forceinline__ void shared_issue(float* abuf, const int32_t* mtile, int K, int k, int c0, int lane, int w,
                                             const float* __restrict__ src, int cin, bool live,
                                             const GemmRsrc* rs = nullptr) {
    constexpr int NQ = 4 * RB / NW;
    const int sl = lane & 7;
    int32_t mq[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) mq[t] = live ? mtile[(8 * (w + NW * t) + (lane >> 3)) * K + k] : -1;
    if constexpr (BUF) {  // buffer addressing as lds_issue (cin % 32 == 0)
        const uint32_t row_bytes = static_cast<uint32_t>(cin) * 4u;
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            const int q = w + NW * t;
            const int r = 8 * q + (lane >> 3);
            const uint32_t cb = static_cast<uint32_t>(c0 + 4 * (sl ^ (r & 7))) * 4u;
            const uint32_t off = mq[t] >= 0 ? static_cast<uint32_t>(mq[t]) * row_bytes + cb : kNoRow;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs->src, (lds_void_ptr)(abuf + 256 * q), 16, off, 0, 0, 0);
        }
        return;
    }
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int q = w + NW * t;
        const int r = 8 * q + (lane >> 3);
        const int c = c0 + 4 * (sl ^ (r & 7));
        const float* ga = (mq[t] >= 0 && c < cin) ? src + static_cast<int64_t>(mq[t]) * cin + c : g_zero_page;
        glds16(ga, abuf + 256 * q);
    }
}

template <int RB>
struct SharedStage {
    float a[RB][16], b[16];
    float sc[RB];  // row factor (importance x pair scale, 0 for a missing row)
};

template <int RB, bool SC = true, bool BUF = false>
__device__ __forceinline__ void shared_regs(const int32_t* mtile, int K, int k, int c0, int lane, const int64_t* o,
                                            int i, int col, const float* __restrict__ sscale,
                                            const float* __restrict__ pscale, const float* __restrict__ Wt, int cin,
                                            int cout, bool live, SharedStage<RB>& st, float (&s1)[RB],
                                            float (&s2)[RB], bool (&v)[RB], const GemmRsrc* rs = nullptr) {
    const int cb = c0 + 16 * (lane >> 5);
    const bool colv = live && col < cout;
    if constexpr (BUF) {
        static_assert(!SC, "buffer addressing: no scales");
        const uint32_t boff =
                colv ? (static_cast<uint32_t>(k * cout + col) * static_cast<uint32_t>(cin) + static_cast<uint32_t>(cb)) * 4u
                     : kNoRow;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs->w, boff + 16u * q, 0, 0));
            st.b[4 * q] = x.x;
            st.b[4 * q + 1] = x.y;
            st.b[4 * q + 2] = x.z;
            st.b[4 * q + 3] = x.w;
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            v[rb] = live && mtile[(32 * rb + i) * K + k] >= 0;
            s1[rb] = s2[rb] = 1.f;
        }
        return;
    }
    const float* wr = Wt + (static_cast<int64_t>(k) * cout + (colv ? col : 0)) * cin;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int c = cb + 4 * q;
        const float4 x = *reinterpret_cast<const float4*>((colv && c < cin) ? wr + c : g_zero_page);
        st.b[4 * q] = x.x;
        st.b[4 * q + 1] = x.y;
        st.b[4 * q + 2] = x.z;
        st.b[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int32_t mi = live ? mtile[(32 * rb + i) * K + k] : -1;
        v[rb] = mi >= 0;
        if constexpr (SC) {
            s1[rb] = *(sscale ? sscale + (v[rb] ? mi : 0) : g_one_page);
            s2[rb] = *(pscale ? pscale + (v[rb] ? o[rb] : 0) * K + k : g_one_page);
        } else {
            s1[rb] = s2[rb] = 1.f;
        }
    }
}

// RB row blocks against one column block: B split once, each row block's A
// split and multiplied into its accumulator (same per-output sums as
// mfma_stage: the reduction order of one accumulator does not change)
template <int NT, int RB>
__device__ __forceinline__ void mfma_stage_rb(const SharedStage<RB>& cu, f32x16 (&acc)[RB]) {
    if constexpr (NT == 0) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(cu.a[rb][r], cu.b[r], acc[rb], 0, 0, 0);
    } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            bf16x8 bh, bm, bl;
            split_bf16x8<NT>(cu.b + 8 * t, bh, bm, bl);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                bf16x8 ah, am, al;
                split_bf16x8<NT>(cu.a[rb] + 8 * t, ah, am, al);
                if constexpr (NT == 6) {
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[rb], 0, 0, 0);
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[rb], 0, 0, 0);
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[rb], 0, 0, 0);
                }
                acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[rb], 0, 0, 0);
            }
        }
    }
}

// The tile: 32*RB output rows (RB row blocks) x NW column blocks; wave w owns
// column block w for all RB row blocks, so each stage's B fragment (the
// filters, read by every wave of every tile) feeds RB accumulators.
template <bool PRE, int NT, int NW, int RB, bool SC = true, bool BUF = false>
__global__ void __launch_bounds__(NW * 64)
implicit_gemm_shared_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ order,
                            const int* order_flag, int K, int64_t n_out,
                            const float* __restrict__ src, const float* __restrict__ sscale,
                            const float* __restrict__ pscale, const float* __restrict__ Wt /*[K][cout][cin]*/,
                            int cin, int cout, const float* __restrict__ oscale, const float* __restrict__ bias,
                            float* __restrict__ out, int nsplit, float* __restrict__ part, GemmPrologue pre,
                            const float* __restrict__ residual, uint32_t* __restrict__ counters) {
    constexpr int R = 32 * RB;
    __shared__ float lpre[PRE ? 2 * (kPreMax + 32) : 1];
    __shared__ __attribute__((aligned(16))) float abuf[2][R * 32];
    __shared__ int32_t mtile[R * 32];
    __shared__ int32_t orow[R];
    const int64_t o0 = xcd_block() * R;  // XCD-contiguous tiles, as implicit_gemm_lds_kernel
    if (o0 >= n_out) return;  // whole workgroup, before any barrier
    float* lps = lpre;
    float* lpb = lpre + (PRE ? kPreMax + 32 : 0);
    if (PRE) {
        for (int c = threadIdx.x; c < kPreMax + 32; c += NW * 64) {
            lps[c] = c < cin ? pre.scale[c] : 0.f;
            lpb[c] = c < cin ? pre.shift[c] : 0.f;
        }
    }
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int i = lane & 31, h = lane >> 5;
    const int col = (blockIdx.y * NW + w) * 32 + i;
    if (order && *order_flag == 0) order = nullptr;
    unsigned used = 0u;  // identical in every wave (same rows)
    if (order && pre.tmap) {  // tile order with its map copy: map rows and output rows loaded together
        __shared__ unsigned used_w[NW];
        for (int t = threadIdx.x; t < R; t += NW * 64) {
            const int64_t oo = o0 + t;
            orow[t] = oo < n_out ? order[oo] : -1;
        }
        const unsigned mw = load_map_tile_direct<R, NW * 64>(pre.tmap + o0 * K, K, threadIdx.x, mtile);
        if (lane == 0) used_w[w] = mw;
        __syncthreads();
#pragma unroll
        for (int v = 0; v < NW; ++v) used |= used_w[v];
    } else {
        for (int t = threadIdx.x; t < R; t += NW * 64) {
            const int64_t oo = o0 + t;
            orow[t] = oo < n_out ? (order ? order[oo] : static_cast<int32_t>(oo)) : -1;
        }
        __syncthreads();
        load_map_tile<R, NW * 64>(map, orow, K, threadIdx.x, mtile);
        __syncthreads();
        for (int k = h; k < K; k += 2) {
            bool any = false;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) any |= mtile[(32 * rb + i) * K + k] >= 0;
            const uint64_t b = __ballot(any);
            used |= ((h ? (b >> 32) : (b & 0xffffffffull)) != 0ull) ? (1u << k) : 0u;
        }
    }
    used = __builtin_amdgcn_readlane(used, 32) | __builtin_amdgcn_readlane(used, 0);
    int64_t o[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) o[rb] = orow[32 * rb + i] >= 0 ? orow[32 * rb + i] : 0;
    f32x16 acc[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[rb][r] = 0.f;
    const int nch = (cin + 31) >> 5;
    const int s = blockIdx.z;
    const int j0 = split_stage(used, nch, K, s, nsplit);
    const int j1 = split_stage(used, nch, K, s + 1, nsplit);
    if (j0 < j1) {  // uniform over the workgroup
        unsigned u = used;
        for (int t = j0 / nch; t > 0; --t) u &= u - 1u;
        int k = __builtin_ctz(u), c0 = (j0 % nch) * 32;
        SharedStage<RB> nx, cu;
        float s1[RB], s2[RB];
        bool vv[RB];
        const GemmRsrc rs = gemm_rsrc(src, Wt, pre);
        shared_issue<NW, RB, BUF>(abuf[0], mtile, K, k, c0, lane, w, src, cin, true, &rs);
        shared_regs<RB, SC, BUF>(mtile, K, k, c0, lane, o, i, col, sscale, pscale, Wt, cin, cout, true, nx, s1, s2, vv,
                                 &rs);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int j = j0; j < j1; ++j) {
            const int b = (j - j0) & 1;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                GemmStage ta;
                lds_read<true>(abuf[b] + 32 * 32 * rb, nullptr, i, h, ta);
#pragma unroll
                for (int r = 0; r < 16; ++r) cu.a[rb][r] = ta.a[r];
                cu.sc[rb] = vv[rb] ? s1[rb] * s2[rb] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) cu.b[r] = nx.b[r];
            const int cj = c0;
            c0 += 32;
            if (c0 >= cin) {
                c0 = 0;
                u &= u - 1u;
                k = u ? __builtin_ctz(u) : 0;
            }
            const bool live = j + 1 < j1;
            // the other buffer was last read in stage j-1, before that stage's barrier
            shared_issue<NW, RB, BUF>(abuf[b ^ 1], mtile, K, k, c0, lane, w, src, cin, live, &rs);
            shared_regs<RB, SC, BUF>(mtile, K, k, c0, lane, o, i, col, sscale, pscale, Wt, cin, cout, live, nx, s1, s2,
                                     vv, &rs);
            __builtin_amdgcn_sched_barrier(0);
            const int cbb = cj + 16 * h;
            if constexpr (PRE || SC) {  // without both the factor is 1 and missing rows are zero already
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        cu.a[rb][r] =
                                (PRE ? pre_act(cu.a[rb][r], lps[cbb + r], lpb[cbb + r]) : cu.a[rb][r]) * cu.sc[rb];
            }
            mfma_stage_rb<NT, RB>(cu, acc);
            // the MFMAs stay above the wait: left to the scheduler, all but one
            // sank below it, so stage j+1's loads were waited on before stage j
            // multiplied (no overlap of the gather latency with the MFMAs)
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own share of stage j+1 landed
            __syncthreads();  // every share landed; stage j's buffer free
        }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        if (nsplit > 1) {
            split_store_finish(acc[rb], orow + 32 * rb, h, col, lane, s, nsplit, n_out, cout, part, counters,
                               ((static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * NW + w) * RB + rb,
                               oscale, bias, residual, out);
            continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t orr = orow[32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h];
            if (orr >= 0 && col < cout) {
                float v = acc[rb][r];
                if (oscale) v *= oscale[orr];
                if (bias) v += bias[col];
                if (residual) v += residual[orr * cout + col];
                out[orr * cout + col] = v;
            }
        }
    }
}

// --------------------------------------------------------------------------
// implicit GEMM on presplit operands (bf16x6 / bf16x3, the default product
// precision): the hi / mid / lo split of every operand element is done ONCE
// per call by presplit_kernel — per input row (with the eval prologue and the
// row importance folded in, as gemm_finish applies them) and per filter
// element — instead of once per (row, column block, stage) inside the GEMM:
// the split kernels above spend ~11 VALU instructions per MFMA on it (VALU-
// bound: 21.8 VALU per MFMA measured with addressing), here the stage loop is
// DMA + ds_read + MFMA only.  The planes hold exactly the values
// split_bf16x8 produces in the other kernels and the MFMAs run in the same
// order, so the sums are bit-identical to implicit_gemm_lds/shared_kernel.
// Needs cin % 8 == 0 (16-B pieces of 8 bf16) and no per-pair scale (pscale:
// neighbour importance, which cannot be folded per row).
//
// Tile: 32 output rows x NW column blocks (wave w: block w).  A per plane:
// LDS image [32 rows][4 pieces of 16 B], piece p of row r in slot
// p ^ ((r >> 2) & 3) (lane (i, h) reads pieces 2h, 2h + 1 of row i: 16
// consecutive lanes hit 16 distinct 4-bank groups), filled with
// global_load_lds_dwordx4 (16 rows per instruction, the NP planes x 2 halves
// dealt over the NW waves); double-buffered when NW > 1 (a barrier per stage
// publishes it), single-buffered for one wave.  B fragments come straight
// from the filter planes into registers (L2-resident).
// --------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(256) presplit_kernel(const float* __restrict__ x, int64_t n, int cin,
                                                       const float* __restrict__ ps, const float* __restrict__ pb,
                                                       const float* __restrict__ rscale, bf16x8* __restrict__ hi,
                                                       bf16x8* __restrict__ mid, bf16x8* __restrict__ lo) {
    const int g8 = cin >> 3;
    const int64_t total = n * g8;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = e / g8;
        const int c = static_cast<int>(e - r * g8) * 8;
        const float4 v0 = *reinterpret_cast<const float4*>(x + r * cin + c);
        const float4 v1 = *reinterpret_cast<const float4*>(x + r * cin + c + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        const float sc = rscale ? rscale[r] : 1.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (ps ? pre_act(v[j], ps[c + j], pb[c + j]) : v[j]) * sc;
        bf16x8 h, m, l;
        split_bf16x8<NT>(v, h, m, l);
        hi[e] = h;
        mid[e] = m;
        if constexpr (NT == 6) lo[e] = l;
    }
}

template <int NT, int NW, int RB>
__global__ void __launch_bounds__(NW * 64)
implicit_gemm_split_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ order, const int* order_flag,
                           int K, int64_t n_out, const __bf16* __restrict__ ap, int64_t plane_a,
                           const __bf16* __restrict__ bp /*[plane][K][cout][cin]*/, int64_t plane_b, int cin,
                           int cout, const float* __restrict__ oscale, const float* __restrict__ bias,
                           float* __restrict__ out, int nsplit, float* __restrict__ part,
                           const float* __restrict__ residual, uint32_t* __restrict__ counters) {
    constexpr int NP = NT == 6 ? 3 : 2;  // planes: hi, mid (, lo)
    constexpr int NB = NW == 1 ? 1 : 2;  // A image buffers
    constexpr int R = 32 * RB;           // output rows per tile
    constexpr int NI = 2 * NP * RB;      // DMA instructions per stage (16 rows of one plane each)
    __shared__ __attribute__((aligned(16))) __bf16 abuf[NB][RB][NP][32 * 32];
    __shared__ int32_t mtile[R * 32];
    __shared__ int32_t orow[R];
    const int64_t o0 = static_cast<int64_t>(blockIdx.x) * R;
    if (o0 >= n_out) return;  // whole workgroup, before any barrier
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int i = lane & 31, h = lane >> 5;
    const int col = (blockIdx.y * NW + w) * 32 + i;
    if (order && *order_flag == 0) order = nullptr;
    for (int t = threadIdx.x; t < R; t += NW * 64) {
        const int64_t oo = o0 + t;
        orow[t] = oo < n_out ? (order ? order[oo] : static_cast<int32_t>(oo)) : -1;
    }
    __syncthreads();
    load_map_tile<R, NW * 64>(map, orow, K, threadIdx.x, mtile);
    __syncthreads();
    unsigned used = 0u;  // identical in every wave (same rows)
    for (int k = h; k < K; k += 2) {
        bool any = false;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) any |= mtile[(32 * rb + i) * K + k] >= 0;
        const uint64_t b = __ballot(any);
        used |= ((h ? (b >> 32) : (b & 0xffffffffull)) != 0ull) ? (1u << k) : 0u;
    }
    used = __builtin_amdgcn_readlane(used, 32) | __builtin_amdgcn_readlane(used, 0);
    f32x16 acc[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[rb][r] = 0.f;
    const int nch = (cin + 31) >> 5;
    const int s = blockIdx.z;
    const int j0 = split_stage(used, nch, K, s, nsplit);
    const int j1 = split_stage(used, nch, K, s + 1, nsplit);
    const __bf16* zp = reinterpret_cast<const __bf16*>(g_zero_page);
    // this wave's DMA share of one stage: instructions q = w, w + NW, ... of
    // the NI (row block, plane, 16-row half) triples; map reads first, then the DMAs
    auto issue = [&](int buf, int k, int c0, bool live) {
        constexpr int NQ = (NI + NW - 1) / NW;
        int32_t mq[NQ];
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            const int q = w + NW * t;
            const int r = 32 * (q / (2 * NP)) + 16 * (q & 1) + (lane >> 2);
            mq[t] = (q < NI && live) ? mtile[r * K + k] : -1;
        }
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            const int q = w + NW * t;
            if (q >= NI) continue;  // wave-uniform
            const int rb = q / (2 * NP), pl = (q % (2 * NP)) >> 1;
            const int r = 16 * (q & 1) + (lane >> 2);  // row within the block
            const int c = c0 + 8 * ((lane & 3) ^ ((r >> 2) & 3));
            const __bf16* ga = (mq[t] >= 0 && c < cin) ? ap + pl * plane_a + static_cast<int64_t>(mq[t]) * cin + c : zp;
            glds16(reinterpret_cast<const float*>(ga),
                   reinterpret_cast<float*>(&abuf[buf][rb][pl][16 * 32 * (q & 1)]));
        }
    };
    auto bload = [&](bf16x8 (&nb)[NP][2], int k, int c0, bool live) {
        const bool colv = live && col < cout;
        const int64_t wo = (static_cast<int64_t>(k) * cout + (colv ? col : 0)) * cin;
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int c = c0 + 16 * h + 8 * t;
                nb[pl][t] = *reinterpret_cast<const bf16x8*>((colv && c < cin) ? bp + pl * plane_b + wo + c : zp);
            }
    };
    if (j0 < j1) {  // uniform over the workgroup
        unsigned u = used;
        for (int t = j0 / nch; t > 0; --t) u &= u - 1u;
        int k = __builtin_ctz(u), c0 = (j0 % nch) * 32;
        bf16x8 nb[NP][2];
        issue(0, k, c0, true);
        bload(nb, k, c0, true);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int j = j0; j < j1; ++j) {
            const int buf = NB == 1 ? 0 : ((j - j0) & 1);
            bf16x8 fa[RB][NP][2], fb[NP][2];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int pl = 0; pl < NP; ++pl)
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int slot = (2 * h + t) ^ ((i >> 2) & 3);
                        fa[rb][pl][t] = *reinterpret_cast<const bf16x8*>(&abuf[buf][rb][pl][32 * i + 8 * slot]);
                    }
#pragma unroll
            for (int pl = 0; pl < NP; ++pl)
#pragma unroll
                for (int t = 0; t < 2; ++t) fb[pl][t] = nb[pl][t];
            c0 += 32;
            if (c0 >= cin) {
                c0 = 0;
                u &= u - 1u;
                k = u ? __builtin_ctz(u) : 0;
            }
            const bool live = j + 1 < j1;
            // one buffer: this stage's fragments are out of LDS before the next DMA
            if constexpr (NB == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(NB == 1 ? 0 : buf ^ 1, k, c0, live);
            bload(nb, k, c0, live);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 2; ++t)  // per accumulator: the order of mfma_stage_split
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) {
                    if constexpr (NT == 6) {
                        acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][1][t], fb[1][t], acc[rb], 0, 0, 0);
                        acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][2][t], fb[0][t], acc[rb], 0, 0, 0);
                        acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][0][t], fb[2][t], acc[rb], 0, 0, 0);
                    }
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][1][t], fb[0][t], acc[rb], 0, 0, 0);
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][0][t], fb[1][t], acc[rb], 0, 0, 0);
                    acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb][0][t], fb[0][t], acc[rb], 0, 0, 0);
                }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own share of stage j+1 landed
            __syncthreads();  // every share landed; stage j's buffer free
        }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        if (nsplit > 1) {
            split_store_finish(acc[rb], orow + 32 * rb, h, col, lane, s, nsplit, n_out, cout, part, counters,
                               ((static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * NW + w) * RB + rb,
                               oscale, bias, residual, out);
            continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t orr = orow[32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h];
            if (orr >= 0 && col < cout) {
                float v = acc[rb][r];
                if (oscale) v *= oscale[orr];
                if (bias) v += bias[col];
                if (residual) v += residual[orr * cout + col];
                out[orr * cout + col] = v;
            }
        }
    }
}

// --------------------------------------------------------------------------
// dW: per offset pair lists, split-K slabs
// --------------------------------------------------------------------------
// k-major flags: flag[k*n_out + o] = map[o*K+k] >= 0
__global__ void pair_flags_kernel(const int32_t* __restrict__ map, int64_t n_out, int K, int64_t* __restrict__ flags) {
    const int64_t total = n_out * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = e / n_out, o = e - k * n_out;
        flags[e] = map[o * K + k] >= 0 ? 1 : 0;
    }
}

__global__ void pair_lists_kernel(const int32_t* __restrict__ map, int64_t n_out, int K, const int64_t* __restrict__ incl,
                                  int32_t* __restrict__ po, int64_t* __restrict__ kstart) {
    const int64_t total = n_out * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = e / n_out, o = e - k * n_out;
        if (map[o * K + k] >= 0) po[incl[e] - 1] = static_cast<int32_t>(o);
        if (o == 0) kstart[k] = e == 0 ? 0 : incl[e - 1];
        if (e == total - 1) kstart[K] = incl[e];
    }
}

// dW[k] tile (ci0, co0) of 32 x 32 over one chunk of offset k's pair list,
// one wave per (tile, k, chunk): the pairs are the MFMA reduction index, so
// lane (i, h) gathers x[in_p][ci0 + i] and g[out_p][co0 + i] of pair
// 2s + h straight into the v_mfma_f32_32x32x2_f32 operand registers (32
// consecutive channels of one row per half-wave: coalesced).  The chunk's
// pair records (out row, in row, scales) are staged in LDS kDwSub at a time,
// so a stage's gathers depend on LDS reads only and the next stage's gathers
// are in flight while the current 16 MFMAs run.  No barriers beyond the wave.
// part[chunk][cin][cout] (dw_plan_kernel).
constexpr int kDwSub = 512;

struct DwStage {
    float a[16], b[16];
};

__device__ __forceinline__ void dw_load(DwStage& st, int base, int h, const int32_t* lo, const int32_t* lm,
                                        const float* lra, const float* lrb, const float* __restrict__ src,
                                        const float* __restrict__ g, int cin, int cout, int ci, int co,
                                        bool live = true) {
    // unconditional loads, absent data read from the zero page (see gemm_load);
    // a dead stage (past the sub-chunk) reads only the zero page
    const bool cv = live && ci < cin, ov = live && co < cout;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int pp = base + 2 * s + h;
        const int32_t mo = lo[pp], mi = lm[pp];
        st.a[s] = *((cv && mi >= 0) ? src + static_cast<int64_t>(mi) * cin + ci : g_zero_page);
        st.b[s] = *((ov && mo >= 0) ? g + static_cast<int64_t>(mo) * cout + co : g_zero_page);
    }
}

__device__ __forceinline__ void dw_finish(DwStage& st, int base, int h, const float* lra, const float* lrb) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int pp = base + 2 * s + h;
        st.a[s] *= lra[pp];
        st.b[s] *= lrb[pp];
    }
}

// Chunk plan of the dW pair lists (one thread): chunks of one length L over
// every offset's list, so the waves get equal pair counts however unevenly the
// offsets are used (the centre offset of a submanifold conv has every output,
// corner offsets a fraction: per-offset chunk counts left the centre's waves
// 3x longer than the average).  plan[k] = first chunk (= partial slab) of
// offset k, plan[K] = number of chunks, plan[K + 1] = L.  direct: one chunk
// per offset (slab k = grad_filters[k], no reduce).
__global__ void dw_plan_kernel(const int64_t* __restrict__ kstart, int K, int64_t max_chunks, int direct,
                               int64_t* __restrict__ plan) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t P = kstart[K];
    // smallest L with sum_k ceil(n_k / L) <= max_chunks: L = ceil(P / (max_chunks - K)) suffices
    const int64_t L = direct ? (int64_t(1) << 62)
                             : max<int64_t>(1, (P + (max_chunks - K) - 1) / max<int64_t>(1, max_chunks - K));
    int64_t c = 0;
    for (int k = 0; k < K; ++k) {
        plan[k] = c;
        c += direct ? 1 : (kstart[k + 1] - kstart[k] + L - 1) / L;
    }
    plan[K] = c;
    plan[K + 1] = L;
}

template <int NT>
__global__ void __launch_bounds__(64)
dweight_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ po, const int64_t* __restrict__ kstart, int K,
               const int64_t* __restrict__ plan, const float* __restrict__ src, const float* __restrict__ sscale,
               const float* __restrict__ pscale, const float* __restrict__ g, const float* __restrict__ oscale, int cin,
               int cout, float* __restrict__ part) {
    __shared__ int32_t lo[kDwSub], lm[kDwSub];
    __shared__ float lra[kDwSub], lrb[kDwSub];
    const int ncot = (cout + 31) >> 5;
    const int ci0 = (blockIdx.x / ncot) * 32, co0 = (blockIdx.x % ncot) * 32;
    const int64_t w = blockIdx.y;  // chunk = partial slab
    if (w >= plan[K]) return;      // whole wave (grid sized for the worst case)
    int k = 0;
    while (plan[k + 1] <= w) ++k;  // uniform scan; empty offsets own no chunk
    const int lane = threadIdx.x, i = lane & 31, h = lane >> 5;
    const int64_t js = kstart[k] + (w - plan[k]) * plan[K + 1];
    const int64_t je = min(kstart[k + 1], js + plan[K + 1]);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int64_t sub = js; sub < je; sub += kDwSub) {
        const int n = static_cast<int>(min(static_cast<int64_t>(kDwSub), je - sub));
        for (int t = lane; t < kDwSub; t += 64) {
            int32_t o = -1, m = -1;
            float ra = 0.f, rb = 0.f;
            if (t < n) {
                o = po[sub + t];
                m = map[static_cast<int64_t>(o) * K + k];
                ra = (sscale ? sscale[m] : 1.f) * (pscale ? pscale[static_cast<int64_t>(o) * K + k] : 1.f);
                rb = oscale ? oscale[o] : 1.f;
            }
            lo[t] = o;
            lm[t] = m;
            lra[t] = ra;
            lrb[t] = rb;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nst = (n + 31) >> 5;
        // two stage buffers in ping-pong, loads issued unconditionally (a dead
        // stage reads the zero page): no register copy and no branch around the
        // loads, so the next stage's loads stay in flight under these MFMAs
        // (a `cur = nxt` copy made every stage wait for the loads just issued)
        DwStage sa, sb;
        dw_load(sa, 0, h, lo, lm, lra, lrb, src, g, cin, cout, ci0 + i, co0 + i);
        for (int j = 0;; j += 2) {
            const bool lb = j + 1 < nst;
            dw_load(sb, lb ? 32 * (j + 1) : 0, h, lo, lm, lra, lrb, src, g, cin, cout, ci0 + i, co0 + i, lb);
            __builtin_amdgcn_sched_barrier(0);
            dw_finish(sa, 32 * j, h, lra, lrb);
            mfma_stage<NT>(sa, acc);  // split forms: element j of MFMA t = pair 2(8t + j) + h
            if (!lb) break;
            const bool la = j + 2 < nst;
            dw_load(sa, la ? 32 * (j + 2) : 0, h, lo, lm, lra, lrb, src, g, cin, cout, ci0 + i, co0 + i, la);
            __builtin_amdgcn_sched_barrier(0);
            dw_finish(sb, 32 * (j + 1), h, lra, lrb);
            mfma_stage<NT>(sb, acc);
            if (!la) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // LDS records are rewritten by the next sub-chunk
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    float* P = part + w * cin * cout;
    const int col = co0 + i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = ci0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < cin && col < cout) P[static_cast<int64_t>(row) * cout + col] = acc[r];
    }
}

// dW with the stage's rows staged through LDS (cin, cout % 4 == 0, 16-B
// aligned rows): the 32 pairs' x segments (32 channels = one 128-B line per
// pair) and g segments arrive by global_load_lds_dwordx4, 4 instructions per
// operand (8 lanes per line) instead of 16 single-dword gathers each, and are
// read back in the MFMA layout with conflict-free ds_read_b32 (lanes = the 32
// consecutive channels of one pair's row).  One buffer per operand: stage j
// is read into registers, then stage j+1's DMA goes into the same buffers and
// runs under stage j's MFMAs.  Same element -> pair map as dweight_kernel
// (element s = pair 2s + h), so the same sums.
constexpr int kDwSubL = 256;

template <int NT>
__global__ void __launch_bounds__(64)
dweight_lds_kernel(const int32_t* __restrict__ map, const int32_t* __restrict__ po,
                   const int64_t* __restrict__ kstart, int K, const int64_t* __restrict__ plan,
                   const float* __restrict__ src, const float* __restrict__ sscale, const float* __restrict__ pscale,
                   const float* __restrict__ g, const float* __restrict__ oscale, int cin, int cout,
                   float* __restrict__ part) {
    __shared__ int32_t lo[kDwSubL], lm[kDwSubL];
    __shared__ float lra[kDwSubL], lrb[kDwSubL];
    __shared__ __attribute__((aligned(16))) float xbuf[32 * 32], gbuf[32 * 32];
    const int ncot = (cout + 31) >> 5;
    const int ci0 = (blockIdx.x / ncot) * 32, co0 = (blockIdx.x % ncot) * 32;
    const int64_t w = blockIdx.y;
    if (w >= plan[K]) return;
    int k = 0;
    while (plan[k + 1] <= w) ++k;
    const int lane = threadIdx.x, i = lane & 31, h = lane >> 5, sl = lane & 7;
    const int64_t js = kstart[k] + (w - plan[k]) * plan[K + 1];
    const int64_t je = min(kstart[k + 1], js + plan[K + 1]);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // DMA of the 32 pairs at base: pair base + 8q + (lane >> 3), 16-B piece sl
    auto issue = [&](int base, bool live) {
        int32_t mq[4], oq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int pp = base + 8 * q + (lane >> 3);
            mq[q] = live ? lm[pp] : -1;
            oq[q] = live ? lo[pp] : -1;
        }
        const int ci = ci0 + 4 * sl, co = co0 + 4 * sl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float* ga = (mq[q] >= 0 && ci < cin) ? src + static_cast<int64_t>(mq[q]) * cin + ci : g_zero_page;
            const float* gb = (oq[q] >= 0 && co < cout) ? g + static_cast<int64_t>(oq[q]) * cout + co : g_zero_page;
            glds16(ga, xbuf + 256 * q);
            glds16(gb, gbuf + 256 * q);
        }
    };
    for (int64_t sub = js; sub < je; sub += kDwSubL) {
        const int n = static_cast<int>(min(static_cast<int64_t>(kDwSubL), je - sub));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight over the record rewrite
        for (int t = lane; t < kDwSubL; t += 64) {
            int32_t o = -1, m = -1;
            float ra = 0.f, rb = 0.f;
            if (t < n) {
                o = po[sub + t];
                m = map[static_cast<int64_t>(o) * K + k];
                ra = (sscale ? sscale[m] : 1.f) * (pscale ? pscale[static_cast<int64_t>(o) * K + k] : 1.f);
                rb = oscale ? oscale[o] : 1.f;
            }
            lo[t] = o;
            lm[t] = m;
            lra[t] = ra;
            lrb[t] = rb;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nst = (n + 31) >> 5;
        issue(0, true);
        for (int j = 0; j < nst; ++j) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage j in LDS
            DwStage cu;
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) {
                const int pp = 2 * s2 + h;
                cu.a[s2] = xbuf[pp * 32 + i];
                cu.b[s2] = gbuf[pp * 32 + i];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // buffers read out before the next DMA
            issue(32 * (j + 1) < kDwSubL ? 32 * (j + 1) : 0, j + 1 < nst);
            __builtin_amdgcn_sched_barrier(0);
            dw_finish(cu, 32 * j, h, lra, lrb);
            mfma_stage<NT>(cu, acc);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dead DMA has landed before the wave exits
    float* P = part + w * cin * cout;
    const int col = co0 + i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = ci0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < cin && col < cout) P[static_cast<int64_t>(row) * cout + col] = acc[r];
    }
}

__global__ void reduce_slabs_kernel(const float* __restrict__ part, int K, const int64_t* __restrict__ plan,
                                    int64_t slab, float* __restrict__ dw) {
    const int64_t total = static_cast<int64_t>(K) * slab;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = e / slab, r = e - k * slab;
        // fixed order (0 for an unused offset): 8 interleaved partial sums over
        // the offset's chunks ascending, combined pairwise — 8 independent loads
        // in flight per thread instead of one serial chain
        const int64_t c0 = plan[k], c1 = plan[k + 1];
        float p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int64_t c = c0;
        for (; c + 8 <= c1; c += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] += part[(c + u) * slab + r];
        }
        for (int u = 0; c < c1; ++c, ++u) p[u] += part[c * slab + r];
        const float s = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
        dw[e] = s;
    }
}

// kernel index of each (query, input) pair (the rulebook of layers.SparseConv)
__global__ void kernel_index_kernel(const float* __restrict__ inp_pos, const float* __restrict__ qpos,
                                    const int32_t* __restrict__ nbr, const int64_t* __restrict__ rs, int64_t n_query,
                                    int k0, int k1, int k2, float inv_vs, int mirror, int32_t* __restrict__ kidx) {
    for (int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; q < n_query;
         q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const float qx = qpos[3 * q], qy = qpos[3 * q + 1], qz = qpos[3 * q + 2];
        for (int64_t e = rs[q], ee = rs[q + 1]; e < ee; ++e) {
            const int64_t i = nbr[e];
            const float qq[3] = {qx, qy, qz};
            const int kd[3] = {k2, k1, k0};  // x <-> filter dim 2, z <-> dim 0
            int id[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const float rel = (inp_pos[3 * i + d] - qq[d]) * inv_vs;
                const float h = 0.5f * static_cast<float>(kd[d]);
                int v = static_cast<int>(floorf(mirror ? h - rel : rel + h));
                v = v < 0 ? 0 : (v >= kd[d] ? kd[d] - 1 : v);
                id[d] = v;
            }
            kidx[e] = (id[2] * k1 + id[1]) * k2 + id[0];
        }
    }
}

// Narrow inputs (cin <= 4: the network's first convolution on raw point
// features, 3 -> m channels): an MFMA tile would spend 29 of its 32 reduction
// lanes on zeros, so one lane per output row walks the K offsets with FMAs on
// the VALU instead — the filter words are wave-uniform (scalar loads), the
// map entries and then the gathered rows of 9 offsets are issued before their
// FMAs (packed v_pk_fma_f32, two columns per instruction).  COLS output channels per lane
// (cout % COLS == 0: no per-column guards, the filter words of an offset are
// one contiguous run of scalar loads); SC: row / pair scales.
// Per row: K map words + <= K*CIN*4 B gathered + COLS*4 B written.
template <int CIN, int COLS, bool SC>
__global__ void __launch_bounds__(256) small_cin_gemm_kernel(const int32_t* __restrict__ map, int K, int64_t n_out,
                                                             const float* __restrict__ src,
                                                             const float* __restrict__ sscale,
                                                             const float* __restrict__ pscale,
                                                             const float* __restrict__ Wt, int cout,
                                                             const float* __restrict__ oscale,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ residual, float* __restrict__ out) {
    const int64_t o = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    const int cb = blockIdx.y * COLS;
    const int64_t orow = o < n_out ? o : 0;  // lanes past the end compute row 0 and store nothing
    const int32_t* mrow = map + orow * K;
    float acc[COLS];
#pragma unroll
    for (int j = 0; j < COLS; ++j) acc[j] = 0.f;
    constexpr int KB = 9;  // offsets whose loads are in flight together (a 3^3 kernel: 3 blocks)
    for (int k0 = 0; k0 < K; k0 += KB) {
        int32_t m[KB];
#pragma unroll
        for (int t = 0; t < KB; ++t) m[t] = k0 + t < K ? mrow[k0 + t] : -1;
        float x[KB][CIN];
#pragma unroll
        for (int t = 0; t < KB; ++t) {
            const bool valid = m[t] >= 0;
            const int64_t mr = valid ? m[t] : 0;
            const float* row = valid ? src + mr * CIN : g_zero_page;
#pragma unroll
            for (int c = 0; c < CIN; ++c) x[t][c] = row[c];
            if constexpr (SC) {
                const float f = valid ? *(sscale ? sscale + mr : g_one_page) *
                                                *(pscale ? pscale + orow * K + k0 + t : g_one_page)
                                      : 0.f;
#pragma unroll
                for (int c = 0; c < CIN; ++c) x[t][c] *= f;
            }
        }
#pragma unroll
        for (int t = 0; t < KB; ++t) {
            if (k0 + t >= K) break;
            const float* w = Wt + (static_cast<int64_t>(k0 + t) * cout + cb) * CIN;
#pragma unroll
            for (int j = 0; j < COLS; ++j) {
#pragma unroll
                for (int c = 0; c < CIN; ++c) acc[j] = fmaf(x[t][c], w[j * CIN + c], acc[j]);
            }
        }
    }
    if (o >= n_out) return;
#pragma unroll
    for (int j = 0; j < COLS; ++j) {
        const int col = cb + j;
        float v = acc[j];
        if (oscale) v *= oscale[o];
        if (bias) v += bias[col];
        if (residual) v += residual[o * cout + col];
        out[o * cout + col] = v;
    }
}

// O3DML_GEMM_SMALL_CIN=0: cin <= 4 on the generic MFMA kernel (A/B)
constexpr int kSmallCols = 16;
static bool use_small_cin(int cin, int cout) {
    static const bool on = [] {
        const char* e = std::getenv("O3DML_GEMM_SMALL_CIN");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on && cin >= 1 && cin <= 4 && cout % kSmallCols == 0;
}

static void launch_small_cin(hipStream_t st, const int32_t* map, int K, int64_t n_out, const float* src,
                             const float* sscale, const float* pscale, const float* Wt, int cin, int cout,
                             const float* oscale, const float* bias, const float* residual, float* out) {
    const dim3 g(static_cast<unsigned>(ceil_div(n_out, 256)), static_cast<unsigned>(cout / kSmallCols));
#define O3DML_SMALL(C, S)                                                                                    \
    small_cin_gemm_kernel<C, kSmallCols, S><<<g, 256, 0, st>>>(map, K, n_out, src, sscale, pscale, Wt, cout, \
                                                               oscale, bias, residual, out)
#define O3DML_SMALL_K(C)                              \
    do {                                              \
        if (sscale || pscale) O3DML_SMALL(C, true);   \
        else O3DML_SMALL(C, false);                   \
    } while (0)
    switch (cin) {
        case 1: O3DML_SMALL_K(1); break;
        case 2: O3DML_SMALL_K(2); break;
        case 3: O3DML_SMALL_K(3); break;
        default: O3DML_SMALL_K(4); break;
    }
#undef O3DML_SMALL_K
#undef O3DML_SMALL
    O3DML_LAUNCH_CHECK();
}

// out[o, c] = (sum_s part[s][o, c]) * oscale[o] + bias[c], splits in order
__global__ void split_reduce_kernel(const float* __restrict__ part, int nsplit, int64_t n_out, int cout,
                                    const float* __restrict__ oscale, const float* __restrict__ bias,
                                    const float* __restrict__ residual, float* __restrict__ out) {
    const int64_t total = n_out * cout;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float v = sum_slabs(part, nsplit, total, e);
        const int64_t o = e / cout;
        if (oscale) v *= oscale[o];
        if (bias) v += bias[e - o * cout];
        if (residual) v += residual[e];
        out[e] = v;
    }
}

// Split of the (offset, Cin-chunk) reduction across waves when the output
// tiles alone cannot fill the chip (deep UNet levels: a few hundred rows, up to
// 448 input channels): enough splits for ~kGemmTargetWaves waves, at least
// kGemmMinStages stages each, partial sums bounded by kGemmSplitBytes.
constexpr int64_t kGemmTargetWaves = 4096;
constexpr int kGemmMinStages = 4;
constexpr int64_t kGemmSplitBytes = int64_t(64) << 20;

// Product precision of the gather-GEMMs (mfma_stage_split): 1 = exact
// f32-input MFMA (default: IEEE f32 products, infinities kept), 0 = bf16x6
// (f32-accurate for finite inputs, a +-inf input turns the outputs that
// gather it into NaN), 2 = bf16x3.  bf16x6 was the default until round 5; it
// measured 1.20x (32 -> 32) / 1.24x (128 -> 128) faster per GEMM and equal on
// the host-bound SparseConvUnet frame (tools/scn_precision_ab.sh), too little
// for its non-finite deviation.  Env O3DML_SPARSE_CONV_EXACT sets the initial
// mode; o3dml_sparse_conv_set_exact.
static int g_gemm_mode = -1;
static int gemm_mode() {
    if (g_gemm_mode < 0) {
        const char* e = std::getenv("O3DML_SPARSE_CONV_EXACT");
        const int v = e ? std::atoi(e) : 1;
        g_gemm_mode = (v == 0 || v == 2) ? v : 1;
    }
    return g_gemm_mode;
}
static int gemm_nt() {  // template argument of the kernels: 0 exact, 3, 6 splits
    const int m = gemm_mode();
    return m == 1 ? 0 : (m == 2 ? 3 : 6);
}

static int gemm_splits(int64_t n_out, int K, int cin, int cout) {
    if (n_out <= 0 || cout <= 0) return 1;
    static const int64_t target = [] {
        const char* e = std::getenv("O3DML_GEMM_TARGET_WAVES");
        return e ? std::max<int64_t>(1, std::atoll(e)) : kGemmTargetWaves;
    }();
    const int64_t tiles = ceil_div(n_out, 32) * ceil_div(cout, 32);
    // O3DML_GEMM_NOSPLIT_TILES = v > 0 (A/B): no split once the output tiles
    // number >= v (the partial slabs and the reduce launch vs occupancy)
    static const int64_t nosplit = [] {
        const char* e = std::getenv("O3DML_GEMM_NOSPLIT_TILES");
        return e ? std::atoll(e) : 0;
    }();
    if (nosplit > 0 && tiles >= nosplit) return 1;
    int64_t ns = ceil_div(target, tiles);
    ns = std::min<int64_t>(ns, std::max<int64_t>(1, (static_cast<int64_t>(K) * ceil_div(cin, 32)) / kGemmMinStages));
    ns = std::min<int64_t>(ns, kGemmSplitBytes / (n_out * cout * static_cast<int64_t>(sizeof(float))));
    // O3DML_GEMM_MAX_SPLITS (A/B): cap on the splits (the reduce reads every slab)
    static const int64_t cap = [] {
        const char* e = std::getenv("O3DML_GEMM_MAX_SPLITS");
        const int64_t v = e ? std::atoll(e) : 64;
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ns, cap)));
}

// Persistent grid of implicit_gemm_lds_kernel: O3DML_GEMM_PERSIST = v > 0
// launches v x the resident workgroups (occupancy x CUs) when the work has
// more waves than that, the waves looping over the items; 0 = one wave per item
static int gemm_persist() {
    static const int v = [] {
        const char* e = std::getenv("O3DML_GEMM_PERSIST");
        return e ? std::max(0, std::atoi(e)) : 1;
    }();
    return v;
}
template <auto Kern>
static int resident_blocks() {  // once per instantiation (one device per process)
    static const int v = [] {
        int nb = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, Kern, kGemmThreads, 0) != hipSuccess) nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
        return nb * cus;
    }();
    return v;
}
template <auto Kern>
static dim3 persist_grid(dim3 g, GemmPrologue& pp) {
    const int64_t rb = static_cast<int64_t>(resident_blocks<Kern>()) * gemm_persist();
    if (rb <= 0 || static_cast<int64_t>(g.x) * g.y * g.z <= rb) return g;
    pp.pcols = static_cast<int>(g.y);
    return dim3(static_cast<unsigned>(rb), 1, 1);
}

static size_t gemm_split_bytes(int64_t n_out, int K, int cin, int cout) {
    const int ns = gemm_splits(n_out, K, cin, cout);
    return ns > 1 ? ws_bytes<float>(ns * n_out * cout) : 0;
}

// Presplit operands (implicit_gemm_split_kernel) — OFF by default: measured
// on the C4 3^3 map (tools/gemm_probe.py, profiles/r03/sparse_conv_presplit_ab.txt)
// it is slower than the in-kernel split at every width and row blocking
// (32->32: 78 vs 69.5 us, 128->128: 382 vs 367 us at its best RB = 2).  The
// in-kernel split's VALU work hides under the MFMA / L2 latency; what bounds
// these kernels is the L2 -> LDS / register traffic of the gathered rows and
// the per-stage filter fragments, which the 6-B bf16 planes raise by 1.5x.
// O3DML_GEMM_PRESPLIT=1 or o3dml_sparse_conv_set_presplit(1) turns it on.
static bool g_presplit = [] {
    const char* e = std::getenv("O3DML_GEMM_PRESPLIT");
    return e ? std::atoi(e) != 0 : false;
}();

// presplit operand planes: 3 bf16 planes of the n_src x cin source rows and of
// the K x cout x cin filters (0 while presplit is off)
static size_t presplit_bytes(int64_t n_src, int K, int cin, int cout) {
    if (!g_presplit) return 0;
    return 3 * ws_bytes<uint16_t>(n_src * cin) + 3 * ws_bytes<uint16_t>(static_cast<int64_t>(K) * cout * cin);
}

// everything run_gemm may take from its workspace
// Filters split once per call for the per-wave kernel (split_filters_kernel,
// BS): the B operand's hi / mid / lo come from a 6-B-per-weight copy instead
// of three roundings per stage in every wave.  O3DML_GEMM_BSPLIT=0 or
// o3dml_sparse_conv_set_bsplit(0) turns it off (same bits either way).
static bool g_bsplit = [] {
    const char* e = std::getenv("O3DML_GEMM_BSPLIT");
    return e ? std::atoi(e) != 0 : true;
}();
static size_t bsplit_bytes(int K, int cin, int cout) {
    return cin == 32 ? ws_bytes<uint16_t>(3 * static_cast<int64_t>(K) * cout * cin) : 0;
}

static size_t gemm_ws_bytes(int64_t n_out, int64_t n_src, int K, int cin, int cout) {
    return gemm_split_bytes(n_out, K, cin, cout) + presplit_bytes(n_src, K, cin, cout) + bsplit_bytes(K, cin, cout);
}

static void run_gemm(hipStream_t st, const int32_t* map, const int32_t* order, const int* order_flag, int K,
                     int64_t n_out, const float* src, int64_t n_src, const float* sscale, const float* pscale,
                     const float* Wt, int cin, int cout, const float* oscale, const float* bias, float* out,
                     Workspace ws, GemmPrologue pre = {nullptr, nullptr}, const float* residual = nullptr,
                     const int32_t* tmap = nullptr) {
    if (n_out == 0 || cout == 0) return;
    pre.tmap = order && use_tile_map() ? tmap : nullptr;
    const bool vec4 = (cin % 4) == 0 && (reinterpret_cast<uintptr_t>(src) % 16) == 0 &&
                      (reinterpret_cast<uintptr_t>(Wt) % 16) == 0;
    int ns = gemm_splits(n_out, K, cin, cout);
    float* part = nullptr;
    if (ns > 1) {
        const size_t pb = ws_bytes<float>(static_cast<int64_t>(ns) * n_out * cout);
        if (ws.base && ws.used + pb <= ws.size) part = ws.take<float>(static_cast<int64_t>(ns) * n_out * cout);
        else ns = 1;
    }
    const dim3 g(static_cast<unsigned>(round8(ceil_div(n_out, 32 * (kGemmThreads / 64)))),
                 static_cast<unsigned>(ceil_div(cout, 32)), static_cast<unsigned>(ns));
    O3DML_REQUIRE(pre.scale == nullptr || cin <= kPreMax, "sparse_conv: prologue needs cin <= %d", kPreMax);
    // split-K finished by each tile's last wave (split_store_finish); the wave
    // tiles of every kernel variant number ceil(n_out / 32) x ceil(cout / 32)
    // rounded up to whole workgroups
    // OFF by default: neutral on the C4 layer (0.172-0.177 ms either way, same
    // session) — kept selectable (O3DML_GEMM_FUSED_REDUCE=1), bit-identical
    static const bool fused_reduce = [] {
        const char* e = std::getenv("O3DML_GEMM_FUSED_REDUCE");
        return e ? std::atoi(e) != 0 : false;
    }();
    uint32_t* counters = nullptr;
    if (ns > 1 && fused_reduce)
        counters = tile_counters(st, (ceil_div(n_out, 128) + 1) * 4 * (ceil_div(cout, 32) + 4));
    const int nt_mode = gemm_nt();
    if (g_presplit && nt_mode != 0 && vec4 && cin % 8 == 0 && pscale == nullptr && ws.base &&
        ws.used + presplit_bytes(n_src, K, cin, cout) <= ws.size) {
        // operands split once (implicit_gemm_split_kernel); the split passes
        // belong to the GEMM's time
        TimedRegion tr("sparse_conv_gemm", st);
        const int64_t pa = n_src * cin, pbn = static_cast<int64_t>(K) * cout * cin;
        __bf16* ap = reinterpret_cast<__bf16*>(ws.take<uint16_t>(3 * pa));
        __bf16* bpl = reinterpret_cast<__bf16*>(ws.take<uint16_t>(3 * pbn));
        auto planes = [](__bf16* b, int64_t n) {
            return std::array<bf16x8*, 3>{reinterpret_cast<bf16x8*>(b), reinterpret_cast<bf16x8*>(b + n),
                                          reinterpret_cast<bf16x8*>(b + 2 * n)};
        };
        const auto A = planes(ap, pa), B = planes(bpl, pbn);
        if (n_src > 0) {
            if (nt_mode == 6)
                presplit_kernel<6><<<stream_grid(pa / 8, 256), 256, 0, st>>>(src, n_src, cin, pre.scale, pre.shift,
                                                                             sscale, A[0], A[1], A[2]);
            else
                presplit_kernel<3><<<stream_grid(pa / 8, 256), 256, 0, st>>>(src, n_src, cin, pre.scale, pre.shift,
                                                                             sscale, A[0], A[1], A[2]);
            O3DML_LAUNCH_CHECK();
        }
        if (nt_mode == 6)
            presplit_kernel<6><<<stream_grid(pbn / 8, 256), 256, 0, st>>>(Wt, static_cast<int64_t>(K) * cout, cin,
                                                                          nullptr, nullptr, nullptr, B[0], B[1], B[2]);
        else
            presplit_kernel<3><<<stream_grid(pbn / 8, 256), 256, 0, st>>>(Wt, static_cast<int64_t>(K) * cout, cin,
                                                                          nullptr, nullptr, nullptr, B[0], B[1], B[2]);
        O3DML_LAUNCH_CHECK();
        const int nw = cout >= 128 && cout % 128 == 0 ? 4 : (cout >= 64 ? 2 : 1);
        static const int env_rb = [] {
            const char* e = std::getenv("O3DML_GEMM_SPLIT_RB");
            return e ? std::atoi(e) : 0;
        }();
        // row blocks per tile: each B fragment (the filters, streamed from L2
        // per stage) feeds RB accumulators
        const int rb = env_rb == 1 || env_rb == 2 || env_rb == 4 ? env_rb : 2;
        const dim3 gs(static_cast<unsigned>(ceil_div(n_out, 32 * rb)), static_cast<unsigned>(ceil_div(cout, 32 * nw)),
                      static_cast<unsigned>(ns));
#define O3DML_GEMM_SP(NT, W, B)                                                                                   \
    implicit_gemm_split_kernel<NT, W, B><<<gs, W * 64, 0, st>>>(map, order, order_flag, K, n_out, ap, pa, bpl,    \
                                                                 pbn, cin, cout, oscale, bias, out, ns, part,      \
                                                                 residual, counters)
#define O3DML_GEMM_SP_W(NT, B)                                                                     \
    do {                                                                                           \
        if (nw == 4) O3DML_GEMM_SP(NT, 4, B); else if (nw == 2) O3DML_GEMM_SP(NT, 2, B); else O3DML_GEMM_SP(NT, 1, B); \
    } while (0)
#define O3DML_GEMM_SP_RB(NT)                                                                  \
    do {                                                                                      \
        if (rb == 4) O3DML_GEMM_SP_W(NT, 4); else if (rb == 2) O3DML_GEMM_SP_W(NT, 2); else O3DML_GEMM_SP_W(NT, 1); \
    } while (0)
        if (nt_mode == 6) O3DML_GEMM_SP_RB(6); else O3DML_GEMM_SP_RB(3);
#undef O3DML_GEMM_SP_RB
#undef O3DML_GEMM_SP_W
#undef O3DML_GEMM_SP
        O3DML_LAUNCH_CHECK();
        tr.end();
        if (ns > 1 && !counters) {
            split_reduce_kernel<<<stream_grid(n_out * cout, 256), 256, 0, st>>>(part, ns, n_out, cout, oscale, bias,
                                                                               residual, out);
            O3DML_LAUNCH_CHECK();
        }
        return;
    }
#define O3DML_GEMM_LAUNCH(V, P)                                                                                    \
    implicit_gemm_kernel<V, P><<<g, kGemmThreads, 0, st>>>(map, order, order_flag, K, n_out, src, sscale, pscale, Wt, cin, cout, oscale, \
                                                           bias, out, ns, part, pre, residual, counters)
    static const bool lds_path = [] {
        const char* e = std::getenv("O3DML_GEMM_LDS");
        return e ? std::atoi(e) != 0 : true;
    }();
    TimedRegion tr("sparse_conv_gemm", st);  // the GEMM kernel alone (bench roofline)
    if (use_small_cin(cin, cout) && !pre.scale) {  // no split: tile counters (if any) stay untouched
        launch_small_cin(st, map, K, n_out, src, sscale, pscale, Wt, cin, cout, oscale, bias, residual, out);
        return;
    }
    static const bool breg = [] {
        const char* e = std::getenv("O3DML_GEMM_BREG");
        return e ? std::atoi(e) != 0 : true;
    }();
    static const bool shared_path = [] {
        const char* e = std::getenv("O3DML_GEMM_SHARED");
        return e ? std::atoi(e) != 0 : true;
    }();
    // buffer addressing (rows and filters through buffer resources): whole
    // 32-channel stages, every byte offset of the operands below the
    // resources' out-of-range sentinel
    static const bool buf_path = [] {
        const char* e = std::getenv("O3DML_GEMM_BUF");
        return e ? std::atoi(e) != 0 : true;
    }();
    const bool buf_ok = buf_path && cin % 32 == 0 && static_cast<uint64_t>(n_src) * cin * 4 < kNoRow &&
                        static_cast<uint64_t>(K) * cout * cin * 4 < kNoRow - 64;
    if (buf_ok) {  // the resources cover exactly the operands
        pre.src_bytes = static_cast<uint32_t>(static_cast<uint64_t>(n_src) * cin * 4);
        pre.w_bytes = static_cast<uint32_t>(static_cast<uint64_t>(K) * cout * cin * 4);
    }
    // the shared-A kernel with buffer addressing: neutral in the same-session
    // A/B (64->96 -3 %, 128->128 +1-2 %: its row addresses are split over the
    // NW waves already) — off unless O3DML_GEMM_SHARED_BUF=1
    static const bool shared_buf = [] {
        const char* e = std::getenv("O3DML_GEMM_SHARED_BUF");
        return e ? std::atoi(e) != 0 : false;
    }();
    // O3DML_GEMM_NW1=1 (A/B): narrow outputs (cout < 64) on the shared-A
    // kernel with ONE wave per workgroup — with O3DML_GEMM_RB=2 a wave of 64
    // rows whose filter fragment feeds two accumulators
    static const bool nw1 = [] {
        const char* e = std::getenv("O3DML_GEMM_NW1");
        return e ? std::atoi(e) != 0 : false;
    }();
    if (vec4 && lds_path && shared_path && (cout >= 64 || nw1)) {
        // A tile shared by NW column-block waves (implicit_gemm_shared_kernel)
        const int nw = cout < 64 ? 1 : ((cout % 128 == 0) ? 4 : 2);
        static const int rb = [] {
            const char* e = std::getenv("O3DML_GEMM_RB");  // 2 row blocks per wave: measured slower
            return (e && std::atoi(e) == 2) ? 2 : 1;
        }();
        const dim3 gs(static_cast<unsigned>(round8(ceil_div(n_out, 32 * rb))),
                      static_cast<unsigned>(ceil_div(cout, 32 * nw)), static_cast<unsigned>(ns));
#define O3DML_GEMM_SH_SC(P, X, W, B, SCL)                                                                      \
    implicit_gemm_shared_kernel<P, X, W, B, SCL><<<gs, W * 64, 0, st>>>(map, order, order_flag, K, n_out, src,   \
                                                                        sscale, pscale, Wt, cin, cout, oscale,   \
                                                                        bias, out, ns, part, pre, residual,      \
                                                                        counters)
#define O3DML_GEMM_SH_BUF(P, X, W, B)                                                                          \
    implicit_gemm_shared_kernel<P, X, W, B, false, true><<<gs, W * 64, 0, st>>>(                               \
            map, order, order_flag, K, n_out, src, sscale, pscale, Wt, cin, cout, oscale, bias, out, ns, part, pre, \
            residual, counters)
#define O3DML_GEMM_SH(P, X, W, B)                                     \
    do {                                                              \
        if (sscale || pscale) O3DML_GEMM_SH_SC(P, X, W, B, true);     \
        else if (buf_ok && shared_buf) O3DML_GEMM_SH_BUF(P, X, W, B); \
        else O3DML_GEMM_SH_SC(P, X, W, B, false);                     \
    } while (0)
#define O3DML_GEMM_SH_RB(P, X, W) \
    if (rb == 2) O3DML_GEMM_SH(P, X, W, 2); else O3DML_GEMM_SH(P, X, W, 1);
#define O3DML_GEMM_SH_NT(P, W)                          \
    switch (gemm_nt()) {                                \
        case 0: O3DML_GEMM_SH_RB(P, 0, W) break;        \
        case 3: O3DML_GEMM_SH_RB(P, 3, W) break;        \
        default: O3DML_GEMM_SH_RB(P, 6, W) break;       \
    }
        if (nw == 4) {
            if (pre.scale) { O3DML_GEMM_SH_NT(true, 4) } else { O3DML_GEMM_SH_NT(false, 4) }
        } else if (nw == 1) {
            if (pre.scale) { O3DML_GEMM_SH_NT(true, 1) } else { O3DML_GEMM_SH_NT(false, 1) }
        } else {
            if (pre.scale) { O3DML_GEMM_SH_NT(true, 2) } else { O3DML_GEMM_SH_NT(false, 2) }
        }
#undef O3DML_GEMM_SH_RB
#undef O3DML_GEMM_SH_NT
#undef O3DML_GEMM_SH
#undef O3DML_GEMM_SH_SC
#undef O3DML_GEMM_SH_BUF
    } else if (vec4 && lds_path) {
#define O3DML_GEMM_LDS_GO(...)                                                                                   \
    do {                                                                                                         \
        GemmPrologue pp = pre;                                                                                   \
        const dim3 gg = persist_grid<__VA_ARGS__>(g, pp);                                                        \
        __VA_ARGS__<<<gg, kGemmThreads, 0, st>>>(map, order, order_flag, K, n_out, src, sscale, pscale, Wt, cin, \
                                                 cout, oscale, bias, out, ns, part, pp, residual, counters);     \
    } while (0)
#define O3DML_GEMM_LDS_SC(P, BR, X, SCL) O3DML_GEMM_LDS_GO(implicit_gemm_lds_kernel<P, BR, X, SCL>)
#define O3DML_GEMM_LDS(P, BR, X)                                      \
    do {                                                              \
        if (sscale || pscale) O3DML_GEMM_LDS_SC(P, BR, X, true);      \
        else if (BR && buf_ok) O3DML_GEMM_LDS_BUF(P, X);              \
        else O3DML_GEMM_LDS_SC(P, BR, X, false);                      \
    } while (0)
#define O3DML_GEMM_LDS_BUF2(P, X, D) O3DML_GEMM_LDS_GO(implicit_gemm_lds_kernel<P, true, X, false, true, D>)
#define O3DML_GEMM_LDS_BUF(P, X)                                 \
    do {                                                         \
        if (depth2) O3DML_GEMM_LDS_BUF2(P, X, 2);                \
        else O3DML_GEMM_LDS_BUF2(P, X, 1);                       \
    } while (0)
        static const bool depth2 = [] {
            const char* e = std::getenv("O3DML_GEMM_DEPTH");
            return e ? std::atoi(e) == 2 : false;
        }();
        const int nt = gemm_nt();
        const int64_t wn = static_cast<int64_t>(K) * cout * cin;
        // one 32-channel chunk per offset only: at cin 32 the split copy saves
        // 3 % (32->32, 32->16 layers), at cin 64 it cost 15 % (64->32;
        // gpurun_out/r4s28, same session)
        const bool bs = g_bsplit && nt == 6 && buf_ok && !depth2 && !sscale && !pscale && cin == 32 &&
                        static_cast<uint64_t>(wn) * 6u < kNoRow - 128 && ws.base &&
                        ws.used + bsplit_bytes(K, cin, cout) <= ws.size;
        if (bs) {
            bf16x8* w3 = reinterpret_cast<bf16x8*>(ws.take<uint16_t>(3 * wn));
            split_filters_kernel<<<stream_grid(wn / 8, 256), 256, 0, st>>>(Wt, wn / 8, w3);
            O3DML_LAUNCH_CHECK();
            pre.wsplit = reinterpret_cast<const __bf16*>(w3);
            pre.wsplit_bytes = static_cast<uint32_t>(wn * 6);
        }
#define O3DML_GEMM_LDS_BS(P) O3DML_GEMM_LDS_GO(implicit_gemm_lds_kernel<P, true, 6, false, true, 1, true>)
        if (nt == 6 && bs) {
            if (pre.scale) O3DML_GEMM_LDS_BS(true); else O3DML_GEMM_LDS_BS(false);
        } else if (nt == 6) {
            if (pre.scale) O3DML_GEMM_LDS(true, true, 6); else O3DML_GEMM_LDS(false, true, 6);
        } else if (nt == 3) {
            if (pre.scale) O3DML_GEMM_LDS(true, true, 3); else O3DML_GEMM_LDS(false, true, 3);
        } else if (pre.scale) {
            if (breg) O3DML_GEMM_LDS(true, true, 0); else O3DML_GEMM_LDS(true, false, 0);
        } else {
            if (breg) O3DML_GEMM_LDS(false, true, 0); else O3DML_GEMM_LDS(false, false, 0);
        }
#undef O3DML_GEMM_LDS
#undef O3DML_GEMM_LDS_SC
#undef O3DML_GEMM_LDS_BUF
#undef O3DML_GEMM_LDS_BUF2
#undef O3DML_GEMM_LDS_BS
#undef O3DML_GEMM_LDS_GO
    } else if (pre.scale) {
        if (vec4) O3DML_GEMM_LAUNCH(true, true); else O3DML_GEMM_LAUNCH(false, true);
    } else {
        if (vec4) O3DML_GEMM_LAUNCH(true, false); else O3DML_GEMM_LAUNCH(false, false);
    }
#undef O3DML_GEMM_LAUNCH
    O3DML_LAUNCH_CHECK();
    tr.end();
    if (ns > 1 && !counters) {
        split_reduce_kernel<<<stream_grid(n_out * cout, 256), 256, 0, st>>>(part, ns, n_out, cout, oscale, bias,
                                                                           residual, out);
        O3DML_LAUNCH_CHECK();
    }
}

// --------------------------------------------------------------------------
// lattice rulebook: when every input and query position sits exactly on one
// voxel lattice (SparseConvUnet: half-integer positions, vs = 1), the
// Linf-ball neighbours of a query are exactly the K lattice offsets, so the
// dense kernel map is built with a hash table of input voxel keys and K
// lookups per output — identical to the map the fixed-radius-search rulebook
// produces, without the search.
// --------------------------------------------------------------------------
constexpr uint64_t kLatEmpty = ~0ull;

__device__ __forceinline__ uint64_t lat_key(int x, int y, int z) {
    return (static_cast<uint64_t>(static_cast<uint32_t>(x + (1 << 20)) & 0x1fffffu) << 42) |
           (static_cast<uint64_t>(static_cast<uint32_t>(y + (1 << 20)) & 0x1fffffu) << 21) |
           static_cast<uint64_t>(static_cast<uint32_t>(z + (1 << 20)) & 0x1fffffu);
}

__device__ __forceinline__ uint32_t lat_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return static_cast<uint32_t>(k);
}

// per-axis [min frac, max frac, min key, max key] of p / vs (frac as float bits,
// keys as ints); blockIdx.y = point set (0 inputs, 1 queries); one partial per
// block -> part[(y * gridDim.x + x) * 12 + j], reduced by lattice_finalize_kernel
constexpr int kLatStatBlocks = 64;

__device__ __forceinline__ void lat_stat_init(int* v) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        v[4 * d + 0] = 0x7fffffff;
        v[4 * d + 1] = 0;
        v[4 * d + 2] = 0x7fffffff;
        v[4 * d + 3] = static_cast<int>(0x80000000u);
    }
}

__device__ __forceinline__ int lat_stat_merge(int j, int a, int b) { return (j & 1) ? max(a, b) : min(a, b); }

// Queries are qpos - qsh (the layer's offset * voxel size, subtracted here in
// f32 as the torch expression out_pos - offset * vs would: same bits, no
// elementwise launches); qsh = 0 for plain queries.
struct QueryShift {
    float d[3];
};

__global__ void __launch_bounds__(256) lattice_stats_kernel(const float* __restrict__ inp_pos, int64_t n_in,
                                                            const float* __restrict__ qpos, int64_t n_q,
                                                            QueryShift qsh, float inv_vs, int* __restrict__ part,
                                                            uint64_t* __restrict__ keys, int64_t cap,
                                                            int* __restrict__ status) {
    __shared__ int red[12][256];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 4) status[threadIdx.x] = 0;  // [2], [3]: no tile orders
    // the voxel hash's empty keys (lattice_insert_kernel runs next)
    for (int64_t e = (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
         e < cap; e += static_cast<int64_t>(gridDim.x) * gridDim.y * blockDim.x)
        keys[e] = kLatEmpty;
    const float* pos = blockIdx.y ? qpos : inp_pos;
    const int64_t n = blockIdx.y ? n_q : n_in;
    const QueryShift sh = blockIdx.y ? qsh : QueryShift{{0.f, 0.f, 0.f}};
    int v[12];
    lat_stat_init(v);
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float u = (pos[3 * i + d] - sh.d[d]) * inv_vs;
            const float fl = floorf(u);
            const float fr = u - fl;  // >= 0, so int ordering of the bits is float ordering
            const int key = fabsf(fl) < 1.0e6f ? static_cast<int>(fl) : 0x7fffffff;
            v[4 * d + 0] = min(v[4 * d + 0], __float_as_int(fr));
            v[4 * d + 1] = max(v[4 * d + 1], __float_as_int(fr));
            v[4 * d + 2] = min(v[4 * d + 2], key);
            v[4 * d + 3] = max(v[4 * d + 3], key);
        }
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) red[j][threadIdx.x] = v[j];
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if (threadIdx.x < w) {
#pragma unroll
            for (int j = 0; j < 12; ++j) red[j][threadIdx.x] = lat_stat_merge(j, red[j][threadIdx.x], red[j][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 12)
        part[(static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * 12 + threadIdx.x] = red[threadIdx.x][0];
}

struct LatticeOffsets {
    int off[3][8];  // key_p - key_q for kernel index j along axis d (x, y, z)
};

// Reduces the stats partials (nblk per set) and derives the per-axis lattice
// offsets: the lattice test is "every input shares one fraction per axis,
// every query shares one, keys within +-2^19, and exactly ksize lattice
// offsets j + (f_in - f_q) lie in [-ks/2, ks/2] with distinct kernel
// indices".  Run by the insert kernel's extra block (no separate finalize
// launch): threads 0-23 reduce, thread 0 derives the offsets into LDS.
// Returns ok (uniform over the block).
__device__ bool lattice_block_offsets(const int* __restrict__ part, int nblk, int ksize, int mirror,
                                      LatticeOffsets& lo_sh, int* st, int* ok_sh) {
    const int t = threadIdx.x;
    if (t < 24) {
        const int set = t / 12, j = t % 12;
        const int init = (j & 1) ? ((j & 2) ? static_cast<int>(0x80000000u) : 0) : 0x7fffffff;
        int v = init;
        for (int b0 = 0; b0 < nblk; b0 += 16) {  // 16 independent loads in flight
            int tmp[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) tmp[u] = b0 + u < nblk ? part[(set * nblk + b0 + u) * 12 + j] : init;
#pragma unroll
            for (int u = 0; u < 16; ++u) v = lat_stat_merge(j, v, tmp[u]);
        }
        st[t] = v;
    }
    __syncthreads();
    if (t == 0) {
        LatticeOffsets lo{};
        const double h = 0.5 * ksize;
        bool ok = true;
        for (int d = 0; d < 3 && ok; ++d) {
            const float fi_lo = __int_as_float(st[4 * d]), fi_hi = __int_as_float(st[4 * d + 1]);
            const float fq_lo = __int_as_float(st[12 + 4 * d]), fq_hi = __int_as_float(st[12 + 4 * d + 1]);
            const bool keys_ok = st[4 * d + 2] > -(1 << 19) && st[4 * d + 3] < (1 << 19) &&
                                 st[12 + 4 * d + 2] > -(1 << 19) && st[12 + 4 * d + 3] < (1 << 19);
            if (fi_lo != fi_hi || fq_lo != fq_hi || !keys_ok) {
                ok = false;
                break;
            }
            const double dc = static_cast<double>(fi_lo) - static_cast<double>(fq_lo);
            int n_within = 0;
            for (int j = -8; j <= 8; ++j) {
                const double dd = j + dc;
                if (dd < -h || dd > h) continue;
                const int kid = mirror ? static_cast<int>(floor(h - dd)) : static_cast<int>(floor(dd + h));
                if (kid < 0 || kid >= ksize || n_within >= ksize) {
                    ok = false;
                    break;
                }
                lo.off[d][kid] = j;
                ++n_within;
            }
            if (n_within != ksize) ok = false;
        }
        lo_sh = lo;
        *ok_sh = ok ? 1 : 0;
    }
    __syncthreads();
    return *ok_sh != 0;
}

// Hashes the input voxels (keys emptied by lattice_stats_kernel, which also
// zeroed the status words) and, in block 0 (one extra block: the serial part
// stays off the insert's critical path), derives the lattice offsets into lo
// and flags a non-lattice set (status 4); any block flags two inputs on one
// voxel (4 as well).  A non-lattice set inserts anyway: its map is discarded.
__global__ void __launch_bounds__(256) lattice_insert_kernel(const float* __restrict__ pos, int64_t n, float inv_vs,
                                                             uint64_t* __restrict__ keys, int32_t* __restrict__ vals,
                                                             uint32_t mask, const int* __restrict__ part, int nblk,
                                                             int ksize, int mirror, LatticeOffsets* __restrict__ lo,
                                                             int* __restrict__ status) {
    if (blockIdx.x == gridDim.x - 1) {
        __shared__ LatticeOffsets lo_sh;
        __shared__ int st_sh[24], ok_sh;
        const bool ok = lattice_block_offsets(part, nblk, ksize, mirror, lo_sh, st_sh, &ok_sh);
        if (threadIdx.x == 0) {
            *lo = lo_sh;
            if (!ok) atomicOr(status, 4);
        }
        return;
    }
    const int64_t inserters = gridDim.x - 1;  // the last block derived the offsets
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += inserters * blockDim.x) {
        const uint64_t k = lat_key(static_cast<int>(floorf(pos[3 * i] * inv_vs)),
                                   static_cast<int>(floorf(pos[3 * i + 1] * inv_vs)),
                                   static_cast<int>(floorf(pos[3 * i + 2] * inv_vs)));
        uint32_t h = lat_hash(k) & mask;
        while (true) {
            const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(&keys[h]),
                                                      static_cast<unsigned long long>(kLatEmpty),
                                                      static_cast<unsigned long long>(k));
            if (prev == kLatEmpty) {
                vals[h] = static_cast<int32_t>(i);
                break;
            }
            if (prev == k) {  // two inputs on one voxel: not a plain lattice set
                atomicOr(status, 4);
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

// map[o*K + k] for k = (kz*ks + ky)*ks + kx: one thread per (output, offset)
__global__ void __launch_bounds__(256) lattice_map_kernel(const float* __restrict__ inp_pos,
                                                          const float* __restrict__ qpos, QueryShift qsh,
                                                          int64_t n_out, float inv_vs,
                                                          float radius, int ks, const LatticeOffsets* __restrict__ lop,
                                                          const uint64_t* __restrict__ keys,
                                                          const int32_t* __restrict__ vals, uint32_t mask,
                                                          const int* __restrict__ status, int32_t* __restrict__ map) {
    const bool skip = (*status & 4) != 0;  // not a lattice set: an all-empty (safe) map
    const LatticeOffsets lo = skip ? LatticeOffsets{} : *lop;
    const int K = ks * ks * ks;
    const int64_t total = n_out * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        if (skip) {
            map[e] = -1;
            continue;
        }
        const int64_t o = e / K;
        const int k = static_cast<int>(e - o * K);
        const float qx = qpos[3 * o] - qsh.d[0], qy = qpos[3 * o + 1] - qsh.d[1], qz = qpos[3 * o + 2] - qsh.d[2];
        const int ix = k % ks, iy = (k / ks) % ks, iz = k / (ks * ks);
        const uint64_t key = lat_key(static_cast<int>(floorf(qx * inv_vs)) + lo.off[0][ix],
                                     static_cast<int>(floorf(qy * inv_vs)) + lo.off[1][iy],
                                     static_cast<int>(floorf(qz * inv_vs)) + lo.off[2][iz]);
        uint32_t h = lat_hash(key) & mask;
        int32_t found = -1;
        while (true) {
            const uint64_t kk = keys[h];
            if (kk == key) {
                found = vals[h];
                break;
            }
            if (kk == kLatEmpty) break;
            h = (h + 1) & mask;
        }
        if (found >= 0) {  // the fixed-radius (Linf) test the search would apply
            const float dx = fabsf(inp_pos[3 * found] - qx), dy = fabsf(inp_pos[3 * found + 1] - qy),
                        dz = fabsf(inp_pos[3 * found + 2] - qz);
            const float m = dx > dy ? dx : dy;
            if ((m > dz ? m : dz) > radius) found = -1;
        }
        map[e] = found;
    }
}

__global__ void map_count_kernel(const int32_t* __restrict__ map, int64_t n_out, int K, float* __restrict__ norm) {
    for (int64_t o = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; o < n_out;
         o += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        int c = 0;
        for (int k = 0; k < K; ++k) c += map[o * K + k] >= 0 ? 1 : 0;
        norm[o] = static_cast<float>(c);
    }
}

}  // namespace o3dml

using namespace o3dml;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
O3DML_API size_t o3dml_sparse_conv_map_workspace_size(int64_t n_out, int64_t n_in, int K) {
    return ws_bytes<int32_t>(n_out * K) + ws_bytes<float>(n_out * K) + ws_bytes<float>(n_out) +
           ws_bytes<float>(n_out) + ws_bytes<int32_t>(n_in * K) + ws_bytes<float>(n_in * K) + ws_bytes<int>(4) +
           ws_bytes<int32_t>(n_out) + ws_bytes<int32_t>(n_in) + ws_bytes<int32_t>(tile_map_entries(n_out, K)) +
           ws_bytes<int32_t>(tile_map_entries(n_in, K)) + order_scratch_bytes(std::max(n_out, n_in));
}

// Tile orders of the map and the inverse map (after the status words) and the
// scratch their sorts use.
struct MapOrders {
    int32_t* order;
    int32_t* iorder;
    int32_t* tmap;   // map rows in tile order
    int32_t* itmap;  // inverse map rows in tile order
    Workspace scratch;
};

static MapOrders map_orders(Workspace& ws, int64_t n_out, int64_t n_in, int K) {
    int32_t* order = ws.take<int32_t>(n_out);
    int32_t* iorder = ws.take<int32_t>(n_in);
    int32_t* tmap = ws.take<int32_t>(tile_map_entries(n_out, K));
    int32_t* itmap = ws.take<int32_t>(tile_map_entries(n_in, K));
    return MapOrders{order, iorder, tmap, itmap, Workspace(ws.base + ws.used, ws.size - ws.used)};
}

// Builds the dense kernel map (and, with want_inverse, the inverse map used by
// the input gradient) from CSR pairs.  Results live at the front of
// `workspace` (layout: map[n_out*K] i32, pscale[n_out*K] f32, norm[n_out],
// oscale[n_out], inv[n_in*K] i32, ipscale[n_in*K] f32, status[4]) and are
// consumed by o3dml_sparse_conv_forward / _backward with the same workspace.
// status_host[0]: bit0 = duplicate (o,k) pair, bit1 = kernel index out of
// range (the dense path cannot represent the neighbourhood).
O3DML_API int o3dml_sparse_conv_build_map(const int32_t* neighbors_index, const int32_t* neighbors_kernel_index,
                                          const float* neighbors_importance, const int64_t* neighbors_row_splits,
                                          int64_t n_out, int64_t n_in, int K, int normalize,
                                          const float* out_importance, int want_inverse, int* status_host,
                                          void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= 32, "sparse_conv: kernel volume must be in [1, 32] (got %d)", K);
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    int32_t* map = ws.take<int32_t>(n_out * K);
    float* pscale = ws.take<float>(n_out * K);
    float* norm = ws.take<float>(n_out);
    float* oscale = ws.take<float>(n_out);
    int32_t* inv = ws.take<int32_t>(n_in * K);
    float* ipscale = ws.take<float>(n_in * K);
    int* status = ws.take<int>(4);
    fill_async(status, 0, sizeof(int) * 4, st);  // [2], [3]: no tile orders yet
    if (n_out > 0) {
        fill_async(map, 0xff, sizeof(int32_t) * n_out * K, st);
        build_kernel_map_kernel<<<stream_grid(n_out, 256), 256, 0, st>>>(
                neighbors_index, neighbors_kernel_index, neighbors_importance, neighbors_row_splits, n_out, n_in, K,
                map, neighbors_importance ? pscale : nullptr, norm, status);
        O3DML_LAUNCH_CHECK();
        recip_norm_kernel<<<stream_grid(n_out, 256), 256, 0, st>>>(normalize ? norm : nullptr, out_importance, n_out,
                                                                  oscale);
        O3DML_LAUNCH_CHECK();
    }
    if (want_inverse && n_in > 0) {  // map entries are < n_in (out-of-range pairs were dropped, status 8)
        fill_async(inv, 0xff, sizeof(int32_t) * n_in * K, st);
        if (n_out > 0) {
            build_inverse_map_kernel<<<stream_grid(n_out * K, 256), 256, 0, st>>>(
                    map, neighbors_importance ? pscale : nullptr, n_out, K, n_in, inv,
                    neighbors_importance ? ipscale : nullptr, status);
            O3DML_LAUNCH_CHECK();
        }
    }
    O3DML_CHECK_HIP(hipMemcpyAsync(status_host, status, sizeof(int), hipMemcpyDeviceToHost, st));
    O3DML_CHECK_HIP(hipStreamSynchronize(st));
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_sparse_conv_lattice_workspace_size(int64_t n_in) {
    int64_t cap = 64;
    while (cap < 2 * n_in) cap <<= 1;
    return ws_bytes<uint64_t>(cap) + ws_bytes<int32_t>(cap) + ws_bytes<int>(2 * kLatStatBlocks * 12) +
           ws_bytes<LatticeOffsets>(1);
}

// Byte offset of the int32 status word inside a map workspace (deferred
// lattice checks read it later, batched, with one host round trip).
O3DML_API size_t o3dml_sparse_conv_map_status_offset(int64_t n_out, int64_t n_in, int K) {
    return ws_bytes<int32_t>(n_out * K) + ws_bytes<float>(n_out * K) + ws_bytes<float>(n_out) +
           ws_bytes<float>(n_out) + ws_bytes<int32_t>(n_in * K) + ws_bytes<float>(n_in * K);
}

// Dense kernel map (same workspace layout as o3dml_sparse_conv_build_map) for
// a cubic ks^3 SparseConv / SparseConvTranspose whose queries are `query_pos`
// (= out_pos -/+ offset * vs) and whose neighbourhood is the Linf ball of
// radius ks*vs/2, built directly when all positions lie on one voxel lattice.
// status_host[0]: 4 = not a lattice set (caller uses the search rulebook).
O3DML_API int o3dml_sparse_conv_lattice_map(const float* inp_pos, int64_t n_in, const float* query_pos, int64_t n_out,
                                            float voxel_size, int ksize, int mirror, int normalize,
                                            const float* out_importance, int want_inverse, int defer_status,
                                            int* status_host, void* workspace, size_t workspace_bytes,
                                            void* lattice_workspace, size_t lattice_workspace_bytes, void* stream) {
    return o3dml_sparse_conv_lattice_map_shifted(inp_pos, n_in, query_pos, nullptr, n_out, voxel_size, ksize, mirror,
                                                 normalize, out_importance, want_inverse, defer_status, status_host,
                                                 workspace, workspace_bytes, lattice_workspace,
                                                 lattice_workspace_bytes, stream);
}

// The same with the queries given as query_pos - query_shift (host float[3],
// or null for none): the layer's out_pos - offset * voxel_size without
// materialising it.
O3DML_API int o3dml_sparse_conv_lattice_map_shifted(const float* inp_pos, int64_t n_in, const float* query_pos,
                                                    const float* query_shift, int64_t n_out, float voxel_size,
                                                    int ksize, int mirror, int normalize, const float* out_importance,
                                                    int want_inverse, int defer_status, int* status_host,
                                                    void* workspace, size_t workspace_bytes, void* lattice_workspace,
                                                    size_t lattice_workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    const QueryShift qsh = query_shift ? QueryShift{{query_shift[0], query_shift[1], query_shift[2]}}
                                       : QueryShift{{0.f, 0.f, 0.f}};
    O3DML_REQUIRE(ksize >= 1 && ksize <= 3, "lattice rulebook: kernel size must be 1..3");
    const int K = ksize * ksize * ksize;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    int32_t* map = ws.take<int32_t>(n_out * K);
    float* pscale = ws.take<float>(n_out * K);
    float* norm = ws.take<float>(n_out);
    float* oscale = ws.take<float>(n_out);
    int32_t* inv = ws.take<int32_t>(n_in * K);
    float* ipscale = ws.take<float>(n_in * K);
    int* status = ws.take<int>(4);
    (void)pscale;
    (void)ipscale;
    *status_host = 0;
    if (n_in == 0 || n_out == 0) {
        *status_host = 4;
        return 0;
    }
    Workspace lws(lattice_workspace, lattice_workspace_bytes);
    int64_t cap = 64;
    while (cap < 2 * n_in) cap <<= 1;
    uint64_t* keys = lws.take<uint64_t>(cap);
    int32_t* vals = lws.take<int32_t>(cap);
    int* part = lws.take<int>(2 * kLatStatBlocks * 12);
    LatticeOffsets* lo = lws.take<LatticeOffsets>(1);
    const float inv_vs = 1.0f / voxel_size;
    // ---- 1. lattice statistics (per-block partials; the offsets are derived
    // from them by every block of the next two kernels: no host round trip,
    // no finalize launch), 2. hash the input voxels, 3. K lookups per output
    const int nblk = static_cast<int>(std::min<int64_t>(kLatStatBlocks, ceil_div(std::max(n_in, n_out), 256)));
    lattice_stats_kernel<<<dim3(nblk, 2), 256, 0, st>>>(inp_pos, n_in, query_pos, n_out, qsh, inv_vs, part, keys,
                                                         cap, status);
    O3DML_LAUNCH_CHECK();
    lattice_insert_kernel<<<stream_grid(n_in, 256) + 1, 256, 0, st>>>(inp_pos, n_in, inv_vs, keys, vals,
                                                                     static_cast<uint32_t>(cap - 1), part, nblk, ksize,
                                                                     mirror, lo, status);
    O3DML_LAUNCH_CHECK();
    lattice_map_kernel<<<stream_grid(n_out * K, 256), 256, 0, st>>>(
            inp_pos, query_pos, qsh, n_out, inv_vs, 0.5f * voxel_size * static_cast<float>(ksize), ksize, lo, keys, vals,
            static_cast<uint32_t>(cap - 1), status, map);
    O3DML_LAUNCH_CHECK();
    if (normalize) {
        map_count_kernel<<<stream_grid(n_out, 256), 256, 0, st>>>(map, n_out, K, norm);
        O3DML_LAUNCH_CHECK();
    }
    if (normalize || out_importance) {
        recip_norm_kernel<<<stream_grid(n_out, 256), 256, 0, st>>>(normalize ? norm : nullptr, out_importance, n_out,
                                                                  oscale);
        O3DML_LAUNCH_CHECK();
    }
    if (want_inverse) {
        fill_async(inv, 0xff, sizeof(int32_t) * n_in * K, st);
        build_inverse_map_kernel<<<stream_grid(n_out * K, 256), 256, 0, st>>>(map, nullptr, n_out, K, n_in, inv,
                                                                            nullptr, status);
        O3DML_LAUNCH_CHECK();
    }
    if (defer_status) return 0;  // status stays on the device (o3dml_sparse_conv_map_status_offset)
    O3DML_CHECK_HIP(hipMemcpyAsync(status_host, status, sizeof(int), hipMemcpyDeviceToHost, st));
    O3DML_CHECK_HIP(hipStreamSynchronize(st));
    O3DML_GUARD_END
}

__global__ void transpose_prep_kernel(int32_t* __restrict__ map, int64_t n, int* __restrict__ status,
                                      const int* __restrict__ cstatus) {
    if (blockIdx.x == 0 && threadIdx.x < 4) status[threadIdx.x] = threadIdx.x == 0 ? cstatus[0] : 0;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < n;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x)
        map[e] = -1;
}

O3DML_API int o3dml_sparse_conv_transpose_map(const void* conv_workspace, size_t conv_workspace_bytes,
                                              int64_t n_coarse, int64_t n_fine, int K, int want_inverse,
                                              void* out_workspace, size_t out_workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= 32, "sparse_conv: kernel volume must be in [1, 32] (got %d)", K);
    {
        const hipError_t pending = hipPeekAtLastError();
        O3DML_REQUIRE(pending == hipSuccess, "sparse_conv_transpose_map: HIP error pending on entry: %s",
                      hipGetErrorString(pending));
    }
    hipStream_t st = as_stream(stream);
    Workspace cw(const_cast<void*>(conv_workspace), conv_workspace_bytes);  // n_out = n_coarse, n_in = n_fine
    const int32_t* cmap = cw.take<int32_t>(n_coarse * K);
    cw.take<float>(n_coarse * K);
    cw.take<float>(n_coarse);
    cw.take<float>(n_coarse);
    cw.take<int32_t>(n_fine * K);
    cw.take<float>(n_fine * K);
    const int* cstatus = cw.take<int>(4);
    Workspace ws(out_workspace, out_workspace_bytes);  // n_out = n_fine, n_in = n_coarse
    int32_t* map = ws.take<int32_t>(n_fine * K);
    ws.take<float>(n_fine * K);
    ws.take<float>(n_fine);
    ws.take<float>(n_fine);
    int32_t* inv = ws.take<int32_t>(n_coarse * K);
    ws.take<float>(n_coarse * K);
    int* status = ws.take<int>(4);
    // the partner's lattice / duplicate status, [2], [3]: no tile orders yet,
    // and the empty map: one launch
    transpose_prep_kernel<<<stream_grid(std::max<int64_t>(n_fine * K, 1), 256), 256, 0, st>>>(map, n_fine * K, status,
                                                                                             cstatus);
    O3DML_LAUNCH_CHECK();
    if (n_coarse > 0 && n_fine > 0) {
        build_inverse_map_kernel<<<stream_grid(n_coarse * K, 256), 256, 0, st>>>(cmap, nullptr, n_coarse, K, n_fine, map,
                                                                                nullptr, status);
        O3DML_LAUNCH_CHECK();
    }
    if (want_inverse && n_coarse > 0) copy_async(inv, cmap, sizeof(int32_t) * n_coarse * K, st);
    O3DML_GUARD_END
}

// Wt [K][cout][cin] at the front of a forward workspace; the rest -> split
static float* forward_filters(const float* filters, int K, int cin, int cout, Workspace& ws, hipStream_t st) {
    float* wt = ws.take<float>(static_cast<int64_t>(K) * cin * cout);
    transpose_filters_kernel<<<stream_grid(static_cast<int64_t>(K) * cin * cout, 256), 256, 0, st>>>(filters, K, cin,
                                                                                                  cout, wt);
    O3DML_LAUNCH_CHECK();
    return wt;
}

static void map_views(void* workspace, size_t bytes, int64_t n_out, int64_t n_in, int K, int32_t** map,
                      float** pscale, float** oscale, int32_t** inv, float** ipscale, const int32_t** order,
                      const int32_t** iorder, const int** order_flag, const int** iorder_flag,
                      const int32_t** tmap = nullptr, const int32_t** itmap = nullptr) {
    Workspace ws(workspace, bytes);
    *map = ws.take<int32_t>(n_out * K);
    *pscale = ws.take<float>(n_out * K);
    ws.take<float>(n_out);
    *oscale = ws.take<float>(n_out);
    *inv = ws.take<int32_t>(n_in * K);
    *ipscale = ws.take<float>(n_in * K);
    int* status = ws.take<int>(4);
    const MapOrders ord = map_orders(ws, n_out, n_in, K);
    // device flags status[2] / status[3] say whether the orders were built
    *order = use_order(n_out, K) ? ord.order : nullptr;
    *iorder = use_order(n_in, K) ? ord.iorder : nullptr;
    if (tmap) *tmap = ord.tmap;
    if (itmap) *itmap = ord.itmap;
    *order_flag = status + 2;
    *iorder_flag = status + 3;
}

// Tile orders for a built map (and its inverse with `inverse` = 1): worth it
// when the map serves several GEMMs or wide channels (host decides).
O3DML_API int o3dml_sparse_conv_tile_order(void* map_workspace, size_t map_workspace_bytes, int64_t n_out,
                                           int64_t n_in, int K, int inverse, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(map_workspace, map_workspace_bytes);
    const int32_t* map = ws.take<int32_t>(n_out * K);
    ws.take<float>(n_out * K);
    ws.take<float>(n_out);
    ws.take<float>(n_out);
    const int32_t* inv = ws.take<int32_t>(n_in * K);
    ws.take<float>(n_in * K);
    int* status = ws.take<int>(4);
    MapOrders ord = map_orders(ws, n_out, n_in, K);
    build_order(map, n_out, K, ord.order, ord.tmap, status + 2, ord.scratch, st);
    if (inverse) build_order(inv, n_in, K, ord.iorder, ord.itmap, status + 3, ord.scratch, st);
    O3DML_GUARD_END
}

// Forward with an input prologue and a residual epilogue (SparseConvUnet eval:
// out = conv(relu(x * pre_scale + pre_shift)) + residual); pre_scale /
// pre_shift [cin] and residual [n_out, cout] are each nullable.  The filters
// come TRANSPOSED, filters_t [K][cout][cin] (eval weights are constant: the
// host keeps the transposed copy instead of a transpose launch per call).
O3DML_API int o3dml_sparse_conv_forward_fused(const float* filters_t, int K, int cin, int cout,
                                              const float* inp_features, int64_t n_in, const float* pre_scale,
                                              const float* pre_shift, const float* residual, const float* bias,
                                              int64_t n_out, float* out_features, void* map_workspace,
                                              size_t map_workspace_bytes, void* workspace, size_t workspace_bytes,
                                              void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE((pre_scale == nullptr) == (pre_shift == nullptr), "pre_scale and pre_shift go together");
    int32_t *map, *inv;
    float *pscale, *oscale, *ipscale;
    const int32_t *order, *iorder, *tmap;
    const int *oflag, *ioflag;
    map_views(map_workspace, map_workspace_bytes, n_out, n_in, K, &map, &pscale, &oscale, &inv, &ipscale, &order,
              &iorder, &oflag, &ioflag, &tmap);
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    ws.take<float>(static_cast<int64_t>(K) * cin * cout);  // (unused Wt slot: filters_t comes transposed)
    run_gemm(st, map, order, oflag, K, n_out, inp_features, n_in, nullptr, nullptr, filters_t, cin, cout, nullptr,
             bias, out_features, ws, GemmPrologue{pre_scale, pre_shift}, residual, tmap);
    O3DML_GUARD_END
}

// transposed filters, split-K partial sums and the presplit operand planes of
// o3dml_sparse_conv_forward(_fused)
O3DML_API size_t o3dml_sparse_conv_forward_workspace_size(int64_t n_out, int64_t n_in, int K, int cin, int cout) {
    return ws_bytes<float>(static_cast<int64_t>(K) * cin * cout) + gemm_ws_bytes(n_out, n_in, K, cin, cout);
}

// out [n_out, cout] = oscale * sum_k gather(inp) @ W[k] (+ bias).  filters:
// [K][cin][cout].  inp_importance (nullable) scales input rows; pair
// importance / normalisation / out_importance come from the map workspace.
O3DML_API int o3dml_sparse_conv_forward(const float* filters, int K, int cin, int cout, const float* inp_features,
                                        int64_t n_in, const float* inp_importance, int has_neighbors_importance,
                                        int use_out_scale, const float* bias, int64_t n_out, float* out_features,
                                        void* map_workspace, size_t map_workspace_bytes, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    int32_t *map, *inv;
    float *pscale, *oscale, *ipscale;
    const int32_t *order, *iorder, *tmap;
    const int *oflag, *ioflag;
    map_views(map_workspace, map_workspace_bytes, n_out, n_in, K, &map, &pscale, &oscale, &inv, &ipscale, &order,
              &iorder, &oflag, &ioflag, &tmap);
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const float* wt = forward_filters(filters, K, cin, cout, ws, st);
    run_gemm(st, map, order, oflag, K, n_out, inp_features, n_in, inp_importance,
             has_neighbors_importance ? pscale : nullptr, wt, cin, cout, use_out_scale ? oscale : nullptr, bias,
             out_features, ws, GemmPrologue{nullptr, nullptr}, nullptr, tmap);
    O3DML_GUARD_END
}

// dW pair-list chunks per offset: enough waves to fill the chip (~4 per
// SIMD), but at least ~256 pairs per chunk (each chunk writes a cin x cout slab).
static int dw_chunks(int64_t n_out, int K, int cin, int cout) {
    const int64_t tiles = ceil_div(cin, 32) * ceil_div(cout, 32) * static_cast<int64_t>(K);
    int64_t nc = ceil_div(int64_t(4096), tiles);
    nc = std::min<int64_t>(nc, std::max<int64_t>(1, n_out / 256));
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(nc, 64)));
}

O3DML_API size_t o3dml_sparse_conv_backward_workspace_size(int64_t n_out, int64_t n_in, int K, int cin, int cout) {
    const int nchunk = dw_chunks(n_out, K, cin, cout);
    return ws_bytes<float>(static_cast<int64_t>(K) * cin * cout) + ws_bytes<float>(n_out * cout) +
           gemm_ws_bytes(n_in, n_out, K, cout, cin) + ws_bytes<int64_t>(n_out * K) * 2 + ws_bytes<int32_t>(n_out * K) +
           ws_bytes<int64_t>(K + 1) + ws_bytes<int64_t>(K + 2) +
           (nchunk > 1 ? ws_bytes<float>(static_cast<int64_t>(K) * (nchunk + 1) * cin * cout) : 0) +
           prim::scan_workspace_bytes(n_out * K);
}

// grad_out [n_out, cout] -> grad_inp [n_in, cin] (nullable) and grad_filters
// [K][cin][cout] (nullable).  Uses the inverse map (build_map with
// want_inverse = 1) for grad_inp.
O3DML_API int o3dml_sparse_conv_backward(const float* filters, int K, int cin, int cout, const float* inp_features,
                                         int64_t n_in, const float* inp_importance, int has_neighbors_importance,
                                         int use_out_scale, const float* grad_out, int64_t n_out, float* grad_inp,
                                         float* grad_filters, void* map_workspace, size_t map_workspace_bytes,
                                         void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    int32_t *map, *inv;
    float *pscale, *oscale, *ipscale;
    const int32_t *order, *iorder, *itmap;
    const int *oflag, *ioflag;
    map_views(map_workspace, map_workspace_bytes, n_out, n_in, K, &map, &pscale, &oscale, &inv, &ipscale, &order,
              &iorder, &oflag, &ioflag, nullptr, &itmap);
    Workspace ws(workspace, workspace_bytes);
    float* wt = ws.take<float>(static_cast<int64_t>(K) * cin * cout);
    float* g = ws.take<float>(n_out * cout);  // unused slot kept for layout stability
    (void)g;
    // the dIn GEMM's scratch (split-K partials, presplit planes)
    const size_t gemm_bytes = gemm_ws_bytes(n_in, n_out, K, cout, cin);
    Workspace gws(ws.base + ws.used, std::min(gemm_bytes, ws.size - ws.used));
    if (gemm_bytes) ws.take<uint8_t>(static_cast<int64_t>(gemm_bytes));
    const float* os = use_out_scale ? oscale : nullptr;
    if (grad_inp && n_in > 0) {
        // dIn[i] = sscale[i] * sum_k (g[inv[i,k]] * oscale[o] * pscale) @ W[k]^T: a
        // GEMM with weights W[k]^T [cout][cin], whose transposed form (what
        // the kernel reads) is W itself.
        // The per-row out-scale belongs to the gathered rows (source = grad_out):
        // fold it in as sscale; pair importance via the inverse pscale.
        (void)wt;
        run_gemm(st, inv, iorder, ioflag, K, n_in, grad_out, n_out, os, has_neighbors_importance ? ipscale : nullptr,
                 filters, cout, cin, inp_importance, nullptr, grad_inp, gws, GemmPrologue{nullptr, nullptr}, nullptr,
                 itmap);
    }
    if (grad_filters) {
        const int64_t KC = static_cast<int64_t>(K) * cin * cout;
        if (n_out == 0) {
            fill_async(grad_filters, 0, sizeof(float) * KC, st);
            return 0;
        }
        int64_t* flags = ws.take<int64_t>(n_out * K);
        int64_t* incl = ws.take<int64_t>(n_out * K);
        int32_t* po = ws.take<int32_t>(n_out * K);
        int64_t* kstart = ws.take<int64_t>(K + 1);
        int64_t* plan = ws.take<int64_t>(K + 2);
        const int nchunk = dw_chunks(n_out, K, cin, cout);
        const int64_t max_chunks = nchunk > 1 ? static_cast<int64_t>(K) * (nchunk + 1) : K;
        float* part = nchunk > 1 ? ws.take<float>(max_chunks * cin * cout) : grad_filters;
        pair_flags_kernel<<<stream_grid(n_out * K, 256), 256, 0, st>>>(map, n_out, K, flags);
        O3DML_LAUNCH_CHECK();
        Workspace sws = ws;
        prim::scan<int64_t, int64_t>(flags, incl, n_out * K, true, sws, st);
        pair_lists_kernel<<<stream_grid(n_out * K, 256), 256, 0, st>>>(map, n_out, K, incl, po, kstart);
        O3DML_LAUNCH_CHECK();
        dw_plan_kernel<<<1, 64, 0, st>>>(kstart, K, max_chunks, nchunk > 1 ? 0 : 1, plan);
        O3DML_LAUNCH_CHECK();
        dim3 gg(static_cast<unsigned>(ceil_div(cin, 32) * ceil_div(cout, 32)), static_cast<unsigned>(max_chunks));
#define O3DML_DW(NT)                                                                                      \
    dweight_kernel<NT><<<gg, 64, 0, st>>>(map, po, kstart, K, plan, inp_features, inp_importance,          \
                                          has_neighbors_importance ? pscale : nullptr, grad_out, os, cin, \
                                          cout, part)
#define O3DML_DWL(NT)                                                                                     \
    dweight_lds_kernel<NT><<<gg, 64, 0, st>>>(map, po, kstart, K, plan, inp_features, inp_importance,      \
                                              has_neighbors_importance ? pscale : nullptr, grad_out, os, cin, \
                                              cout, part)
        static const bool dw_lds = [] {
            const char* e = std::getenv("O3DML_DW_LDS");
            return e ? std::atoi(e) != 0 : true;
        }();
        const bool lds_ok = dw_lds && cin % 4 == 0 && cout % 4 == 0 &&
                            reinterpret_cast<uintptr_t>(inp_features) % 16 == 0 &&
                            reinterpret_cast<uintptr_t>(grad_out) % 16 == 0;
        if (lds_ok) {
            switch (gemm_nt()) {
                case 0: O3DML_DWL(0); break;
                case 3: O3DML_DWL(3); break;
                default: O3DML_DWL(6); break;
            }
        } else {
            switch (gemm_nt()) {
                case 0: O3DML_DW(0); break;
                case 3: O3DML_DW(3); break;
                default: O3DML_DW(6); break;
            }
        }
#undef O3DML_DWL
#undef O3DML_DW
        O3DML_LAUNCH_CHECK();
        if (nchunk > 1) {
            reduce_slabs_kernel<<<stream_grid(KC, 256), 256, 0, st>>>(part, K, plan,
                                                                      static_cast<int64_t>(cin) * cout, grad_filters);
            O3DML_LAUNCH_CHECK();
        }
    }
    O3DML_GUARD_END
}

// ksize_host[3] = filter dims (k0,k1,k2) = (z,y,x) extents.
// presplit operands on (1, default) / off (0); < 0 queries.  Returns the previous setting.
O3DML_API int o3dml_sparse_conv_set_bsplit(int on) {
    const int prev = g_bsplit ? 1 : 0;
    if (on >= 0) g_bsplit = on != 0;
    return prev;
}

O3DML_API int o3dml_sparse_conv_set_presplit(int on) {
    const int prev = g_presplit ? 1 : 0;
    if (on >= 0) g_presplit = on != 0;
    return prev;
}

O3DML_API int o3dml_sparse_conv_set_exact(int exact) {
    const int prev = gemm_mode();
    if (exact >= 0) {
        if (exact > 2) return -1;
        g_gemm_mode = exact;
    }
    return prev;
}

O3DML_API int o3dml_sparse_conv_kernel_index(const float* inp_positions, const float* query_positions,
                                             const int32_t* neighbors_index, const int64_t* neighbors_row_splits,
                                             int64_t n_query, const int32_t* ksize_host, float voxel_size,
                                             int mirror, int32_t* kernel_index, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(voxel_size > 0.f, "voxel_size must be > 0");
    if (n_query == 0) return 0;
    const float inv = 1.0f / voxel_size;
    kernel_index_kernel<<<stream_grid(n_query, 256), 256, 0, as_stream(stream)>>>(
            inp_positions, query_positions, neighbors_index, neighbors_row_splits, n_query, ksize_host[0],
            ksize_host[1], ksize_host[2], inv, mirror, kernel_index);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
