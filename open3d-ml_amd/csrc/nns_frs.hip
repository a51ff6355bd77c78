// nns_frs.hip — fixed-radius neighbour search (Open3D ops.fixed_radius_search /
// layers.FixedRadiusSearch; reference callers kpconv.py:2016-2034 batch_neighbors
// <- dataloaders/concat_batcher.py:228,257,261, and layers.SparseConv's Linf
// search sparseconvnet.py:362-367).
//
// Output: per query every point of its batch item with dist <= r (L2 squared /
// L1 / Linf) among the points of the hash buckets Open3D visits (the bucket of
// the query's own 2r-cell and of the cells of the 8 corners q +- r), in the
// canonical order of oracle/o3d_oracle.c: buckets ascending, point ids
// ascending inside a bucket — i.e. ascending position in hash_table_index.
//
// Query groups over Open3D's own buckets.  Two queries whose 9 visited
// buckets are identical visit exactly the same points in the same order.  A
// wave takes 64 consecutive queries in (batch, Morton r-cell) order, splits
// them into such groups (typically the queries of one octant of a 2r-cell)
// and, per group:
//   1. streams the group's buckets in ascending order — Open3D's visit order —
//      with coalesced 16-B loads, keeping only points within the metric's
//      distance of the group's bounding box (the box test uses the same fp32
//      operations as the exact test on smaller operands, so it never drops a
//      neighbour), compacted IN ORDER into an LDS list;
//   2. tests the list against the group's queries with S = 64 / G lanes per
//      query (G = group size rounded up to a power of two): lane (g, s) tests
//      entries s, s + S, ... of query g; a ballot + mbcnt ranks every hit, so
//      rows come out in canonical order with no sort.
// The first kRowCap neighbours of a query go to its temp row (indexed by
// query id), the count to counts[qid]; the fill phase copies the temp rows
// into the final CSR and re-runs the rare longer rows straight into place.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "primitives.hpp"
#include "spatial_hash.hpp"

namespace o3dml {

// out[j] = (points[index[j]], index[j]) — the points in Open3D bucket order, so
// one bucket is one contiguous 16-B-per-point stream.  XCD-contiguous: the
// workgroups of one XCD gather one contiguous range (one or two batch items at
// a time), so the random reads inside a batch item stay in that XCD's L2.
__global__ void __launch_bounds__(256) gather_sorted_points_kernel(const float* __restrict__ points,
                                                                   const uint32_t* __restrict__ index, int64_t n,
                                                                   float4* __restrict__ out, int sentinel,
                                                                   int64_t* __restrict__ zero_a, int n_zero_a,
                                                                   int64_t* __restrict__ zero_b) {
    const int64_t per = ceil_div(n, static_cast<int64_t>(gridDim.x));
    const int64_t blk = xcd_block();
    const int64_t e = min(n, (blk + 1) * per);
    constexpr int U = 4;  // four independent index -> point chains in flight per thread
    for (int64_t j0 = blk * per + threadIdx.x; j0 < e; j0 += U * static_cast<int64_t>(blockDim.x)) {
        uint32_t id[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * static_cast<int64_t>(blockDim.x);
            id[u] = j < e ? index[j] : 0u;
        }
        float x[U], y[U], z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u] = points[3 * static_cast<int64_t>(id[u])];
            y[u] = points[3 * static_cast<int64_t>(id[u]) + 1];
            z[u] = points[3 * static_cast<int64_t>(id[u]) + 2];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * static_cast<int64_t>(blockDim.x);
            if (j < e) out[j] = make_float4(x[u], y[u], z[u], __uint_as_float(id[u]));
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (sentinel) {  // out[n]: beyond every radius
            const float inf = __builtin_huge_valf();
            out[n] = make_float4(inf, inf, inf, 0.f);
        }
        // zeroed words of the caller (instead of memset launches)
        for (int j = 0; j < n_zero_a; ++j) zero_a[j] = 0;
        if (zero_b) *zero_b = 0;
    }
}

#ifndef O3DML_FRS_ROWCAP
#define O3DML_FRS_ROWCAP 64
#endif
constexpr int kRowCap = O3DML_FRS_ROWCAP;  // neighbours kept per query in the temp rows (<= 64)
static_assert(kRowCap >= 1 && kRowCap <= 64, "the row copy takes one row per wave instruction");
// voxel-class directory per bucket (bucket_classes_kernel): sizes of classes
// 0 and 1, 2 spare words, then per class 0-2 the box min x, y, z, max x, y, z
constexpr int kDirWords = 24;

// Lane split of a group of ng queries: S = floor(64 / ng) in bits 0-7 and
// M = ceil(65536 / S) in bits 8-31 (g = lane * M >> 16 = floor(lane / S)).
struct LaneSplitTab {
    uint32_t v[65];
    constexpr LaneSplitTab() : v() {
        for (int ng = 0; ng <= 64; ++ng) {
            const uint32_t S = ng == 0 ? 64u : 64u / static_cast<uint32_t>(ng);
            v[ng] = S | (((65536u + S - 1u) / S) << 8);
        }
    }
};
__constant__ constexpr LaneSplitTab kLaneSplitTab{};
#define kLaneSplit kLaneSplitTab.v

#ifndef O3DML_DIAG
#define O3DML_DIAG 0  // 1: skip the candidate test loop, 2: also skip streaming (cost-split diagnostics)
#endif
#ifndef O3DML_STREAM_U
#define O3DML_STREAM_U 2
#endif
#ifndef O3DML_FRS_DMA
#define O3DML_FRS_DMA 0  // stream rounds by LDS DMA into the candidate list (A/B switch)
#endif
typedef __attribute__((address_space(3))) void* frs_lds_ptr;
#ifndef O3DML_FRS_OOBST
#define O3DML_FRS_OOBST 0  // branch-free temp-row stores (A/B switch)
#endif
constexpr int kStreamU = O3DML_STREAM_U;  // 64-point loads in flight per lane while streaming buckets
// LDS candidate list per wave (float4), incl. the padding of the last slice:
// 4 KiB + 1 KiB of query slots keeps 32 waves per CU (LDS no tighter than the
// 64-VGPR limit of 8 waves per SIMD)
constexpr int kCandCap = 256;

// Wave-wide float min / max: DPP within rows of 16 lanes, then the 4 row
// results through v_readlane (uniform result, no LDS round trip).
// O3DML_FRS_DPPMIN (default): each step is ONE v_min_f32_dpp / v_max_f32_dpp
// (the DPP source folded into the VOP2 min/max); fminf through a
// v_mov_b32_dpp costs that mov plus two canonicalising v_max_f32 (fminf's
// signalling-NaN rule) per step — 5 instructions instead of 1.  The s_nop
// covers the VALU-write -> DPP-read hazard inside the asm block.
#ifndef O3DML_FRS_DPPMIN
#define O3DML_FRS_DPPMIN 1
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
#define O3DML_DPP_STEP(NAME, OP, CTRL)                                                                   \
    __device__ __forceinline__ float NAME(float v) {                                                    \
        float r;                                                                                        \
        asm volatile("s_nop 1\n\t" OP "_dpp %0, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf"            \
                     : "=v"(r)                                                                          \
                     : "v"(v));                                                                         \
        return r;                                                                                       \
    }
O3DML_DPP_STEP(dmin_q1, "v_min_f32", "quad_perm:[1,0,3,2]")
O3DML_DPP_STEP(dmin_q2, "v_min_f32", "quad_perm:[2,3,0,1]")
O3DML_DPP_STEP(dmin_hm, "v_min_f32", "row_half_mirror")
O3DML_DPP_STEP(dmin_rm, "v_min_f32", "row_mirror")
O3DML_DPP_STEP(dmax_q1, "v_max_f32", "quad_perm:[1,0,3,2]")
O3DML_DPP_STEP(dmax_q2, "v_max_f32", "quad_perm:[2,3,0,1]")
O3DML_DPP_STEP(dmax_hm, "v_max_f32", "row_half_mirror")
O3DML_DPP_STEP(dmax_rm, "v_max_f32", "row_mirror")
#undef O3DML_DPP_STEP
// min (MAX: max) over each row of 16 lanes, in every lane of the row
template <bool MAX>
__device__ __forceinline__ float row_ext_f(float v) {
#if O3DML_FRS_DPPMIN
    if constexpr (MAX) return dmax_rm(dmax_hm(dmax_q2(dmax_q1(v))));
    return dmin_rm(dmin_hm(dmin_q2(dmin_q1(v))));
#else
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
    v = op(v, dpp_f<0xB1>(v));   // quad_perm(1,0,3,2)
    v = op(v, dpp_f<0x4E>(v));   // quad_perm(2,3,0,1)
    v = op(v, dpp_f<0x141>(v));  // row_half_mirror
    v = op(v, dpp_f<0x140>(v));  // row_mirror
    return v;
#endif
}
__device__ __forceinline__ float rdlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_min_f(float v) {
    v = row_ext_f<false>(v);
    return fminf(fminf(rdlane_f(v, 0), rdlane_f(v, 16)), fminf(rdlane_f(v, 32), rdlane_f(v, 48)));
}
__device__ __forceinline__ float wave_max_f(float v) {
    v = row_ext_f<true>(v);
    return fmaxf(fmaxf(rdlane_f(v, 0), rdlane_f(v, 16)), fmaxf(rdlane_f(v, 32), rdlane_f(v, 48)));
}
// min / max over lanes 0-15 (DPP within row 0), read from lane 0
__device__ __forceinline__ float row0_min_f(float v) { return rdlane_f(row_ext_f<false>(v), 0); }
__device__ __forceinline__ float row0_max_f(float v) { return rdlane_f(row_ext_f<true>(v), 0); }

// Distance of p to the box [lo, hi] with the metric's own operation order;
// every operand is <= the corresponding one of dist_metric(p, q) for any q in
// the box, and each step is monotone, so box_dist <= dist_metric(p, q).
template <int METRIC>
__device__ __forceinline__ float box_dist(const float4& p, float lx, float ly, float lz, float hx, float hy,
                                          float hz) {
    // signed gap to the box: p minus p clamped into [lo, hi] (one v_med3 each)
    const float gx = p.x - __builtin_amdgcn_fmed3f(p.x, lx, hx);
    const float gy = p.y - __builtin_amdgcn_fmed3f(p.y, ly, hy);
    const float gz = p.z - __builtin_amdgcn_fmed3f(p.z, lz, hz);
    if constexpr (METRIC == kL2) {
        return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
    } else if constexpr (METRIC == kL1) {
        return (fabsf(gx) + fabsf(gy)) + fabsf(gz);
    } else {
        const float ax = fabsf(gx), ay = fabsf(gy), az = fabsf(gz);
        const float m = ax > ay ? ax : ay;
        return m > az ? m : az;
    }
}

// Distance bound between two boxes, [al, ah] and [bl, bh], with the metric's
// operation order: each gap is <= the |difference| of any two points of the
// boxes and every step is monotone, so the bound is <= dist_metric(p, q) for
// every p in one box and q in the other.
template <int METRIC>
__device__ __forceinline__ float box_box_dist(float alx, float aly, float alz, float ahx, float ahy, float ahz,
                                              float blx, float bly, float blz, float bhx, float bhy, float bhz) {
    const float gx = fmaxf(fmaxf(alx - bhx, blx - ahx), 0.f);
    const float gy = fmaxf(fmaxf(aly - bhy, bly - ahy), 0.f);
    const float gz = fmaxf(fmaxf(alz - bhz, blz - ahz), 0.f);
    if constexpr (METRIC == kL2) {
        return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, gx * gx));
    } else if constexpr (METRIC == kL1) {
        return (gx + gy) + gz;
    } else {
        const float m = gx > gy ? gx : gy;
        return m > gz ? m : gz;
    }
}

// Rank of this lane among the kept lanes of km (mbcnt with a zero accumulator,
// an inline constant: the list position nc is then added in the address
// computation, one v_add_lshl, instead of moved into a VGPR for mbcnt).
__device__ __forceinline__ int keep_slot(uint64_t km) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(km >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(km), 0u)));
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

// popcount(x) + acc in one v_bcnt_u32_b32 (its second operand is added)
__device__ __forceinline__ uint32_t bcnt_add(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t rdlane(int v, uint32_t lane) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(v, static_cast<int>(lane)));
}

// lb[k] (uniform) into lane k for k = K..8
template <int K>
__device__ __forceinline__ int bin_lanes(int v, const uint32_t* lb) {
    if constexpr (K < 9) return bin_lanes<K + 1>(write_lane<K>(v, static_cast<int>(lb[K])), lb);
    return v;
}

// MODE 0: every query of the (sorted) query array; its first kRowCap
//         neighbours go to temp row qid, the full count to counts[qid]; ids of
//         queries with more than kRowCap neighbours are listed in `over` for
//         a MODE 1 re-run.  qkeys >> bshift is the query's batch item.
// MODE 1: the listed queries over[0 .. *m_dev) (one per wave; qpts is then
//         the raw [M, 3] query array) written straight into the final rows
//         at rs[qid].
#ifndef O3DML_FRS_NUM_SGPR
#define O3DML_FRS_NUM_SGPR 80  // <= 80 SGPRs keep 8 waves per SIMD (the 800-entry SGPR file)
#endif
// 8 waves per SIMD asked of the register allocator (<= 64 VGPRs): the
// search is VALU-issue bound and needs every wave (65 VGPRs -> 7 waves: +3 %).
// Not with distances (those builds would spill VGPRs to scratch).
#ifndef O3DML_FRS_WAVES
#define O3DML_FRS_WAVES 8
#endif
// REL16 temp rows hold the low 16 bits of the absolute id (the copy recovers
// the id from the item base), so the stream stores candidates unchanged
#ifndef O3DML_FRS_ABS16
#define O3DML_FRS_ABS16 1
#endif
#define O3DML_FRS_ATTR \
    __attribute__((amdgpu_num_sgpr(O3DML_FRS_NUM_SGPR), amdgpu_waves_per_eu(DIST ? 1 : O3DML_FRS_WAVES, 8)))
template <int METRIC, bool IGNORE, bool DIST, int MODE, class TIdx, bool REL16>
__global__ void __launch_bounds__(64) O3DML_FRS_ATTR
frs_group_kernel(const float4* __restrict__ pts, uint32_t n_pts, const uint32_t* __restrict__ cs,
                 const float4* __restrict__ qpts, const uint32_t* __restrict__ qsel,
                 const uint32_t* __restrict__ qkeys, int bshift, int64_t m_host, const int64_t* __restrict__ m_dev,
                 float r, float inv, float thr, int nb, const int64_t* __restrict__ qrs,
                 const uint32_t* __restrict__ hts, const int64_t* __restrict__ prs,
                 uint32_t* __restrict__ counts, uint32_t* __restrict__ tidx,
                 float* __restrict__ tdist, uint32_t* __restrict__ over, int64_t* __restrict__ n_over,
                 const int64_t* __restrict__ rs, TIdx* __restrict__ out_idx, float* __restrict__ out_dist,
                 const int64_t* __restrict__ total, int64_t cap, const uint32_t* __restrict__ dir,
                 int64_t dir_cap, int qlog, int64_t dense_w) {
    __shared__ float4 cand[kCandCap];
    __shared__ float4 qsh[64];
    __shared__ int64_t qrow[MODE == 0 ? 1 : 64];  // MODE 0: the row is the query id (qsh .w)
    const int lane = threadIdx.x;
    const float inf = __builtin_huge_valf();
    const float4 far = make_float4(inf, inf, inf, 0.f);  // never within any radius of a finite query
    // MODE 1 of a bounded fill whose rows do not fit the caller's capacity:
    // nothing is written (the caller re-runs the fill with exact buffers)
    const int64_t m = MODE == 1 && cap >= 0 && *total > cap ? 0 : (m_dev ? *m_dev : m_host);
    // MODE 0: 2^qlog queries per wave (64; 32 or 16 when there are too few
    // queries to give every SIMD a few waves); MODE 1: one query per wave
    const int64_t nchunks = MODE == 0 ? (m + (1 << qlog) - 1) >> qlog : m;
    // buffer resource over pts[0 .. 2 n_pts + 1] (bucket order, the far
    // sentinel, the class sub-lists p2) when its byte size fits the 32-bit range
    const bool pts_rsrc_ok = n_pts < 0x07FFFFFEu;
    // class directory present for every bin of the table
    const bool sub = dir != nullptr && static_cast<int64_t>(hts[nb]) <= dir_cap;
    // REL16 temp rows (2 B x kRowCap per query; REL16 implies they fit 2^31 B,
    // rel16_rows) through a buffer resource: one VALU per hit for the address
    const __amdgpu_buffer_rsrc_t rows_rsrc = __builtin_amdgcn_make_buffer_rsrc(
            tidx, static_cast<short>(0), REL16 ? static_cast<int>(m * 2 * kRowCap) : 0, kBufferFlags);
    const __amdgpu_buffer_rsrc_t pts_rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float4*>(pts), static_cast<short>(0), static_cast<int>((2u * n_pts + 1u) * 16u), kBufferFlags);
    // XCD-aware: workgroups are dealt round-robin to the 8 XCDs, so with a grid
    // of exactly 8 * per blocks, block b takes chunk (b % 8) * per + b / 8 —
    // every XCD sweeps one contiguous, spatially coherent range and its L2
    // keeps the shared buckets.  Otherwise plain grid stride.
    const int64_t per = (nchunks + 7) >> 3;
    const bool xcd_map = static_cast<int64_t>(gridDim.x) == 8 * per;
    int64_t chunk = xcd_map ? static_cast<int64_t>(blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
    for (; chunk < nchunks; chunk = xcd_map ? nchunks : chunk + gridDim.x) {
        const int64_t t = MODE == 0 ? (chunk << qlog) + lane : chunk;
        const bool valid = t < m && (MODE == 0 ? lane < (1 << qlog) : lane == 0);
        float4 q4 = far;
        QueryBins qb;
#pragma unroll
        for (int k = 0; k < 9; ++k) qb.b[k] = 0xffffffffu;
        int64_t row = 0;  // MODE 1: the query's final row start
        uint32_t pbase = 0;  // REL16: first point id of the query's batch item
        if (valid) {
            if constexpr (MODE == 0) {
                if (qsel) {
                    const uint32_t qs = qsel[t];
                    if (qpts) {  // the raw [M, 3] queries read through the (batch, Morton) order
                        const float* qp = reinterpret_cast<const float*>(qpts) + 3 * static_cast<int64_t>(qs);
                        q4 = make_float4(qp[0], qp[1], qp[2], __uint_as_float(qs));
                    } else {
                        q4 = pts[qs];  // self search in bucket order: the queries are points
                    }
                } else {
                    q4 = qpts[t];
                }
            } else {  // qpts = the raw query array [M, 3], over = the listed query ids
                const uint32_t id = over[t];
                const float* qp = reinterpret_cast<const float*>(qpts) + 3 * static_cast<int64_t>(id);
                q4 = make_float4(qp[0], qp[1], qp[2], __uint_as_float(id));
            }
            const uint32_t qid = __float_as_uint(q4.w);
            const int b = qkeys ? (bshift >= 32 ? 0 : static_cast<int>(qkeys[t] >> bshift)) : batch_of(qid, qrs, nb);
            if constexpr (REL16) pbase = static_cast<uint32_t>(prs[b]);
            const uint32_t first = hts[b], tsize = hts[b + 1] - first;
            qb = query_bins(q4.x, q4.y, q4.z, r, inv, first, tsize);
            // MODE 1 into a dense [M, dense_w] matrix: row qid starts at qid * dense_w
            if constexpr (MODE == 1) row = dense_w > 0 ? static_cast<int64_t>(qid) * dense_w : rs[qid];
        }
        uint64_t todo = __builtin_amdgcn_ballot_w64(valid);
        while (todo) {
            const int leader = __builtin_ctzll(todo);
            uint32_t lb[9];
            bool same = valid;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                lb[k] = rdlane(static_cast<int>(qb.b[k]), leader);
                same = same && qb.b[k] == lb[k];
            }
            const uint64_t gm = __builtin_amdgcn_ballot_w64(same);
            // a group shares its buckets, hence its batch item
            const uint32_t gbase = REL16 ? rdlane(static_cast<int>(pbase), leader) : 0u;
            todo &= ~gm;
            const int ng = __popcll(gm);
            __syncthreads();  // previous group done with qsh / cand
            if (same) {
                const uint32_t slot = mbcnt64(gm);
                qsh[slot] = q4;
                if constexpr (MODE == 1) qrow[slot] = row;
            }
            // group bounding box: groups of <= 16 (nearly all) reduce the member
            // slots qsh[0, ng) within one 16-lane DPP row, larger ones the whole wave
            float lx, ly, lz, hx, hy, hz;
            if (ng <= 16) {
                __syncthreads();
                const float4 v = lane < ng ? qsh[lane & 15] : far;
                const float4 w = lane < ng ? v : make_float4(-inf, -inf, -inf, 0.f);
                lx = row0_min_f(v.x), ly = row0_min_f(v.y), lz = row0_min_f(v.z);
                hx = row0_max_f(w.x), hy = row0_max_f(w.y), hz = row0_max_f(w.z);
            } else {
                lx = wave_min_f(same ? q4.x : inf), ly = wave_min_f(same ? q4.y : inf),
                lz = wave_min_f(same ? q4.z : inf);
                hx = wave_max_f(same ? q4.x : -inf), hy = wave_max_f(same ? q4.y : -inf),
                hz = wave_max_f(same ? q4.z : -inf);
            }
            // lane -> (query g, slice s)
            // S = floor(64 / ng) lanes per query (not a power of two: 9 queries
            // take 63 lanes, not 9 of 16 slots x 4); g = lane / S by the
            // multiply-shift of the table, exact for lane < 64
            const uint32_t split = kLaneSplit[ng];
            const int S = static_cast<int>(split & 0xffu);
            const int g = static_cast<int>((static_cast<uint32_t>(lane) * (split >> 8)) >> 16);
            const int sl = lane - g * S;
            __syncthreads();
            float4 mq = far;  // lanes past the group test the far point: never a hit
            int64_t mrow = 0;
            if (g < ng) {
                mq = qsh[g];
                mrow = MODE == 0 ? static_cast<int64_t>(__float_as_uint(mq.w)) : qrow[g];
            }
            uint32_t cnt = 0;  // neighbours of query g so far (uniform over its S lanes)
            const uint32_t row_b = static_cast<uint32_t>(mrow) * (2u * kRowCap);  // REL16: byte offset of the row
            const uint64_t gmask = S == 64 ? ~0ull : (g < ng ? ((1ull << S) - 1ull) << (g * S) : 0ull);
            const uint32_t gm_lo = static_cast<uint32_t>(gmask), gm_hi = static_cast<uint32_t>(gmask >> 32);
            // Bucket list of the group in visit order, empty and repeated bins
            // dropped: lane j < nbk holds the start (in pts, or in the class
            // sub-lists p2) and the length of the j-th stream segment.  Built in
            // parallel (lane k < 9 takes bin k) and compacted through the
            // candidate list, free here.  With the class directory, a bucket's
            // classes whose box is out of reach of the group's box are skipped
            // (box_box_dist: exact, see bucket_classes_kernel); one class left
            // streams its sub-list, none skips the bucket, more stream it whole.
            uint32_t vst, vlen;
            int nbk;
            {
                const uint32_t vb = static_cast<uint32_t>(bin_lanes<0>(-1, lb));
                uint32_t s0 = 0, e0 = 0;
                // the bin's bounds and its class directory entry in flight together
                // (the directory exists for every bin when `sub`)
                uint4 w0 = {}, w1 = {}, w2 = {}, w3 = {}, w4 = {}, w5 = {};
                if (lane < 9) {
                    s0 = cs[vb];
                    e0 = cs[vb + 1];
                    if (sub) {
                        const uint4* dp = reinterpret_cast<const uint4*>(dir + static_cast<size_t>(vb) * kDirWords);
                        w0 = dp[0], w1 = dp[1], w2 = dp[2], w3 = dp[3], w4 = dp[4], w5 = dp[5];
                    }
                }
                // the bins are sorted: a repeat sits right after its first copy
                const uint32_t prev = static_cast<uint32_t>(
                        __builtin_amdgcn_update_dpp(-1, static_cast<int>(vb), 0x111, 0xF, 0xF, false));  // row_shr:1
                const bool first = lane < 9 && e0 > s0 && prev != vb;
                uint32_t st = s0, ln = e0 - s0;
                if (first && sub) {
                    const uint32_t n0 = w0.x, n1 = w0.y, n2 = ln - n0 - n1;
                    auto f = [](uint32_t u) { return __uint_as_float(u); };
                    const bool r0 = n0 > 0 && box_box_dist<METRIC>(f(w1.x), f(w1.y), f(w1.z), f(w1.w), f(w2.x),
                                                                   f(w2.y), lx, ly, lz, hx, hy, hz) <= thr;
                    const bool r1 = n1 > 0 && box_box_dist<METRIC>(f(w2.z), f(w2.w), f(w3.x), f(w3.y), f(w3.z),
                                                                   f(w3.w), lx, ly, lz, hx, hy, hz) <= thr;
                    const bool r2 = n2 > 0 && box_box_dist<METRIC>(f(w4.x), f(w4.y), f(w4.z), f(w4.w), f(w5.x),
                                                                   f(w5.y), lx, ly, lz, hx, hy, hz) <= thr;
                    const int nr = static_cast<int>(r0) + static_cast<int>(r1) + static_cast<int>(r2);
                    const uint32_t base = n_pts + 1 + s0;  // the bucket's classes in p2
                    if (nr == 0) {
                        ln = 0;
                    } else if (nr == 1) {
                        st = r0 && n0 == ln ? s0 : base + (r0 ? 0u : (r1 ? n0 : n0 + n1));  // one voxel: pts
                        ln = r0 ? n0 : (r1 ? n1 : n2);
                    }
                }
                const bool live = first && ln > 0;
                const uint64_t km = __builtin_amdgcn_ballot_w64(live);
                nbk = __popcll(km);
                uint32_t* tab = reinterpret_cast<uint32_t*>(cand);
                if (live) {
                    const uint32_t j = mbcnt64(km);
                    tab[j] = st;
                    tab[16 + j] = ln;
                }
                __syncthreads();
                vst = lane < nbk ? tab[lane] : 0u;
                vlen = lane < nbk ? tab[16 + lane] : 0u;
                __syncthreads();
            }
#if O3DML_DIAG == 2
            nbk = 0;  // diagnostics: grouping and bucket tables only, no streaming
#endif
            // stop filling while the next round (and the test padding) might not fit
            const int fill_lim = kCandCap - 64 * kStreamU - (S - 1);
            // Stream cursor (uniform): bucket bk, boff of its entries consumed.  A
            // round of 64 lanes takes the rest of bucket bk (lanes < t) and the
            // head of bucket bk + 1, never more than two buckets; lanes past the
            // group's buckets (or past bucket bk + 1) read the far sentinel.
            int bk = 0;
            uint32_t boff = 0;
            auto round_src = [&]() -> uint32_t {
                if (bk >= nbk) return n_pts;
                const uint32_t st0 = rdlane(static_cast<int>(vst), bk) + boff;
                const uint32_t t = rdlane(static_cast<int>(vlen), bk) - boff;
                if (t > 64) {
                    boff += 64;
                    return st0 + lane;
                }
                const uint32_t n1 = rdlane(static_cast<int>(vlen), bk + 1);  // 0 past the list
                const uint32_t d1 = rdlane(static_cast<int>(vst), bk + 1) - t;
                const uint32_t src = static_cast<uint32_t>(lane) < t ? st0 + lane : d1 + lane;
                if (t + n1 <= 64) {
                    bk += 2;
                    boff = 0;
                } else {
                    bk += 1;
                    boff = 64 - t;
                }
                return static_cast<uint32_t>(lane) < t + n1 ? src : n_pts;
            };
            // all addresses of a step first, then all its loads (in flight together)
            auto load_step = [&](float4* c, auto buf) {
                uint32_t src[kStreamU];
#pragma unroll
                for (int u = 0; u < kStreamU; ++u) src[u] = round_src();
                if constexpr (decltype(buf)::value) {  // 16-B buffer loads: 32-bit offsets, never split
#pragma unroll
                    for (int u = 0; u < kStreamU; ++u)
                        c[u] = __builtin_bit_cast(float4,
                                                  __builtin_amdgcn_raw_buffer_load_b128(pts_rsrc, src[u] * 16u, 0, 0));
                } else {
#pragma unroll
                    for (int u = 0; u < kStreamU; ++u) c[u] = pts[src[u]];
                }
            };
            // the stream + test loop, instantiated for buffer loads and (huge
            // point sets) plain 64-bit loads: no per-step branch between them
            auto stream_and_test = [&](auto buf) {
            int nc = 0;
            while (true) {
                // 1. fill the LDS list: steps of kStreamU x 64 loads, all in flight
                //    (a software-pipelined variant that issued the next step before
                //    filtering this one measured 8 % slower: more VGPRs, fewer waves)
#if O3DML_FRS_DMA
                // LDS-DMA variant (buffer path): the kStreamU rounds land in the
                // list itself at nc + 64 u (no VGPRs held by loads in flight),
                // then each round is read back, filtered and compacted in place
                // (round u's targets end below round u + 1's landing zone)
                if constexpr (decltype(buf)::value) {
                    while (bk < nbk && nc <= fill_lim) {
                        uint32_t src[kStreamU];
#pragma unroll
                        for (int u = 0; u < kStreamU; ++u) src[u] = round_src();
                        const int nc0 = nc;
#pragma unroll
                        for (int u = 0; u < kStreamU; ++u)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(pts_rsrc, (frs_lds_ptr)(cand + nc0 + 64 * u), 16,
                                                                     src[u] * 16u, 0, 0, 0);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                        for (int u = 0; u < kStreamU; ++u) {
                            float4 c = cand[nc0 + 64 * u + lane];
                            const bool keep = box_dist<METRIC>(c, lx, ly, lz, hx, hy, hz) <= thr;
                            const uint64_t km = __builtin_amdgcn_ballot_w64(keep);
                            if constexpr (REL16 && !O3DML_FRS_ABS16) c.w = __uint_as_float(__float_as_uint(c.w) - gbase);
                            if (keep)
                                (cand + nc)[keep_slot(km)] = c;
                            nc += __popcll(km);
                        }
                    }
                }
                while (!decltype(buf)::value && bk < nbk && nc <= fill_lim) {
#else
                while (bk < nbk && nc <= fill_lim) {
#endif
                    float4 c[kStreamU];
                    load_step(c, buf);
#pragma unroll
                    for (int u = 0; u < kStreamU; ++u) {
                        const bool keep = box_dist<METRIC>(c[u], lx, ly, lz, hx, hy, hz) <= thr;
                        const uint64_t km = __builtin_amdgcn_ballot_w64(keep);
                        if constexpr (REL16 && !O3DML_FRS_ABS16)  // ids relative to the batch item
                            c[u].w = __uint_as_float(__float_as_uint(c[u].w) - gbase);
                        if (keep)
                            (cand + nc)[keep_slot(km)] = c[u];
                        nc += __popcll(km);
                    }
                }
                // 2. pad to whole S-entry slices with the far point, then test the
                //    list against the group's queries, in order (4 slices per
                //    step, then single slices); hits are ranked by ballot so every
                //    row is written in canonical order
                // nc rounded up to whole slices: ceil(nc / S) by the table's
                // multiply-shift (exact for nc + S - 1 < 65536 / S; nc <= kCandCap)
                const int ncp = static_cast<int>(((static_cast<uint32_t>(nc + S - 1) * (split >> 8)) >> 16) *
                                                 static_cast<uint32_t>(S));
                if (nc + lane < ncp) cand[nc + lane] = far;
                __syncthreads();
#if O3DML_DIAG == 0
                auto test = [&](float4 p) {
                    // w pinned here: the candidate comes in one ds_read_b128 (4 LDS
                    // cycles per wave) instead of ds_read_b96 (8) + a b32 for w
                    asm volatile("" : "+v"(p.w));
                    const float d = dist_metric<METRIC>(p.x, p.y, p.z, mq.x, mq.y, mq.z);
                    const bool hit = d <= thr && !(IGNORE && p.x == mq.x && p.y == mq.y && p.z == mq.z);
                    const uint64_t bal = __builtin_amdgcn_ballot_w64(hit);
                    const uint32_t mlo = static_cast<uint32_t>(bal) & gm_lo;
                    const uint32_t mhi = static_cast<uint32_t>(bal >> 32) & gm_hi;
#if O3DML_FRS_OOBST
                    if constexpr (MODE == 0 && REL16 && !DIST) {
                        // every lane stores: a miss gets an offset past the rows'
                        // buffer resource, which the buffer unit drops (no exec
                        // mask save / restore and branch per test)
                        const uint32_t pos = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, cnt));
                        const uint32_t ps = min(pos, static_cast<uint32_t>(kRowCap - 1));
                        __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(__float_as_uint(p.w)),
                                                              rows_rsrc, hit ? row_b + (ps << 1) : 0x80000000u, 0,
                                                              0);
                        cnt = bcnt_add(mhi, bcnt_add(mlo, cnt));
                        return;
                    }
#endif
                    if (hit) {
                        // mbcnt's accumulator operand adds the running count for free
                        const uint32_t pos = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, cnt));
                        if constexpr (MODE == 0) {
                            // rows longer than kRowCap are re-run (MODE 1), so their
                            // temp row may take anything in its last slot
                            const uint32_t ps = min(pos, static_cast<uint32_t>(kRowCap - 1));
                            if constexpr (REL16)  // 16-bit ids relative to the batch item: 128-B rows
                                __builtin_amdgcn_raw_buffer_store_b16(
                                        static_cast<unsigned short>(__float_as_uint(p.w)), rows_rsrc,
                                        row_b + (ps << 1), 0, 0);
                            else
                                tidx[mrow * kRowCap + ps] = __float_as_uint(p.w);
                            if constexpr (DIST) tdist[mrow * kRowCap + ps] = d;
                        } else {
                            out_idx[mrow + pos] = static_cast<TIdx>(__float_as_uint(p.w));
                            if constexpr (DIST) out_dist[mrow + pos] = d;
                        }
                    }
                    cnt = bcnt_add(mhi, bcnt_add(mlo, cnt));
                };
                int e0 = 0;
                for (; e0 + 4 * S <= ncp; e0 += 4 * S) {
                    float4 p[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) p[u] = cand[e0 + u * S + sl];
#pragma unroll
                    for (int u = 0; u < 4; ++u) test(p[u]);
                }
                for (; e0 < ncp; e0 += S) test(cand[e0 + sl]);
#endif
                __syncthreads();
                nc = 0;
                if (bk >= nbk) break;
            }
            };
            if (pts_rsrc_ok)
                stream_and_test(std::true_type{});
            else
                stream_and_test(std::false_type{});
            if constexpr (MODE == 0) {
                if (g < ng && sl == 0) {
                    counts[__float_as_uint(mq.w)] = cnt;
                    if (cnt > static_cast<uint32_t>(kRowCap))
                        over[atomicAdd(reinterpret_cast<unsigned long long*>(n_over), 1ull)] =
                                static_cast<uint32_t>(mrow);
                }
            }
        }
    }
}

// Final rows from the temp rows (already in canonical order, temp row = query
// id, so both sides stream in order).  A wave owns 64 consecutive rows;
// lanes = entries of one row, 8 rows in flight: one coalesced load of the
// row's live entries (lanes past the count read a zero word, so no load sits
// under a branch) and one coalesced store.  REL16: the temp rows hold 16-bit
// ids relative to the batch item's first point (one 128-B line per row), the
// item base is added back here.  Rows longer than kRowCap are written by the
// MODE 1 re-run.
__device__ uint32_t g_frs_zero[4];
#ifndef O3DML_COPY_ROWS
#define O3DML_COPY_ROWS 64  // all 64 rows of the wave: copy 218 -> 213 us vs 32 (16: 240; profiles/r05/frs_copy_rows_ab.txt)
#endif
constexpr int kCopyRows = O3DML_COPY_ROWS;  // rows whose loads are in flight together

template <bool DIST, bool REL16, class TIdx>
__global__ void __launch_bounds__(256) group_rows_copy_kernel(int64_t m, const uint32_t* __restrict__ counts,
                                                              const int64_t* __restrict__ rs,
                                                              const int64_t* __restrict__ qrs,
                                                              const int64_t* __restrict__ prs, int nb,
                                                              const uint32_t* __restrict__ tidx,
                                                              const float* __restrict__ tdist,
                                                              TIdx* __restrict__ idx, float* __restrict__ dist,
                                                              int64_t cap) {
    if (cap >= 0 && rs[m] > cap) return;  // bounded fill, rows do not fit: write nothing
    const int lane = threadIdx.x & 63;
    const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tidx);
    for (int64_t base = wave * 64; base < m; base += nwaves * 64) {
        const int64_t t = base + lane;
        int n = 0;
        int64_t o = 0;
        uint32_t pb = 0;
        if constexpr (REL16) {  // the 64 rows usually share one batch item: one uniform (scalar) search
            const int64_t ub = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(base >> 6))) << 6;
            const int b0 = batch_of(ub, qrs, nb);
            const int64_t last = min(ub + 63, m - 1);
            pb = static_cast<uint32_t>(prs[b0]);
            if (qrs[b0 + 1] <= last && t < m) pb = static_cast<uint32_t>(prs[batch_of(t, qrs, nb)]);
        }
        if (t < m) {
            const uint32_t c = counts[t];
            n = c <= static_cast<uint32_t>(kRowCap) ? static_cast<int>(c) : 0;
            o = rs[t];
        }
        for (int k = 0; k < 64; k += kCopyRows) {
            uint32_t v[kCopyRows];
            float dv[kCopyRows];
#pragma unroll
            for (int u = 0; u < kCopyRows; ++u) {
                const int nu = __builtin_amdgcn_readlane(n, k + u);
                const int64_t src = (base + k + u) * kRowCap + lane;
                const bool live = lane < nu;
                if constexpr (REL16)
                    v[u] = *(live ? t16 + src : reinterpret_cast<const uint16_t*>(g_frs_zero));
                else
                    v[u] = *(live ? tidx + src : g_frs_zero);
                if constexpr (DIST) dv[u] = *(live ? tdist + src : reinterpret_cast<const float*>(g_frs_zero));
            }
#pragma unroll
            for (int u = 0; u < kCopyRows; ++u) {
                const int nu = __builtin_amdgcn_readlane(n, k + u);
                const int64_t ou = static_cast<int64_t>(
                        (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(o >> 32), k + u))) << 32) |
                        static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(o), k + u)));
                const uint32_t pbu = REL16 ? static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pb), k + u)) : 0u;
                if (lane < nu) {
                    // ABS16: the low 16 bits of the id; the id is pbu + ((v - pbu) mod 2^16),
                    // as every id of the item lies in [pbu, pbu + 2^16)
                    idx[ou + lane] = static_cast<TIdx>(O3DML_FRS_ABS16 && REL16 ? pbu + ((v[u] - pbu) & 0xffffu)
                                                                                 : v[u] + pbu);
                    if constexpr (DIST) dist[ou + lane] = dv[u];
                }
            }
        }
    }
}

// Final rows into a dense int32 [M, width] matrix padded with `pad` (KPConv's
// batch_neighbors, kpconv.py:2002-2034: fixed_radius_search + ragged_to_dense
// in one pass).  One wave per row; rows longer than kRowCap get only their
// padding here (the MODE 1 re-run writes their entries at row * width).
template <bool REL16>
__global__ void __launch_bounds__(256) group_rows_dense_kernel(int64_t m, const uint32_t* __restrict__ counts,
                                                               const int64_t* __restrict__ qrs,
                                                               const int64_t* __restrict__ prs, int nb,
                                                               const uint32_t* __restrict__ tidx, int64_t width,
                                                               int32_t pad, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tidx);
    for (int64_t t = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; t < m; t += nwaves) {
        const uint32_t c = counts[t];
        const int64_t n = c <= static_cast<uint32_t>(kRowCap) ? static_cast<int64_t>(c) : 0;  // entries copied here
        const int64_t n_all = static_cast<int64_t>(c);
        const uint32_t pb = REL16 ? static_cast<uint32_t>(prs[batch_of(t, qrs, nb)]) : 0u;
        int32_t* row = out + t * width;
        for (int64_t j = lane; j < width; j += 64) {
            if (j < n)
                row[j] = static_cast<int32_t>(REL16 ? (O3DML_FRS_ABS16 ? pb + ((t16[t * kRowCap + j] - pb) & 0xffffu)
                                                                       : t16[t * kRowCap + j] + pb)
                                                    : tidx[t * kRowCap + j]);
            else if (j >= n_all)
                row[j] = pad;
        }
    }
}

// Query order: (batch, Morton code of the query's r-cell) — the lowest Morton
// level is the octant of the Open3D 2r-cell, so queries with identical visit
// lists (one group) are adjacent, and consecutive chunks are spatial
// neighbours that share buckets in L2.  Cell coordinates wrap modulo
// 2^cell_bits (locality only; any order is correct — grouping inside the
// kernel compares the full bucket lists).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// (batch, Morton r-cell) key of every query.  F4: the queries are the points
// in Open3D bucket order (pts, float4), so the sorted payload is a position in
// pts — the search then reads each query from the same lines its group
// streams (large self searches); else the raw [M, 3] query array.
template <bool F4>
__global__ void __launch_bounds__(256) group_query_keys_kernel(const float* __restrict__ queries, int64_t m,
                                                               float inv2, int n_batch,
                                                               const int64_t* __restrict__ qrs, int cell_bits,
                                                               uint32_t* __restrict__ keys) {
    __shared__ int64_t s_rs[kLdsSplits];
    const int64_t* rsp = stage_splits(s_rs, qrs, n_batch);
    const uint32_t mask = (1u << cell_bits) - 1u;
    constexpr int W = F4 ? 4 : 3;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < m;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(i, rsp, n_batch);
        float x, y, z;
        if constexpr (F4) {
            const float4 p = reinterpret_cast<const float4*>(queries)[i];
            x = p.x, y = p.y, z = p.z;
        } else {
            x = queries[W * i], y = queries[W * i + 1], z = queries[W * i + 2];
        }
        const uint32_t cx = static_cast<uint32_t>(static_cast<int32_t>(floorf(x * inv2))) & mask;
        const uint32_t cy = static_cast<uint32_t>(static_cast<int32_t>(floorf(y * inv2))) & mask;
        const uint32_t cz = static_cast<uint32_t>(static_cast<int32_t>(floorf(z * inv2))) & mask;
        const uint32_t mort = spread3(cx) | (spread3(cy) << 1) | (spread3(cz) << 2);
        keys[i] = (static_cast<uint32_t>(b) << (3 * cell_bits)) | mort;
    }
}

// Voxel classes of the buckets.  Open3D's table has about one bucket per
// occupied 2r-voxel, so a bucket a query group visits holds ~2 voxels and the
// group usually reaches one of them.  bucket_classes_kernel splits every
// bucket into three classes — the voxel of its first entry, the first other
// voxel seen, the rest — and writes a second copy of the points,
// p2 = pts[n + 1 ..], ordered by (bucket, class, id), plus a directory entry
// per bucket: the sizes of classes 0 and 1 and the exact float bounding box
// of each class.  The search skips a class when the distance bound between
// its box and the group's box exceeds the radius (monotone float ops in the
// metric's order, as box_dist: every skipped point would fail the exact test
// for every member), and streams one class's sub-list when it is the only one
// left (ids ascending: Open3D's order), the whole bucket otherwise.
//
// Self search (queries = points) also takes the query order from here: each
// bucket's entries by (class, octant), so the queries of one group — same
// voxel, same octant, hence the same 9 visited bins — are adjacent and 64
// consecutive queries form few groups, with no sort of the queries (qpts,
// qbatch[t] = batch item of query t; 256 entries at a time: longer buckets
// are ordered chunk by chunk, any order is correct).
constexpr int kSelfChunk = 256;  // bucket entries ordered at once

// wave-wide int min / max: DPP within the 16-lane rows, then the 4 row results
template <bool MAX>
__device__ __forceinline__ int32_t wave_ext_i(int32_t v) {
    auto op = [](int32_t a, int32_t b) { return MAX ? max(a, b) : min(a, b); };
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm(1,0,3,2)
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm(2,3,0,1)
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));  // row_mirror
    return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
              op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int32_t wave_min_i(int32_t v) { return wave_ext_i<false>(v); }
__device__ __forceinline__ int32_t wave_max_i(int32_t v) { return wave_ext_i<true>(v); }

// O3DML_BC_WAVES: waves per SIMD asked of the register allocator (A/B
// builds; 0 = the compiler's choice, 90 VGPRs -> 5 waves per SIMD)
#ifndef O3DML_BC_WAVES
#define O3DML_BC_WAVES 0
#endif
#if O3DML_BC_WAVES > 0
#define O3DML_BC_ATTR __attribute__((amdgpu_waves_per_eu(O3DML_BC_WAVES, 8)))
#else
#define O3DML_BC_ATTR
#endif
__global__ void __launch_bounds__(256) O3DML_BC_ATTR bucket_classes_kernel(const float* __restrict__ points,
                                                             const uint32_t* __restrict__ hti,
                                                             float4* __restrict__ pts, int64_t n_pts,
                                                             const uint32_t* __restrict__ cs,
                                                             const uint32_t* __restrict__ hts, int nb, float inv,
                                                             float cell, uint32_t* __restrict__ dir, int64_t dir_cap,
                                                             uint32_t* __restrict__ qsel,
                                                             uint32_t* __restrict__ qbatch,
                                                             int64_t* __restrict__ zero_a, int n_zero_a,
                                                             int64_t* __restrict__ zero_b) {
    constexpr int E = kSelfChunk / 64;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const float inf = __builtin_huge_valf();
        pts[n_pts] = make_float4(inf, inf, inf, 0.f);  // the far sentinel: beyond every radius
        for (int j = 0; j < n_zero_a; ++j) zero_a[j] = 0;  // zeroed words of the caller
        if (zero_b) *zero_b = 0;
    }
    __shared__ uint32_t s_hts[kLdsSplits];
    __shared__ uint32_t wcnt[4][32];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool lds_hts = nb + 1 <= kLdsSplits;
    if (lds_hts)
        for (int i = threadIdx.x; i <= nb; i += blockDim.x) s_hts[i] = hts[i];
    __syncthreads();
    const uint32_t* H = lds_hts ? s_hts : hts;
    const int64_t nbins = H[nb];
    const bool with_dir = dir != nullptr && nbins <= dir_cap;  // else the search streams whole buckets
    float4* p2 = pts + n_pts + 1;
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    const uint64_t lt = lanemask_lt();
    // XCD-contiguous (xcd_block): each XCD orders the buckets whose points its
    // L2 received from the XCD-contiguous gather
    int64_t bin = xcd_block() * 4 + wv;
    uint32_t s = bin < nbins ? cs[bin] : 0u, e = bin < nbins ? cs[bin + 1] : 0u;
    for (; bin < nbins; bin += nwaves) {
        // next bucket's bounds in flight while this one is ordered
        const int64_t nbin = bin + nwaves;
        const uint32_t ns = nbin < nbins ? cs[nbin] : 0u, ne = nbin < nbins ? cs[nbin + 1] : 0u;
        if (s < e) {
            int lo = 0, hi = nb - 1;  // batch item of the bucket (uniform)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (H[mid] <= bin) lo = mid; else hi = mid - 1;
            }
            float4 p[E];
            int32_t vx[E], vy[E], vz[E];
            uint32_t oct[E];
            int rows = 0;
            // the bucket's points gathered through Open3D's hash_table_index;
            // the first pass also writes them to pts in that order (one
            // bucket = one contiguous 16-B-per-point stream for the search)
            auto load_chunk = [&](uint32_t c0, uint32_t len, bool store) {
                rows = static_cast<int>((len + 63) >> 6);  // rows past it are skipped (uniform)
                // every id and point load unconditional (clamped to entry c0,
                // len >= 1) and issued before any store: under the per-row
                // conditions each point gather waited for the previous row's
                // pts store (vmcnt counts stores), four round trips in series
                uint32_t id[E];
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    const uint32_t i = lane + 64 * h;
                    id[h] = hti[c0 + (i < len ? i : 0u)];
                }
                float qx[E], qy[E], qz[E];
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    const float* q = points + 3 * static_cast<int64_t>(id[h]);
                    qx[h] = q[0];
                    qy[h] = q[1];
                    qz[h] = q[2];
                }
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    if (h >= rows) {
                        vx[h] = vy[h] = vz[h] = 0;
                        oct[h] = 0u;
                        continue;
                    }
                    const uint32_t i = lane + 64 * h;
                    p[h] = i < len ? make_float4(qx[h], qy[h], qz[h], __uint_as_float(id[h]))
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
                    if (store && i < len) pts[c0 + i] = p[h];
                    // the 2r-voxel as the hash build computes it; the octant
                    // (query order only) from the fractional part
                    const float fx = p[h].x * inv, fy = p[h].y * inv, fz = p[h].z * inv;
                    const float gx = floorf(fx), gy = floorf(fy), gz = floorf(fz);
                    vx[h] = static_cast<int32_t>(gx);
                    vy[h] = static_cast<int32_t>(gy);
                    vz[h] = static_cast<int32_t>(gz);
                    oct[h] = (fx - gx >= 0.5f ? 1u : 0u) | (fy - gy >= 0.5f ? 2u : 0u) | (fz - gz >= 0.5f ? 4u : 0u);
                }
            };
            // pass 1: the class voxels and sizes, and the voxel range of class 2
            int32_t ax = 0, ay = 0, az = 0, bx = 0, by = 0, bz = 0;
            bool have1 = false;
            uint32_t n0 = 0, n1 = 0;
            int32_t rlx = INT32_MAX, rly = INT32_MAX, rlz = INT32_MAX, rhx = INT32_MIN, rhy = INT32_MIN,
                    rhz = INT32_MIN;  // lane-partial voxel range of class 2
            auto classify = [&](int h) {
                const bool is0 = vx[h] == ax && vy[h] == ay && vz[h] == az;
                const bool is1 = have1 && !is0 && vx[h] == bx && vy[h] == by && vz[h] == bz;
                return is0 ? 0 : (is1 ? 1 : 2);
            };
            const bool one_chunk = e - s <= static_cast<uint32_t>(kSelfChunk);
            for (uint32_t c0 = s; c0 < e; c0 += kSelfChunk) {
                const uint32_t len = min(e - c0, static_cast<uint32_t>(kSelfChunk));
                load_chunk(c0, len, true);
                if (c0 == s) {
                    ax = rdlane(vx[0], 0);
                    ay = rdlane(vy[0], 0);
                    az = rdlane(vz[0], 0);
                }
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    if (h >= rows) break;
                    const bool valid = lane + 64 * h < len;
                    if (!have1) {  // first entry of another voxel (entry order)
                        const uint64_t other = __builtin_amdgcn_ballot_w64(
                                valid && !(vx[h] == ax && vy[h] == ay && vz[h] == az));
                        if (other) {
                            const int l = __builtin_ctzll(other);
                            bx = rdlane(vx[h], l);
                            by = rdlane(vy[h], l);
                            bz = rdlane(vz[h], l);
                            have1 = true;
                        }
                    }
                    const int c = classify(h);
                    n0 += __popcll(__builtin_amdgcn_ballot_w64(valid && c == 0));
                    n1 += __popcll(__builtin_amdgcn_ballot_w64(valid && c == 1));
                    if (valid && c == 2) {
                        rlx = min(rlx, vx[h]), rly = min(rly, vy[h]), rlz = min(rlz, vz[h]);
                        rhx = max(rhx, vx[h]), rhy = max(rhy, vy[h]), rhz = max(rhz, vz[h]);
                    }
                }
            }
            if (with_dir) {
                // class boxes from the voxel ranges: a point p of voxel W has
                // floor(fl(p inv)) = W, so p inv lies in [W - 1/16, W + 1 + 1/8]
                // while |W| < 2^20 (relative rounding 2^-24 of the product); the
                // box [(W - 0.5) 2r, (W + 1.5) 2r] in float holds it with >= 1/4
                // voxel to spare for the rounding of the box edges and of
                // 1 / inv vs 2r (within 2^16 voxels: 1/32-voxel margins, the
                // rounding being < 1/128 voxel).  Beyond 2^20: no box.
                const uint32_t n2 = (e - s) - n0 - n1;
                if (n2 > 0) {
                    rlx = wave_min_i(rlx), rly = wave_min_i(rly), rlz = wave_min_i(rlz);
                    rhx = wave_max_i(rhx), rhy = wave_max_i(rhy), rhz = wave_max_i(rhz);
                }
                // lane 4 + 6 k + d: class k, value d (min x y z, max x y z)
                const int j = lane - 4, k = j / 6, d = j % 6;
                const int32_t vlo[3][3] = {{ax, ay, az}, {bx, by, bz}, {rlx, rly, rlz}};
                const int32_t vhi[3][3] = {{ax, ay, az}, {bx, by, bz}, {rhx, rhy, rhz}};
                uint32_t w = lane == 0 ? n0 : (lane == 1 ? n1 : 0u);
                if (j >= 0 && j < 18) {
                    int32_t vl = 0, vh = 0;
#pragma unroll
                    for (int kk = 0; kk < 3; ++kk)
#pragma unroll
                        for (int dd = 0; dd < 3; ++dd)
                            if (kk == k && dd == d % 3) vl = vlo[kk][dd], vh = vhi[kk][dd];
                    const bool ok = vl > -(1 << 20) && vh < (1 << 20);
                    // within 2^16 voxels of the origin the rounding is < 1/128 voxel:
                    // a 1/32-voxel margin suffices
                    const bool near0 = vl > -(1 << 16) && vh < (1 << 16);
                    const float mg = near0 ? 0.03125f : 0.5f;
                    const float edge = d < 3 ? (static_cast<float>(vl) - mg) * cell
                                             : (static_cast<float>(vh) + (1.0f + mg)) * cell;
                    w = __float_as_uint(ok ? edge : (d < 3 ? -__builtin_huge_valf() : __builtin_huge_valf()));
                }
                if (lane < kDirWords) dir[bin * kDirWords + lane] = w;
            }
            // pass 2: p2 by (class, id) — not for a one-voxel bucket, whose only
            // class is the bucket itself (the search streams it from pts);
            // queries by (class, octant) per chunk
            const bool single = n0 == e - s;
            uint32_t run0 = 0, run1 = n0, run2 = n0 + n1;
            for (uint32_t c0 = s; c0 < e; c0 += kSelfChunk) {
                const uint32_t len = min(e - c0, static_cast<uint32_t>(kSelfChunk));
                if (!one_chunk) load_chunk(c0, len, false);
                if (qsel && lane < 32) wcnt[wv][lane] = 0;
                __builtin_amdgcn_wave_barrier();
                uint32_t dig[E], loff[E];
#pragma unroll
                for (int h = 0; h < E; ++h) {  // rows in order: stable within a class
                    if (h >= rows) break;
                    const bool valid = lane + 64 * h < len;
                    const int c = classify(h);
                    const uint64_t m0 = __builtin_amdgcn_ballot_w64(valid && c == 0);
                    const uint64_t m1 = __builtin_amdgcn_ballot_w64(valid && c == 1);
                    const uint64_t m2 = __builtin_amdgcn_ballot_w64(valid && c == 2);
                    const uint64_t mine = c == 0 ? m0 : (c == 1 ? m1 : m2);
                    const uint32_t run = c == 0 ? run0 : (c == 1 ? run1 : run2);
                    if (valid && !single) p2[s + run + __popcll(mine & lt)] = p[h];
                    run0 += __popcll(m0);
                    run1 += __popcll(m1);
                    run2 += __popcll(m2);
                    if (qsel) {
                        const uint32_t d = (static_cast<uint32_t>(c) << 3) | oct[h];
                        dig[h] = d;
                        uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
                        for (int bb = 0; bb < 5; ++bb) {
                            const bool bit = (d >> bb) & 1u;
                            const uint64_t mm = __builtin_amdgcn_ballot_w64(bit);
                            peers &= bit ? mm : ~mm;
                        }
                        const uint32_t rank = __popcll(peers & lt);
                        const uint32_t before = valid ? wcnt[wv][d] : 0u;
                        loff[h] = before + rank;
                        if (valid && rank == 0) wcnt[wv][d] = before + static_cast<uint32_t>(__popcll(peers));
                    }
                }
                if (qsel) {
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t cnt = lane < 32 ? wcnt[wv][lane] : 0u;
                    const uint32_t base = wave_inclusive_scan(cnt) - cnt;  // class bases
#pragma unroll
                    for (int h = 0; h < E; ++h) {
                        if (h >= rows) break;
                        const uint32_t i = lane + 64 * h;
                        const uint32_t pos = static_cast<uint32_t>(
                                                     __shfl(static_cast<int>(base), static_cast<int>(dig[h]), 64)) +
                                             loff[h];
                        if (i < len) {
                            qsel[c0 + pos] = c0 + i;
                            qbatch[c0 + pos] = static_cast<uint32_t>(lo);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        s = ns;
        e = ne;
    }
}

// Self search queries in Open3D's bucket order (bucket_classes_kernel) —
// unless a batch item is so large that the hash order of its buckets, which
// is spatially random, costs more in L2 misses than a Morton sort of the
// queries (>= 2^22 points: search 6.19 -> 4.55 ms at 2^24 points, the sort
// and query gather 0.9 ms; break-even at 2^22).  Ordering the buckets
// spatially instead was measured and lost: ~63 % of the cells share their
// bucket with another cell at Open3D's table size, and those are placed with
// the bucket's first cell, off their own spatial position.
#ifndef O3DML_FRS_SELF_ORDER_MAX
#define O3DML_FRS_SELF_ORDER_MAX (int64_t(1) << 22)
#endif
static bool frs_self_order(int64_t n_batch, const int64_t* prs_host, int64_t n_points) {
    const char* e = std::getenv("O3DML_FRS_SELF_ORDER");  // "0" never, "1" always (A/B)
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    int64_t mx = n_points / std::max<int64_t>(n_batch, 1);
    if (prs_host) {
        mx = 0;
        for (int64_t b = 0; b < n_batch; ++b) mx = std::max(mx, prs_host[b + 1] - prs_host[b]);
    }
    return mx < O3DML_FRS_SELF_ORDER_MAX;
}

// Morton-ordered queries (items of >= 2^22 points, or queries != points):
// the search reads the raw [M, 3] queries through the sorted order (default)
// instead of a gathered float4 copy — the gather cost 0.38 ms at 2^24 points
// and the search hides the scattered 12-B query reads.  O3DML_FRS_QGATHER=1:
// the gathered copy (A/B).
static bool frs_query_gather() {
    static const bool v = [] {
        const char* e = std::getenv("O3DML_FRS_QGATHER");
        return e && e[0] == '1';
    }();
    return v;
}

// Self searches of large items (Morton query order) sort the POINTS IN
// BUCKET ORDER by their Morton r-cell, so the search reads each query (16 B,
// aligned) from pts — lines its group streams anyway — instead of 12 B from
// the raw array through a random gather (one 128-B line per query that no
// other access reuses).  O3DML_FRS_SELF_PTS=0: the raw-array order (A/B).
static bool frs_self_pts_order() {
    static const bool v = [] {
        const char* e = std::getenv("O3DML_FRS_SELF_PTS");
        return !(e && e[0] == '0');
    }();
    return v;
}

// log2 of the queries per wave of the MODE 0 search: 64 while that still
// gives >= 4096 waves (4 per SIMD), else 32 / 16 — a small call (one C1 scene,
// 65,536 queries: 1,024 waves of 64) is latency-bound on one wave per SIMD.
// More waves of fewer queries split a few groups that 64-query waves keep
// whole (more bucket streaming), which only pays while the chip is short of waves.
static int frs_qlog(int64_t m) {
    static const int env = [] {
        const char* e = std::getenv("O3DML_FRS_QLOG");
        return e ? std::atoi(e) : 0;
    }();
    if (env >= 2 && env <= 6) return env;
    if (m >= 4096 * 64) return 6;
    return m >= 4096 * 32 ? 5 : 4;
}

static unsigned group_grid(int64_t m, int queries_per_wave = 64) {
    const int64_t per = ((m + queries_per_wave - 1) / queries_per_wave + 7) / 8;
    return static_cast<unsigned>(std::max<int64_t>(8, std::min<int64_t>(8 * per, 1 << 20)));
}

template <int MODE, class TIdx>
static void launch_group(int metric, bool ignore, bool with_dist, bool rel16, hipStream_t st, unsigned grid,
                         const float4* pts, uint32_t n_pts, const uint32_t* cs, const float4* qpts,
                         const uint32_t* qsel,
                         const uint32_t* qkeys, int bshift, int64_t m, const int64_t* m_dev, float r, float inv,
                         float thr, int nb, const int64_t* qrs, const uint32_t* hts, const int64_t* prs,
                         uint32_t* counts, uint32_t* tidx, float* tdist, uint32_t* over, int64_t* n_over,
                         const int64_t* rs, TIdx* idx, float* dist, const uint32_t* dir, int64_t dir_cap,
                         const int64_t* total = nullptr, int64_t cap = -1, int qlog = 6, int64_t dense_w = 0) {
#define O3DML_GRP(M, I, D, R)                                                                                   \
    frs_group_kernel<M, I, D, MODE, TIdx, R><<<grid, 64, 0, st>>>(pts, n_pts, cs, qpts, qsel, qkeys, bshift, m, m_dev, \
                                                                   r, inv, thr, nb, qrs, hts, prs, counts, tidx,  \
                                                                   tdist, over, n_over, rs, idx, dist, total, cap, dir, dir_cap, qlog, \
                                                                   dense_w)
#define O3DML_GRP_R(M, I, D)                                  \
    do {                                                      \
        if (MODE == 0 && rel16)                               \
            O3DML_GRP(M, I, D, MODE == 0);                    \
        else                                                  \
            O3DML_GRP(M, I, D, false);                        \
    } while (0)
#define O3DML_GRP_D(M, I)              \
    do {                               \
        if (with_dist)                 \
            O3DML_GRP_R(M, I, true);   \
        else                           \
            O3DML_GRP_R(M, I, false);  \
    } while (0)
    if (metric == kL2) {
        if (ignore) O3DML_GRP_D(kL2, true); else O3DML_GRP_D(kL2, false);
    } else if (metric == kL1) {
        if (ignore) O3DML_GRP_D(kL1, true); else O3DML_GRP_D(kL1, false);
    } else {
        if (ignore) O3DML_GRP_D(kLinf, true); else O3DML_GRP_D(kLinf, false);
    }
#undef O3DML_GRP_D
#undef O3DML_GRP_R
#undef O3DML_GRP
    O3DML_LAUNCH_CHECK();
}

// Workspace kept between _count and _fill (same layout in both entries).
struct FrsPlan {
    int64_t* scalars;  // [0] overflow count
    float4* pts;       // [2 (N + 1)] points in Open3D bucket order, a far sentinel, the class sub-lists p2
    float4* qpts;      // [M] queries in (batch, Morton) order
    uint32_t* keys;    // [M]
    uint32_t* skeys;   // [M]
    uint32_t* qorder;  // [M]
    uint32_t* counts;  // [M]
    uint32_t* over;    // [M]
    uint32_t* tidx;    // [M * kRowCap]
    float* tdist;      // [M * kRowCap] (with distances)
    uint32_t* dir;     // [dir_cap * kDirWords] voxel-class directory per bucket
    int64_t dir_cap;   // bins the directory holds (dir_bins)
};

// Bins the class directory holds: twice Open3D's default table (N_b / 64
// bins per item); a table with more bins streams whole buckets
static int64_t dir_bins(int64_t n, int64_t nb) { return n / 32 + 2 * nb + 64; }

static FrsPlan take_plan(Workspace& ws, int64_t n, int64_t m, int64_t nb, bool dist) {
    FrsPlan p;
    p.scalars = ws.take<int64_t>(4);
    p.pts = ws.take<float4>(2 * (n + 1));  // + far sentinel + p2
    p.qpts = ws.take<float4>(m);
    p.keys = ws.take<uint32_t>(m);
    p.skeys = ws.take<uint32_t>(m);
    p.qorder = ws.take<uint32_t>(m);
    p.counts = ws.take<uint32_t>(m);
    p.over = ws.take<uint32_t>(m);
    p.tidx = ws.take<uint32_t>(m * kRowCap);
    p.tdist = dist ? ws.take<float>(m * kRowCap) : nullptr;
    p.dir_cap = dir_bins(n, nb);
    p.dir = ws.take<uint32_t>(p.dir_cap * kDirWords);
    return p;
}

// Temp rows hold 16-bit ids relative to the batch item's first point when no
// batch item has more than 65,536 points (host copy of the point row splits).
#ifndef O3DML_FRS_REL16
#define O3DML_FRS_REL16 1
#endif
// Side stream for the re-run of rows longer than kRowCap, one per device of
// the CALLER'S stream (not the current device: the tensors may live on
// another GPU).  The re-run needs only the count's outputs and writes rows the
// row copy skips, so it runs beside the copy: fork = an event recorded on the
// caller's stream when the fill is issued (after the count, before the copy),
// join = the caller's stream waits for the side stream.  The fork/launch/join
// sequence holds the device's lock, so concurrent searches on other streams
// or threads can neither re-record the fork nor the join in between (an event
// wait binds the event's state at the time of the wait call).  Created once,
// never freed.
struct FrsSide {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    std::mutex mu;
};
static int stream_device(hipStream_t st) {
    int dev = 0;
    if (st) {
        hipDevice_t d = 0;
        O3DML_CHECK_HIP(hipStreamGetDevice(st, &d));
        dev = static_cast<int>(d);
    } else {
        O3DML_CHECK_HIP(hipGetDevice(&dev));
    }
    return dev;
}
static FrsSide& frs_side(int dev) {
    static std::mutex mu;
    static FrsSide side[64];
    std::lock_guard<std::mutex> lock(mu);
    FrsSide& x = side[dev & 63];
    if (!x.s) {
        int cur = 0;
        O3DML_CHECK_HIP(hipGetDevice(&cur));
        O3DML_CHECK_HIP(hipSetDevice(dev));  // the stream and events belong to the caller's device
        O3DML_CHECK_HIP(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking));
        O3DML_CHECK_HIP(hipEventCreateWithFlags(&x.fork, hipEventDisableTiming));
        O3DML_CHECK_HIP(hipEventCreateWithFlags(&x.join, hipEventDisableTiming));
        O3DML_CHECK_HIP(hipSetDevice(cur));
    }
    return x;
}
// Restores the current device on scope exit (launches follow the stream's device).
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        O3DML_CHECK_HIP(hipGetDevice(&prev));
        if (prev != dev) O3DML_CHECK_HIP(hipSetDevice(dev)); else prev = -1;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// [total, overflow count] straight into the caller's pinned host buffer
__global__ void frs_totals_kernel(const int64_t* __restrict__ rs, int64_t m, const int64_t* __restrict__ scalars,
                                  int64_t* __restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = rs[m];
        out[1] = scalars[0];
    }
}

// out = [total, overflow count, widest row] (the dense neighbour matrix of
// KPConv's batch_neighbors needs the width): one workgroup
__global__ void __launch_bounds__(1024) frs_sizes_kernel(const int64_t* __restrict__ rs, int64_t m,
                                                         const int64_t* __restrict__ scalars,
                                                         int64_t* __restrict__ out) {
    int64_t w = 0;
    for (int64_t q = threadIdx.x; q < m; q += blockDim.x) w = max(w, rs[q + 1] - rs[q]);
    w = wave_max(w);
    __shared__ int64_t part[16];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t r = 0;
        for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) r = max(r, part[i]);
        out[0] = rs[m];
        out[1] = scalars[0];
        out[2] = r;
    }
}

static bool rel16_rows(int64_t n_batch, const int64_t* prs_host, int64_t n_queries) {
    if (!prs_host || !O3DML_FRS_REL16) return false;
    if (n_queries > 0x7FFFFFFF / (2 * kRowCap)) return false;  // the rows' buffer resource covers < 2^31 B
    for (int64_t b = 0; b < n_batch; ++b)
        if (prs_host[b + 1] - prs_host[b] > 65536) return false;
    return true;
}

static size_t plan_bytes(int64_t n, int64_t m, int64_t nb) {
    return ws_bytes<int64_t>(4) + ws_bytes<float4>(2 * (n + 1)) + ws_bytes<float4>(m) + 3 * ws_bytes<uint32_t>(m) +
           2 * ws_bytes<uint32_t>(m) + 2 * ws_bytes<uint32_t>(m * kRowCap) +
           ws_bytes<uint32_t>(dir_bins(n, nb) * kDirWords);
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_fixed_radius_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t n_batch) {
    return plan_bytes(n_points, n_queries, n_batch) +
           std::max(prim::scan_workspace_bytes(n_queries), prim::radix_sort_workspace_bytes<uint32_t>(n_queries));
}

namespace o3dml {
// The count phase; totals (nullable, e.g. pinned host memory): [total, rows
// longer than kRowCap] written by the scan's last tile.
static void frs_count_impl(const float* points, int64_t n_points, const float* queries, int64_t n_queries,
                           float radius, int64_t n_batch, const int64_t* points_row_splits,
                           const int64_t* queries_row_splits, const int64_t* points_row_splits_host,
                           const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                           const uint32_t* hash_table_cell_splits, int metric, int ignore_query_point,
                           int self_search, int with_distances, int64_t* neighbors_row_splits, void* workspace,
                           size_t workspace_bytes, hipStream_t st, int64_t* totals) {
    O3DML_REQUIRE(metric >= 0 && metric <= 2, "metric must be L1(0), L2(1) or Linf(2)");
    O3DML_REQUIRE(radius > 0.f, "radius must be > 0");
    O3DML_REQUIRE(n_queries < (int64_t(1) << 31) && n_points < (int64_t(1) << 31), "too many points");
    O3DML_REQUIRE(n_batch >= 1, "need at least one batch item");
    Workspace ws(workspace, workspace_bytes);
    FrsPlan pl = take_plan(ws, n_points, n_queries, n_batch, with_distances != 0);
    if (n_queries == 0 || n_points == 0) {
        fill_async(pl.scalars, 0, sizeof(int64_t) * 4, st);
        fill_async(neighbors_row_splits, 0, sizeof(int64_t) * (n_queries + 1), st);
        if (totals) frs_totals_kernel<<<1, 64, 0, st>>>(neighbors_row_splits, n_queries, pl.scalars, totals);
        return;
    }
    const float thr = metric == kL2 ? radius * radius : radius;
    const float inv = 1.0f / (2.0f * radius);
    const int batch_bits = prim::bits_needed(static_cast<uint64_t>(n_batch - 1));
    const uint32_t* qkeys;
    int bshift;
    const bool self_order = self_search && frs_self_order(n_batch, points_row_splits_host, n_points);
    // large self search: Morton order over the bucket-order points (qsel = positions in pl.pts)
    const bool self_pts = self_search && !self_order && frs_self_pts_order();
    // the points in Open3D bucket order, class sub-lists + directory; for a
    // self search also the query order: Open3D's bucket order with the
    // (voxel, octant) groups made adjacent inside each bucket — no sort of the
    // queries at all.  Also zeroes the plan scalars and neighbors_row_splits[0].
    bucket_classes_kernel<<<static_cast<unsigned>(std::min<int64_t>(ceil_div(n_points, 64 * 4), 1 << 16)), 256, 0,
                            st>>>(points, hash_table_index, pl.pts, n_points, hash_table_cell_splits,
                                  hash_table_splits, (int)n_batch, inv, 2.0f * radius, pl.dir, pl.dir_cap,
                                  self_order ? pl.qorder : nullptr, self_order ? pl.keys : nullptr, pl.scalars, 4,
                                  neighbors_row_splits);
    O3DML_LAUNCH_CHECK();
    if (self_order) {
        qkeys = pl.keys;
        bshift = 0;
    } else {
        // (batch, Morton r-cell) order: <= 24 key bits = 3 radix passes;
        // Morton coordinates wrap modulo 2^cell_bits
        const int cell_bits = std::max(1, std::min(8, (24 - batch_bits) / 3));
        // a self search keys the points in bucket order (positions in pl.pts,
        // the batch items' ranges unchanged); other queries key themselves
        if (self_search && frs_self_pts_order())
            group_query_keys_kernel<true><<<stream_grid(n_queries, 256), 256, 0, st>>>(
                    reinterpret_cast<const float*>(pl.pts), n_queries, 2.0f * inv, (int)n_batch, queries_row_splits,
                    cell_bits, pl.keys);
        else
            group_query_keys_kernel<false><<<stream_grid(n_queries, 256), 256, 0, st>>>(
                    queries, n_queries, 2.0f * inv, (int)n_batch, queries_row_splits, cell_bits, pl.keys);
        O3DML_LAUNCH_CHECK();
        {
            Workspace sws = ws;
            prim::radix_sort_pairs<uint32_t>(pl.keys, nullptr, pl.skeys, pl.qorder, n_queries,
                                             batch_bits + 3 * cell_bits, sws, st);
        }
        if (frs_query_gather() && !self_pts) {
            gather_sorted_points_kernel<<<xcd_grid(n_queries, 256), 256, 0, st>>>(queries, pl.qorder, n_queries,
                                                                                 pl.qpts, 0, nullptr, 0, nullptr);
            O3DML_LAUNCH_CHECK();
        }
        qkeys = pl.skeys;
        bshift = batch_bits == 0 ? 32 : 3 * cell_bits;
    }
    {
        TimedRegion tr("frs_group_search", st);
        const int qlog = frs_qlog(n_queries);
        launch_group<0, int32_t>(metric, ignore_query_point != 0, with_distances != 0,
                                 rel16_rows(n_batch, points_row_splits_host, n_queries), st,
                                 group_grid(n_queries, 1 << qlog), pl.pts,
                                 static_cast<uint32_t>(n_points), hash_table_cell_splits,
                                 self_order || self_pts ? nullptr
                                                        : (frs_query_gather() ? pl.qpts
                                                                              : reinterpret_cast<const float4*>(queries)),
                                 self_order || self_pts || !frs_query_gather() ? pl.qorder : nullptr, qkeys, bshift,
                                 n_queries, nullptr, radius, inv, thr, (int)n_batch, queries_row_splits,
                                 hash_table_splits, points_row_splits, pl.counts, pl.tidx, pl.tdist, pl.over,
                                 pl.scalars, nullptr, nullptr, nullptr, pl.dir, pl.dir_cap, nullptr, -1, qlog);
    }
    Workspace sws = ws;
    prim::scan<uint32_t, int64_t>(pl.counts, neighbors_row_splits + 1, n_queries, true, sws, st, totals,
                                  pl.scalars);
}
}  // namespace o3dml

O3DML_API int o3dml_fixed_radius_search_count(const float* points, int64_t n_points, const float* queries,
                                              int64_t n_queries, float radius, int64_t n_batch,
                                              const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                              const int64_t* points_row_splits_host,
                                              const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                              const uint32_t* hash_table_cell_splits, int metric,
                                              int ignore_query_point, int self_search, int with_distances,
                                              int64_t* neighbors_row_splits, void* workspace,
                                              size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    frs_count_impl(points, n_points, queries, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                   points_row_splits_host, hash_table_splits, hash_table_index, hash_table_cell_splits, metric,
                   ignore_query_point, self_search, with_distances, neighbors_row_splits, workspace,
                   workspace_bytes, as_stream(stream), nullptr);
    O3DML_GUARD_END
}

O3DML_API int o3dml_fixed_radius_search_totals(const int64_t* neighbors_row_splits, int64_t n_queries,
                                               void* workspace, int64_t* totals, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    frs_totals_kernel<<<1, 64, 0, st>>>(neighbors_row_splits, n_queries, static_cast<const int64_t*>(workspace),
                                        totals);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// device int64 [3] = total, rows longer than 64, widest row — for callers
// that read several sizes back in one transfer (KPFCNN collate)
O3DML_API int o3dml_fixed_radius_search_sizes(const int64_t* neighbors_row_splits, int64_t n_queries,
                                              const void* workspace, int64_t* sizes, void* stream) {
    O3DML_GUARD_BEGIN
    frs_sizes_kernel<<<1, 1024, 0, as_stream(stream)>>>(neighbors_row_splits, n_queries,
                                                        static_cast<const int64_t*>(workspace), sizes);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_fixed_radius_search_fill(const float* points, int64_t n_points, const float* queries,
                                             int64_t n_queries, float radius, int64_t n_batch,
                                             const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                             const int64_t* points_row_splits_host,
                                             const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
                                             const uint32_t* hash_table_cell_splits, int metric,
                                             int ignore_query_point, int self_search, int with_distances,
                                             const int64_t* neighbors_row_splits, int index_bits,
                                             void* neighbors_index, float* neighbors_distance, void* workspace,
                                             size_t workspace_bytes, void* stream) {
    return o3dml_fixed_radius_search_fill_bounded(
            points, n_points, queries, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
            points_row_splits_host, hash_table_splits, hash_table_index, hash_table_cell_splits, metric,
            ignore_query_point, self_search, with_distances, neighbors_row_splits, index_bits, neighbors_index,
            neighbors_distance, -1, 3, workspace, workspace_bytes, stream);
}

namespace o3dml {
// The fill phase: CSR rows (dense_w = 0) or a dense int32 [M, dense_w] matrix
// padded with `pad` (neighbors_row_splits then only bounds nothing: capacity -1).
static void frs_fill_impl(const float* queries, int64_t n_points, int64_t n_queries, float radius, int64_t n_batch,
                          const int64_t* points_row_splits, const int64_t* queries_row_splits,
                          const int64_t* points_row_splits_host, const uint32_t* hash_table_splits,
                          const uint32_t* hash_table_cell_splits, int metric, int ignore_query_point,
                          int with_distances, const int64_t* neighbors_row_splits, int index_bits,
                          void* neighbors_index, float* neighbors_distance, int64_t capacity, int parts,
                          int64_t dense_w, int32_t pad, void* workspace, size_t workspace_bytes, hipStream_t st,
                          hipEvent_t fork_at = nullptr) {
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    O3DML_REQUIRE(!with_distances || neighbors_distance, "with_distances needs a distance buffer");
    O3DML_REQUIRE(dense_w == 0 || (index_bits == 32 && !with_distances && capacity < 0),
                  "dense rows are int32 without distances");
    if (n_queries == 0 || n_points == 0) return;
    Workspace ws(workspace, workspace_bytes);
    FrsPlan pl = take_plan(ws, n_points, n_queries, n_batch, with_distances != 0);  // built by _count (same workspace)
    const float thr = metric == kL2 ? radius * radius : radius;
    const float inv = 1.0f / (2.0f * radius);
    int64_t* rs = const_cast<int64_t*>(neighbors_row_splits);
    const bool rel16 = rel16_rows(n_batch, points_row_splits_host, n_queries);
    float* dist = with_distances ? neighbors_distance : nullptr;
    const int dev = stream_device(st);
    DeviceScope dscope(dev);
    FrsSide* side = nullptr;
    std::unique_lock<std::mutex> side_lock;
    if (parts & 2) {  // fork before the row copy is queued: the re-run runs beside it
        side = &frs_side(dev);
        side_lock = std::unique_lock<std::mutex>(side->mu);
        // fork_at: an event the caller just recorded at this point of the
        // stream (one event record fewer between the count and the copy)
        if (!fork_at) O3DML_CHECK_HIP(hipEventRecord(side->fork, st));
    }
    if ((parts & 1) && dense_w > 0) {
        const unsigned gd = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_queries, 4), 1 << 16)));
        if (rel16)
            group_rows_dense_kernel<true><<<gd, 256, 0, st>>>(n_queries, pl.counts, queries_row_splits,
                                                              points_row_splits, (int)n_batch, pl.tidx, dense_w, pad,
                                                              static_cast<int32_t*>(neighbors_index));
        else
            group_rows_dense_kernel<false><<<gd, 256, 0, st>>>(n_queries, pl.counts, queries_row_splits,
                                                               points_row_splits, (int)n_batch, pl.tidx, dense_w, pad,
                                                               static_cast<int32_t*>(neighbors_index));
        O3DML_LAUNCH_CHECK();
    } else if (parts & 1) {
        TimedRegion tr("frs_group_rows", st);
        const unsigned gc = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_queries, 256), 1 << 16)));
#define O3DML_GCOPY3(D, R, T)                                                                                   \
    group_rows_copy_kernel<D, R, T><<<gc, 256, 0, st>>>(n_queries, pl.counts, rs, queries_row_splits,          \
                                                        points_row_splits, (int)n_batch, pl.tidx, pl.tdist,    \
                                                        static_cast<T*>(neighbors_index), dist, capacity)
#define O3DML_GCOPY(T)                                                                                          \
    do {                                                                                                        \
        if (dist) {                                                                                             \
            if (rel16) O3DML_GCOPY3(true, true, T); else O3DML_GCOPY3(true, false, T);                         \
        } else {                                                                                                \
            if (rel16) O3DML_GCOPY3(false, true, T); else O3DML_GCOPY3(false, false, T);                       \
        }                                                                                                       \
    } while (0)
        if (index_bits == 32) O3DML_GCOPY(int32_t); else O3DML_GCOPY(int64_t);
#undef O3DML_GCOPY
#undef O3DML_GCOPY3
        O3DML_LAUNCH_CHECK();
    }
    // rows longer than kRowCap: re-run those queries straight into the final
    // rows; the overflow count stays on the device (no host round trip), so a
    // fixed grid strides over however many there are (usually none)
    if (!(parts & 2)) return;  // the caller read a zero overflow count
    O3DML_CHECK_HIP(hipStreamWaitEvent(side->s, fork_at ? fork_at : side->fork, 0));
    const hipStream_t st_main = st;
    st = side->s;
#ifndef O3DML_FRS_OVER_GRID
#define O3DML_FRS_OVER_GRID 256
#endif
    const unsigned go = static_cast<unsigned>(std::min<int64_t>(n_queries, O3DML_FRS_OVER_GRID));
    const float4* qraw = reinterpret_cast<const float4*>(queries);  // MODE 1 reads [M, 3] via the over list
    if (index_bits == 32)
        launch_group<1, int32_t>(metric, ignore_query_point != 0, dist != nullptr, false, st, go, pl.pts,
                                 static_cast<uint32_t>(n_points), hash_table_cell_splits, qraw, nullptr, nullptr, 32,
                                 0,
                                 pl.scalars, radius, inv, thr, (int)n_batch, queries_row_splits, hash_table_splits,
                                 points_row_splits, nullptr, nullptr, nullptr, pl.over, nullptr, rs,
                                 static_cast<int32_t*>(neighbors_index), dist, pl.dir, pl.dir_cap,
                                 dense_w > 0 ? nullptr : rs + n_queries, capacity, 6, dense_w);
    else
        launch_group<1, int64_t>(metric, ignore_query_point != 0, dist != nullptr, false, st, go, pl.pts,
                                 static_cast<uint32_t>(n_points), hash_table_cell_splits, qraw, nullptr, nullptr, 32,
                                 0,
                                 pl.scalars, radius, inv, thr, (int)n_batch, queries_row_splits, hash_table_splits,
                                 points_row_splits, nullptr, nullptr, nullptr, pl.over, nullptr, rs,
                                 static_cast<int64_t*>(neighbors_index), dist, pl.dir, pl.dir_cap, rs + n_queries,
                                 capacity);
    O3DML_CHECK_HIP(hipEventRecord(side->join, st));
    O3DML_CHECK_HIP(hipStreamWaitEvent(st_main, side->join, 0));
}
}  // namespace o3dml

O3DML_API int o3dml_fixed_radius_search_fill_bounded(
        const float* points, int64_t n_points, const float* queries, int64_t n_queries, float radius,
        int64_t n_batch, const int64_t* points_row_splits, const int64_t* queries_row_splits,
        const int64_t* points_row_splits_host, const uint32_t* hash_table_splits, const uint32_t* hash_table_index,
        const uint32_t* hash_table_cell_splits, int metric, int ignore_query_point, int self_search,
        int with_distances, const int64_t* neighbors_row_splits, int index_bits, void* neighbors_index,
        float* neighbors_distance, int64_t capacity, int parts, void* workspace, size_t workspace_bytes,
        void* stream) {
    O3DML_GUARD_BEGIN
    (void)points;
    (void)hash_table_index;
    (void)self_search;
    frs_fill_impl(queries, n_points, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                  points_row_splits_host, hash_table_splits, hash_table_cell_splits, metric, ignore_query_point,
                  with_distances, neighbors_row_splits, index_bits, neighbors_index, neighbors_distance, capacity,
                  parts, 0, 0, workspace, workspace_bytes, as_stream(stream));
    O3DML_GUARD_END
}

O3DML_API int o3dml_fixed_radius_search_fill_dense(
        const float* queries, int64_t n_points, int64_t n_queries, float radius, int64_t n_batch,
        const int64_t* points_row_splits, const int64_t* queries_row_splits, const int64_t* points_row_splits_host,
        const uint32_t* hash_table_splits, const uint32_t* hash_table_cell_splits, int metric,
        int ignore_query_point, const int64_t* neighbors_row_splits, int64_t width, int32_t pad_value,
        int32_t* neighbors_dense, int parts, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(width >= 1, "dense width must be >= 1 (the widest row)");
    frs_fill_impl(queries, n_points, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                  points_row_splits_host, hash_table_splits, hash_table_cell_splits, metric, ignore_query_point, 0,
                  neighbors_row_splits, 32, neighbors_dense, nullptr, -1, parts, width, pad_value, workspace,
                  workspace_bytes, as_stream(stream));
    O3DML_GUARD_END
}

// ---------------------------------------------------------------------------
// layers.FixedRadiusSearch in one call (the host cost of a small search is
// several Python-side launches otherwise): optional table build into the
// caller's table buffers, count, totals to pinned memory and/or sizes to the
// device, the count-done event, the speculative row copy.
// ---------------------------------------------------------------------------
namespace o3dml {
static size_t layer_search_bytes(int64_t n, int64_t m, int64_t nb, int64_t total_bins) {
    const size_t scratch = std::max(std::max(prim::scan_workspace_bytes(m), prim::radix_sort_workspace_bytes<uint32_t>(m)),
                                    o3dml_build_spatial_hash_table_workspace_size(n, total_bins));
    return plan_bytes(n, m, nb) + scratch;
}
}  // namespace o3dml

O3DML_API size_t o3dml_fixed_radius_search_layer_workspace_size(int64_t n_points, int64_t n_queries,
                                                                int64_t n_batch, int64_t total_bins) {
    return layer_search_bytes(n_points, n_queries, n_batch, total_bins);
}

O3DML_API int o3dml_fixed_radius_search_layer(
        const float* points, int64_t n_points, const float* queries, int64_t n_queries, float radius,
        int64_t n_batch, const int64_t* points_row_splits, const int64_t* queries_row_splits,
        const int64_t* points_row_splits_host, const uint32_t* hash_table_splits,
        const uint32_t* hash_table_splits_host, int64_t total_bins, uint32_t* hash_table_index,
        uint32_t* hash_table_cell_splits, int build_table, int metric, int ignore_query_point, int self_search,
        int with_distances, int64_t* neighbors_row_splits, int64_t* totals, int64_t* sizes, int index_bits,
        void* neighbors_index, float* neighbors_distance, int64_t capacity, int stage, void* count_done,
        void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(stage >= 0 && stage <= 4, "stage must be 0 / 4 (build + count [+ copy]) or fill parts 1..3");
    const size_t need = layer_search_bytes(n_points, n_queries, n_batch, total_bins);
    O3DML_REQUIRE(workspace_bytes >= need, "layer workspace too small");
    hipStream_t st = as_stream(stream);
    if (stage > 0 && stage < 4) {
        frs_fill_impl(queries, n_points, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                      points_row_splits_host, hash_table_splits, hash_table_cell_splits, metric, ignore_query_point,
                      with_distances, neighbors_row_splits, index_bits, neighbors_index, neighbors_distance,
                      capacity, stage, 0, 0, workspace, need, st);
        return 0;
    }
    if (build_table) {  // the table's scratch is the search plan's scratch tail (free until the count)
        const size_t plan = plan_bytes(n_points, n_queries, n_batch);
        const int rc = o3dml_build_spatial_hash_table(points, n_points, radius, n_batch, points_row_splits,
                                                      hash_table_splits, hash_table_splits_host, total_bins,
                                                      hash_table_index, hash_table_cell_splits,
                                                      static_cast<char*>(workspace) + plan, need - plan, stream);
        if (rc) return rc;
    }
    frs_count_impl(points, n_points, queries, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                   points_row_splits_host, hash_table_splits, hash_table_index, hash_table_cell_splits, metric,
                   ignore_query_point, self_search, with_distances, neighbors_row_splits, workspace, need, st, totals);
    if (sizes) {  // [total, rows longer than 64, widest row] on the device
        frs_sizes_kernel<<<1, 1024, 0, st>>>(neighbors_row_splits, n_queries, static_cast<const int64_t*>(workspace),
                                             sizes);
        O3DML_LAUNCH_CHECK();
    }
    // the host waits for the totals only, not for the row copy queued next
    if (count_done) O3DML_CHECK_HIP(hipEventRecord(static_cast<hipEvent_t>(count_done), st));
    // stage 4: the re-run of long rows queued beside the copy as well (it
    // reads the overflow count on the device: nothing to do when it is 0)
    if (capacity >= 0)
        frs_fill_impl(queries, n_points, n_queries, radius, n_batch, points_row_splits, queries_row_splits,
                      points_row_splits_host, hash_table_splits, hash_table_cell_splits, metric, ignore_query_point,
                      with_distances, neighbors_row_splits, index_bits, neighbors_index, neighbors_distance,
                      capacity, stage == 4 ? 3 : 1, 0, 0, workspace, need, st,
                      static_cast<hipEvent_t>(count_done));
    O3DML_GUARD_END
}
