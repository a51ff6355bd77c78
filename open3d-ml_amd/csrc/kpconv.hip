// kpconv.hip — fused KPConv neighbourhood aggregation (SURVEY.md §8a A18;
// ml3d/torch/models/kpconv.py:1005-1159, KPConv.forward).
//
// The reference materialises [n, nb, K, 3] differences, [n, K, nb] influences
// and [n, nb, Cin] gathered features, then  WF = influences @ gathered
// ([n, K, Cin]) and  out = sum_k WF[:, k] @ W[k].  Here one wave owns one
// query: the K x nb influences are computed once into LDS (lane per
// neighbour), then lanes own channels and accumulate the K weighted sums
// while streaming the neighbours' feature rows (coalesced, each row read
// once); WF is written once.  out = WF.view(n, K*Cin) @ W.view(K*Cin, Cout)
// is then a plain dense GEMM (hipBLASLt through torch).
//
// Shadow neighbours (index == n_support, the reference's point at 1e6 with a
// zero feature, kpconv.py:1048, 1139) contribute exactly zero and are skipped.
// Influence: 0 constant, 1 linear max(0, 1 - d/extent), 2 gaussian
// exp(-d^2 / (2 sigma^2)), sigma = 0.3 extent (kpconv.py radius_gaussian);
// closest: only the nearest kernel point of each neighbour contributes.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "primitives.hpp"

namespace o3dml {

constexpr int kKpMaxK = 32;    // kernel points

// gaussian sigma^2 term of the reference's radius_gaussian (kpconv.py:808-818,
// eps 1e-9 in the denominator)
__device__ __forceinline__ float kp_gauss_den(float extent) {
    const float sig = 0.3f * extent;
    return 2.f * (sig * sig) + 1e-9f;
}

// Influences of one neighbour (offset d = p - q) on the K kernel points into
// wrow.  Returns false when DEFORM and no kernel point is within extent: the
// deformable reference drops such neighbours before the influences
// (kpconv.py:1076-1103, the in_range / topk filter), which matters for the
// constant and gaussian influences.
template <int INFL, bool CLOSEST>
__device__ __forceinline__ bool kp_influences(float dx, float dy, float dz, const float* __restrict__ kq, int K,
                                              float extent, bool deform, float* __restrict__ wrow) {
    float best = INFINITY;
    int bk = 0;
    bool in_range = false;
    const float e2 = extent * extent;
#pragma unroll
    for (int k = 0; k < kKpMaxK; ++k) {  // compile-time indices: wrow may live in registers
        if (k >= K) continue;
        const float ex = dx - kq[3 * k], ey = dy - kq[3 * k + 1], ez = dz - kq[3 * k + 2];
        const float d2 = ex * ex + ey * ey + ez * ez;
        in_range = in_range || d2 < e2;
        float v;
        if constexpr (INFL == 0) v = 1.f;
        else if constexpr (INFL == 1) v = fmaxf(1.f - sqrtf(d2) / extent, 0.f);
        else v = __expf(-d2 / kp_gauss_den(extent));
        if (CLOSEST && d2 < best) {
            best = d2;
            bk = k;
        }
        wrow[k] = v;
    }
    if constexpr (CLOSEST) {
#pragma unroll
        for (int k = 0; k < kKpMaxK; ++k)
            if (k < K && k != bk) wrow[k] = 0.f;
    }
    return in_range || !deform;
}

template <int INFL, bool CLOSEST, class TI>
__global__ void __launch_bounds__(256) kpconv_wf_kernel(const float* __restrict__ q_pts, const float* __restrict__ s_pts,
                                                        int64_t n_support, const TI* __restrict__ nbr, int64_t n,
                                                        int nb, const float* __restrict__ x, int cin,
                                                        const float* __restrict__ kp, int K, int kp_per_query,
                                                        float extent, const float* __restrict__ modulations,
                                                        float* __restrict__ wf) {
    __shared__ float w_all[4][64][kKpMaxK + 1];
    __shared__ int32_t id_all[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*w)[kKpMaxK + 1] = w_all[wv];
    int32_t* ids = id_all[wv];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    for (int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + wv; q < n; q += nwaves) {
        const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
        const float* kq = kp + (kp_per_query ? q * K * 3 : 0);
        for (int c0 = 0; c0 < cin; c0 += 64) {
            const int c = c0 + lane;
            float acc[kKpMaxK];
#pragma unroll
            for (int k = 0; k < kKpMaxK; ++k) acc[k] = 0.f;
            for (int j0 = 0; j0 < nb; j0 += 64) {
                // influences of this chunk of neighbours: lane per neighbour
                const int j = j0 + lane;
                int64_t idx = -1;
                if (j < nb) {
                    const int64_t v = static_cast<int64_t>(nbr[q * nb + j]);
                    if (v >= 0 && v < n_support) idx = v;  // shadow neighbours contribute zero
                }
                if (idx >= 0 && !kp_influences<INFL, CLOSEST>(s_pts[3 * idx] - qx, s_pts[3 * idx + 1] - qy,
                                                              s_pts[3 * idx + 2] - qz, kq, K, extent, kp_per_query,
                                                              w[lane]))
                    idx = -1;  // deformable: out of every kernel point's range
                ids[lane] = static_cast<int32_t>(idx);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // lanes own channels: acc[k] += w[j][k] * x[ids[j]][c]
                const int jn = nb - j0 < 64 ? nb - j0 : 64;
                if (c < cin) {
                    for (int jj = 0; jj < jn; ++jj) {
                        const int32_t id = ids[jj];
                        if (id < 0) continue;
                        const float xv = x[static_cast<int64_t>(id) * cin + c];
#pragma unroll
                        for (int k = 0; k < kKpMaxK; ++k)
                            if (k < K) acc[k] = __builtin_fmaf(w[jj][k], xv, acc[k]);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (c < cin) {
                float* o = wf + q * static_cast<int64_t>(K) * cin + c;
#pragma unroll
                for (int k = 0; k < kKpMaxK; ++k)
                    if (k < K) o[static_cast<int64_t>(k) * cin] = modulations ? acc[k] * modulations[q * K + k] : acc[k];
            }
        }
    }
}

// ---- MFMA aggregation (rigid kernel points, K <= 16, no closest mode) ----
// The kernels above give one wave one query and walk its channels 64 at a
// time, re-reading K influences from LDS per (neighbour, channel): the deep
// layers (150 queries x 512 channels at C3 layer 4) fill 38 workgroups of
// the 256 CUs, and layer 0 is LDS-bound.  Here a wave owns one (query,
// 16T-channel tile) — n x ceil(Cin / 16T) waves — and the aggregation is the
// per-query product
//     WF_q [16 kernel points x 16T channels] = A_q [16 x nb] X_q [nb x 16T]
// on v_mfma_f32_16x16x4_f32 (exact f32, cdna_hip_programming.md): lane l
// computes the influence of neighbour 4s + (l >> 4) on kernel point l & 15
// (its A element) and gathers x[nbr][c0 + 16t + (l & 15)] (its B elements,
// 64 contiguous bytes per 16 lanes); the neighbours' relative positions and
// ids are staged 64 at a time in LDS (one coalesced load per lane).  The
// backward scatters dX_q [nb x 16T] = A_q^T dWF_q with the same influences
// (dWF_q read once per wave as the B operand), one fp32 atomic per
// (neighbour, channel) as before.
constexpr int kKpMfmaK = 16;

typedef float kp_f32x4 __attribute__((ext_vector_type(4)));

template <int INFL>
__device__ __forceinline__ float kp_influence(float ex, float ey, float ez, float extent) {
    const float d2 = ex * ex + ey * ey + ez * ez;
    if constexpr (INFL == 0) return 1.f;
    else if constexpr (INFL == 1) return fmaxf(1.f - sqrtf(d2) / extent, 0.f);
    else return __expf(-d2 / kp_gauss_den(extent));
}

// lane l of the wave: neighbour j0 + l of query q -> LDS (p - q, id or -1)
template <class TI>
__device__ __forceinline__ void kp_stage_neighbours(const float* __restrict__ s_pts, int64_t n_support,
                                                    const TI* __restrict__ nbr, int64_t q, int nb, int j0, float qx,
                                                    float qy, float qz, float4* __restrict__ sh) {
    const int lane = threadIdx.x & 63;
    float4 e = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
    if (j0 + lane < nb) {
        const int64_t v = static_cast<int64_t>(nbr[q * nb + j0 + lane]);
        if (v >= 0 && v < n_support)
            e = make_float4(s_pts[3 * v] - qx, s_pts[3 * v + 1] - qy, s_pts[3 * v + 2] - qz,
                            __int_as_float(static_cast<int>(v)));
    }
    sh[lane] = e;
}

__device__ __forceinline__ void kp_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int INFL, int T, class TI>
__global__ void __launch_bounds__(256) kpconv_wf_mfma_kernel(const float* __restrict__ q_pts,
                                                             const float* __restrict__ s_pts, int64_t n_support,
                                                             const TI* __restrict__ nbr, int64_t n, int nb,
                                                             const float* __restrict__ x, int cin,
                                                             const float* __restrict__ kp, int K, float extent,
                                                             int ctiles, float* __restrict__ wf) {
    __shared__ float4 sh_all[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wave = static_cast<int64_t>(blockIdx.x) * 4 + wv;
    if (wave >= n * ctiles) return;  // wave-uniform
    float4* sh = sh_all[wv];
    const int64_t q = wave / ctiles;
    const int c0 = static_cast<int>(wave - q * ctiles) * 16 * T;
    const int kk = lane & 15, jr = lane >> 4;
    const bool kval = kk < K;
    const float kx = kval ? kp[3 * kk] : 0.f, ky = kval ? kp[3 * kk + 1] : 0.f, kz = kval ? kp[3 * kk + 2] : 0.f;
    const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
    kp_f32x4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = kp_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < nb; j0 += 64) {
        kp_wave_sync();
        kp_stage_neighbours(s_pts, n_support, nbr, q, nb, j0, qx, qy, qz, sh);
        kp_wave_sync();
        // groups of 4 steps (16 neighbours; staged entries past nb are id -1)
        const int groups = (min(64, nb - j0) + 15) >> 4;
        for (int gi = 0; gi < groups; ++gi)
#pragma unroll
        for (int st = 4 * gi; st < 4 * gi + 4; ++st) {
            const float4 p = sh[4 * st + jr];
            const int id = __float_as_int(p.w);
            const float a = (id >= 0 && kval) ? kp_influence<INFL>(p.x - kx, p.y - ky, p.z - kz, extent) : 0.f;
            const float* xr = x + static_cast<int64_t>(id) * cin + c0 + kk;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const float b = (id >= 0 && c0 + 16 * t + kk < cin) ? xr[16 * t] : 0.f;
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
            }
        }
    }
    // acc[t][r] = WF[q][k = 4 jr + r][c0 + 16 t + kk]
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int c = c0 + 16 * t + kk;
        if (c >= cin) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * jr + r;
            if (k < K) wf[(q * K + k) * static_cast<int64_t>(cin) + c] = acc[t][r];
        }
    }
}

template <int INFL, int T, class TI>
__global__ void __launch_bounds__(256) kpconv_wf_backward_mfma_kernel(const float* __restrict__ q_pts,
                                                                      const float* __restrict__ s_pts,
                                                                      int64_t n_support, const TI* __restrict__ nbr,
                                                                      int64_t n, int nb,
                                                                      const float* __restrict__ dwf, int cin,
                                                                      const float* __restrict__ kp, int K,
                                                                      float extent, int ctiles,
                                                                      float* __restrict__ dx) {
    __shared__ float4 sh_all[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wave = static_cast<int64_t>(blockIdx.x) * 4 + wv;
    if (wave >= n * ctiles) return;  // wave-uniform
    float4* sh = sh_all[wv];
    const int64_t q = wave / ctiles;
    const int c0 = static_cast<int>(wave - q * ctiles) * 16 * T;
    const int jl = lane & 15, kr = lane >> 4;
    const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
    // B operands: dWF[q][k = 4 s + kr][c0 + 16 t + jl]; this lane's kernel points 4 s + kr
    float gb[4][T], kx[4], ky[4], kz[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int k = 4 * s + kr;
        const bool kv = k < K;
        kx[s] = kv ? kp[3 * k] : 0.f;
        ky[s] = kv ? kp[3 * k + 1] : 0.f;
        kz[s] = kv ? kp[3 * k + 2] : 0.f;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int c = c0 + 16 * t + jl;
            gb[s][t] = (kv && c < cin) ? dwf[(q * K + k) * static_cast<int64_t>(cin) + c] : 0.f;
        }
    }
    for (int j0 = 0; j0 < nb; j0 += 64) {
        kp_wave_sync();
        kp_stage_neighbours(s_pts, n_support, nbr, q, nb, j0, qx, qy, qz, sh);
        kp_wave_sync();
        const int jn = min(64, nb - j0);
        for (int jt = 0; jt < jn; jt += 16) {
            // A operand: influence of kernel point 4 s + kr on neighbour jt + jl
            const float4 p = sh[jt + jl];
            const bool live = __float_as_int(p.w) >= 0;
            kp_f32x4 acc[T];
#pragma unroll
            for (int t = 0; t < T; ++t) acc[t] = kp_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float a = (live && 4 * s + kr < K)
                                        ? kp_influence<INFL>(p.x - kx[s], p.y - ky[s], p.z - kz[s], extent)
                                        : 0.f;
#pragma unroll
                for (int t = 0; t < T; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, gb[s][t], acc[t], 0, 0, 0);
            }
            // acc[t][r] = dX[neighbour jt + 4 kr + r][c0 + 16 t + jl]
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int id = __float_as_int(sh[jt + 4 * kr + r].w);
                if (id < 0) continue;
                float* d = dx + static_cast<int64_t>(id) * cin + c0 + jl;
#pragma unroll
                for (int t = 0; t < T; ++t)
                    if (c0 + 16 * t + jl < cin) atomicAdd(d + 16 * t, acc[t][r]);
            }
        }
    }
}

static bool kp_mfma_enabled() {
    const char* e = std::getenv("O3DML_KPCONV_MFMA");
    return !e || std::atoi(e) != 0;
}

// the MFMA path: rigid shared kernel points, K <= 16, no closest / modulations
template <bool BWD, class TI>
static void launch_kp_mfma(int influence, hipStream_t st, const float* qp, const float* sp, int64_t ns,
                           const void* nbr, int64_t n, int nb, const float* in, int cin, const float* kp, int K,
                           float extent, float* out) {
    const int T = cin <= 16 ? 1 : (cin <= 32 ? 2 : 4);
    const int ctiles = static_cast<int>(ceil_div(cin, 16 * T));
    const unsigned g = static_cast<unsigned>(ceil_div(n * ctiles, 4));
    const TI* nb_ = static_cast<const TI*>(nbr);
#define O3DML_KPM(I, TT)                                                                                           \
    do {                                                                                                           \
        if constexpr (BWD)                                                                                         \
            kpconv_wf_backward_mfma_kernel<I, TT, TI><<<g, 256, 0, st>>>(qp, sp, ns, nb_, n, nb, in, cin, kp, K,   \
                                                                         extent, ctiles, out);                     \
        else                                                                                                       \
            kpconv_wf_mfma_kernel<I, TT, TI><<<g, 256, 0, st>>>(qp, sp, ns, nb_, n, nb, in, cin, kp, K, extent,    \
                                                                ctiles, out);                                      \
    } while (0)
#define O3DML_KPM_T(I)                          \
    do {                                        \
        if (T == 1) O3DML_KPM(I, 1);            \
        else if (T == 2) O3DML_KPM(I, 2);       \
        else O3DML_KPM(I, 4);                   \
    } while (0)
    if (influence == 0) O3DML_KPM_T(0);
    else if (influence == 1) O3DML_KPM_T(1);
    else O3DML_KPM_T(2);
#undef O3DML_KPM_T
#undef O3DML_KPM
    O3DML_LAUNCH_CHECK();
}

// Backward of the aggregation for the features: dx[ids[j]][c] += sum_k
// w[j][k] * dWF[q][k][c] (fp32 atomics; modulations folded into dWF by the
// caller).  Same shape as the forward: one wave per query, the influences of
// 64 neighbours at a time computed lane-per-neighbour into LDS, then lanes own
// channels with the query's K gradient rows held in registers (read once),
// one atomic per (neighbour, channel).  Shadow neighbours are skipped
// wave-uniformly.
template <int INFL, bool CLOSEST, class TI>
__global__ void __launch_bounds__(256) kpconv_wf_backward_kernel(const float* __restrict__ q_pts,
                                                                 const float* __restrict__ s_pts, int64_t n_support,
                                                                 const TI* __restrict__ nbr, int64_t n, int nb,
                                                                 const float* __restrict__ dwf, int cin,
                                                                 const float* __restrict__ kp, int K, int kp_per_query,
                                                                 float extent, float* __restrict__ dx) {
    __shared__ float w_all[4][64][kKpMaxK + 1];
    __shared__ int32_t id_all[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*w)[kKpMaxK + 1] = w_all[wv];
    int32_t* ids = id_all[wv];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    for (int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + wv; q < n; q += nwaves) {
        const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
        const float* kq = kp + (kp_per_query ? q * K * 3 : 0);
        for (int c0 = 0; c0 < cin; c0 += 64) {
            const int c = c0 + lane;
            float gk[kKpMaxK];
            const float* g = dwf + q * static_cast<int64_t>(K) * cin + c;
#pragma unroll
            for (int k = 0; k < kKpMaxK; ++k) gk[k] = (k < K && c < cin) ? g[static_cast<int64_t>(k) * cin] : 0.f;
            for (int j0 = 0; j0 < nb; j0 += 64) {
                const int j = j0 + lane;
                int64_t idx = -1;
                if (j < nb) {
                    const int64_t v = static_cast<int64_t>(nbr[q * nb + j]);
                    if (v >= 0 && v < n_support) idx = v;
                }
                if (idx >= 0 && !kp_influences<INFL, CLOSEST>(s_pts[3 * idx] - qx, s_pts[3 * idx + 1] - qy,
                                                              s_pts[3 * idx + 2] - qz, kq, K, extent, kp_per_query,
                                                              w[lane]))
                    idx = -1;
                ids[lane] = static_cast<int32_t>(idx);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int jn = nb - j0 < 64 ? nb - j0 : 64;
                if (c < cin) {
                    for (int jj = 0; jj < jn; ++jj) {
                        const int32_t id = ids[jj];
                        if (id < 0) continue;
                        float sum = 0.f;
#pragma unroll
                        for (int k = 0; k < kKpMaxK; ++k)
                            if (k < K) sum = __builtin_fmaf(w[jj][k], gk[k], sum);
                        atomicAdd(dx + static_cast<int64_t>(id) * cin + c, sum);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
}

// Gradient w.r.t. per-query (deformed) kernel points and modulations
// (deformable KPConv training, kpconv.py:1005-1159): with A[j][k] =
// dWF[q][k][:] . x[j][:] (dWF before the modulation),
//   dkp[q][k] = m[q][k] * sum_j A[j][k] * dw(j,k)/dkp,
//   dm[q][k]  = sum_j A[j][k] * w(j,k),
// dw/dkp = diff / (extent * |diff|) (linear, inside the support),
// w * diff / sigma'^2 (gaussian, sigma'^2 = den / 2), 0 (constant), diff =
// (p_j - q) - kp_k; closest mode: only each neighbour's nearest kernel point.
// One wave per query: lanes = neighbours (64 at a time); the query's dWF rows
// staged per 64-channel block in LDS and read as broadcasts, each lane
// streaming its neighbour's feature row; sums over neighbours by DPP.
template <int INFL, bool CLOSEST, class TI>
__global__ void __launch_bounds__(256) kpconv_kp_grad_kernel(const float* __restrict__ q_pts,
                                                             const float* __restrict__ s_pts, int64_t n_support,
                                                             const TI* __restrict__ nbr, int64_t n, int nb,
                                                             const float* __restrict__ x, int cin,
                                                             const float* __restrict__ dwf,
                                                             const float* __restrict__ kp, int K, float extent,
                                                             const float* __restrict__ modulations,
                                                             float* __restrict__ dkp, float* __restrict__ dmod) {
    __shared__ float g_all[4][kKpMaxK][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*G)[64] = g_all[wv];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    for (int64_t q = static_cast<int64_t>(blockIdx.x) * 4 + wv; q < n; q += nwaves) {
        const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
        const float* kq = kp + q * K * 3;
        float gk[kKpMaxK][3], gm[kKpMaxK];
#pragma unroll
        for (int k = 0; k < kKpMaxK; ++k) gk[k][0] = gk[k][1] = gk[k][2] = gm[k] = 0.f;
        for (int j0 = 0; j0 < nb; j0 += 64) {
            const int j = j0 + lane;
            int64_t idx = -1;
            if (j < nb) {
                const int64_t v = static_cast<int64_t>(nbr[q * nb + j]);
                if (v >= 0 && v < n_support) idx = v;
            }
            float px = 0.f, py = 0.f, pz = 0.f, w[kKpMaxK];
            if (idx >= 0) {
                px = s_pts[3 * idx] - qx;
                py = s_pts[3 * idx + 1] - qy;
                pz = s_pts[3 * idx + 2] - qz;
                if (!kp_influences<INFL, CLOSEST>(px, py, pz, kq, K, extent, true, w)) idx = -1;
            }
            // A[j][k] = dWF[q][k][:] . x[j][:]
            float a[kKpMaxK];
#pragma unroll
            for (int k = 0; k < kKpMaxK; ++k) a[k] = 0.f;
            for (int c0 = 0; c0 < cin; c0 += 64) {
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < kKpMaxK; ++k)
                    if (k < K) G[k][lane] = c0 + lane < cin ? dwf[(q * K + k) * cin + c0 + lane] : 0.f;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (idx >= 0) {
                    const float* xr = x + idx * cin;
                    const int cn = min(64, cin - c0);
                    for (int cc = 0; cc < cn; ++cc) {
                        const float xv = xr[c0 + cc];
#pragma unroll
                        for (int k = 0; k < kKpMaxK; ++k)
                            if (k < K) a[k] = __builtin_fmaf(G[k][cc], xv, a[k]);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (idx >= 0) {
#pragma unroll
                for (int k = 0; k < kKpMaxK; ++k) {
                    if (k >= K) continue;
                    gm[k] = __builtin_fmaf(a[k], w[k], gm[k]);
                    if constexpr (INFL == 0) continue;
                    if (CLOSEST && w[k] == 0.f) continue;  // not this neighbour's closest kernel point
                    const float ex = px - kq[3 * k], ey = py - kq[3 * k + 1], ez = pz - kq[3 * k + 2];
                    float f;
                    if constexpr (INFL == 1) {
                        const float d = sqrtf(ex * ex + ey * ey + ez * ez);
                        f = (d > 0.f && d < extent) ? a[k] / (extent * d) : 0.f;
                    } else {
                        f = a[k] * w[k] * 2.f / kp_gauss_den(extent);
                    }
                    gk[k][0] = __builtin_fmaf(f, ex, gk[k][0]);
                    gk[k][1] = __builtin_fmaf(f, ey, gk[k][1]);
                    gk[k][2] = __builtin_fmaf(f, ez, gk[k][2]);
                }
            }
        }
        // sums over the 64 lanes (neighbours)
#pragma unroll
        for (int k = 0; k < kKpMaxK; ++k) {
            if (k >= K) continue;
            float v0 = gk[k][0], v1 = gk[k][1], v2 = gk[k][2], v3 = gm[k];
            for (int o = 32; o >= 1; o >>= 1) {
                v0 += __shfl_xor(v0, o, 64);
                v1 += __shfl_xor(v1, o, 64);
                v2 += __shfl_xor(v2, o, 64);
                v3 += __shfl_xor(v3, o, 64);
            }
            if (lane == 0) {
                const float m = modulations ? modulations[q * K + k] : 1.f;
                dkp[(q * K + k) * 3] = m * v0;
                dkp[(q * K + k) * 3 + 1] = m * v1;
                dkp[(q * K + k) * 3 + 2] = m * v2;
                if (dmod) dmod[q * K + k] = v3;
            }
        }
    }
}

// min_d2 of the deformable reference (kpconv.py:1071): for every (query,
// kernel point) the neighbour column with the smallest squared distance to
// the kernel point, shadow neighbours at (1e6, 1e6, 1e6) included; the first
// minimum wins.  The caller recomputes the distance from that column with
// torch ops, so the fitting loss differentiates into the kernel points.
template <class TI>
__global__ void kpconv_min_d2_kernel(const float* __restrict__ q_pts, const float* __restrict__ s_pts,
                                     int64_t n_support, const TI* __restrict__ nbr, int64_t n, int nb,
                                     const float* __restrict__ kp, int K, int32_t* __restrict__ col) {
    const int64_t total = n * K;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = e / K;
        const float kx = kp[3 * e], ky = kp[3 * e + 1], kz = kp[3 * e + 2];
        const float qx = q_pts[3 * q], qy = q_pts[3 * q + 1], qz = q_pts[3 * q + 2];
        float best = INFINITY;
        int bj = 0;
        for (int j = 0; j < nb; ++j) {
            const int64_t v = static_cast<int64_t>(nbr[q * nb + j]);
            const bool real = v >= 0 && v < n_support;
            const float px = (real ? s_pts[3 * v] : 1e6f) - qx, py = (real ? s_pts[3 * v + 1] : 1e6f) - qy,
                        pz = (real ? s_pts[3 * v + 2] : 1e6f) - qz;
            const float ex = px - kx, ey = py - ky, ez = pz - kz;
            const float d2 = ex * ex + ey * ey + ez * ez;
            if (d2 < best) {
                best = d2;
                bj = j;
            }
        }
        col[e] = bj;
    }
}

// KPFCNN pooling (kpconv.py:821-858): out[q, c] = max over the first nb
// columns j of row q of x_pad[inds[q, j], c], where x_pad is x with one zero
// row appended (index n_support = shadow).  closest_pool is nb = 1 (column 0
// only).  argmax[q, c] keeps the winning support index (n_support = the
// shadow row) for the backward; the first maximum wins.  Lanes own channels,
// so each gathered row is a coalesced read.
template <class TI>
__global__ void __launch_bounds__(256) pool_max_kernel(const float* __restrict__ x, int64_t n_support, int c,
                                                       const TI* __restrict__ inds, int64_t ld, int64_t n, int nb,
                                                       float* __restrict__ out, int32_t* __restrict__ argmax) {
    const int64_t total = n * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = e / c;
        const int ch = static_cast<int>(e - q * c);
        const TI* row = inds + q * ld;
        float best = -INFINITY;
        int64_t arg = n_support;
        for (int j = 0; j < nb; ++j) {
            int64_t id = static_cast<int64_t>(row[j]);
            if (id < 0 || id > n_support) id = n_support;
            const float v = id < n_support ? x[id * c + ch] : 0.f;
            if (v > best) {
                best = v;
                arg = id;
            }
        }
        if (nb == 0) best = 0.f;
        out[e] = best;
        if (argmax) argmax[e] = static_cast<int32_t>(arg);
    }
}

__global__ void __launch_bounds__(256) pool_max_backward_kernel(const float* __restrict__ g,
                                                                const int32_t* __restrict__ argmax, int64_t n, int c,
                                                                int64_t n_support, float* __restrict__ dx) {
    const int64_t total = n * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t a = argmax[e];
        if (a >= 0 && a < n_support) atomicAdd(dx + a * c + (e % c), g[e]);
    }
}

// ---- deterministic backward (torch.use_deterministic_algorithms(True)) ----
// The two scatter-adds above (fp32 atomics, summation order = scheduling
// order) become fixed-order gathers: the pairs p = q * nb + j of the
// neighbour matrix are radix-sorted (stably) by support index
// (prim::build_inverse), and one wave per support sums its pairs in
// ascending p.  Bitwise identical run to run; extra cost: the sort and, in
// the feature gradient, re-reading dWF[q] per pair (only the kernel points
// with non-zero influence).
template <class TI>
__global__ void kp_pair_keys_kernel(const TI* __restrict__ nbr, int64_t ld, int64_t n, int nb, int64_t n_support,
                                    uint32_t* __restrict__ keys) {
    const int64_t total = n * nb;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = e / nb;
        const int64_t v = static_cast<int64_t>(nbr[q * ld + (e - q * nb)]);
        keys[e] = static_cast<uint32_t>(v >= 0 && v < n_support ? v : n_support);
    }
}

template <class TI>
static prim::Inverse kp_inverse(const void* nbr, int64_t ld, int64_t n, int nb, int64_t n_support, Workspace& ws,
                                hipStream_t st) {
    uint32_t* keys = ws.take<uint32_t>(n * nb);
    kp_pair_keys_kernel<TI><<<stream_grid(n * nb, 256), 256, 0, st>>>(static_cast<const TI*>(nbr), ld, n, nb,
                                                                      n_support, keys);
    O3DML_LAUNCH_CHECK();
    return prim::build_inverse(keys, n * nb, n_support, ws, st);
}

template <int INFL, bool CLOSEST>
__global__ void __launch_bounds__(256) kpconv_wf_backward_det_kernel(
        const float* __restrict__ q_pts, const float* __restrict__ s_pts, int64_t n_support,
        const uint32_t* __restrict__ pairs, const int64_t* __restrict__ off, int nb, const float* __restrict__ dwf,
        int cin, const float* __restrict__ kp, int K, int kp_per_query, float extent, float* __restrict__ dx) {
    __shared__ float w_all[4][64][kKpMaxK + 1];
    __shared__ int32_t q_all[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*w)[kKpMaxK + 1] = w_all[wv];
    int32_t* qs = q_all[wv];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    for (int64_t s = static_cast<int64_t>(blockIdx.x) * 4 + wv; s < n_support; s += nwaves) {
        const float sx = s_pts[3 * s], sy = s_pts[3 * s + 1], sz = s_pts[3 * s + 2];
        const int64_t beg = off[s], end = off[s + 1];
        for (int c0 = 0; c0 < cin; c0 += 64) {
            const int c = c0 + lane;
            float acc = 0.f;
            for (int64_t p0 = beg; p0 < end; p0 += 64) {
                const int64_t p = p0 + lane;
                int32_t q = -1;
                if (p < end) {
                    q = static_cast<int32_t>(pairs[p] / static_cast<uint32_t>(nb));
                    const float* kq = kp + (kp_per_query ? static_cast<int64_t>(q) * K * 3 : 0);
                    if (!kp_influences<INFL, CLOSEST>(sx - q_pts[3 * q], sy - q_pts[3 * q + 1], sz - q_pts[3 * q + 2],
                                                      kq, K, extent, kp_per_query, w[lane]))
                        q = -1;
                }
                qs[lane] = q;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int jn = end - p0 < 64 ? static_cast<int>(end - p0) : 64;
                if (c < cin) {
                    for (int jj = 0; jj < jn; ++jj) {
                        const int32_t qq = qs[jj];
                        if (qq < 0) continue;
                        const float* g = dwf + static_cast<int64_t>(qq) * K * cin + c;
                        for (int k = 0; k < K; ++k) {
                            const float wk = w[jj][k];
                            if (wk != 0.f) acc = __builtin_fmaf(wk, g[static_cast<int64_t>(k) * cin], acc);
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (c < cin) dx[s * cin + c] = acc;
        }
    }
}

// dx[s, ch] = sum over the queries q whose pooled row holds s (each q once,
// ascending) with argmax[q, ch] == s of g[q, ch]
__global__ void __launch_bounds__(256) pool_max_backward_det_kernel(const float* __restrict__ g,
                                                                    const int32_t* __restrict__ argmax,
                                                                    const uint32_t* __restrict__ pairs,
                                                                    const int64_t* __restrict__ off, int nb, int c,
                                                                    int64_t n_support, float* __restrict__ dx) {
    const int64_t total = n_support * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t s = e / c;
        const int ch = static_cast<int>(e - s * c);
        float acc = 0.f;
        int64_t prev = -1;
        for (int64_t p = off[s]; p < off[s + 1]; ++p) {
            const int64_t q = pairs[p] / static_cast<uint32_t>(nb);
            if (q == prev) continue;  // s repeated in row q: one argmax entry
            prev = q;
            if (argmax[q * c + ch] == s) acc += g[q * c + ch];
        }
        dx[e] = acc;
    }
}

template <bool BWD, class TI>
static void launch_kp(int influence, int closest, unsigned g, hipStream_t st, const float* qp, const float* sp,
                      int64_t ns, const void* nbr, int64_t n, int nb, const float* in, int cin, const float* kp, int K,
                      int kpq, float extent, const float* mod, float* out) {
#define O3DML_KP(I, C)                                                                                            \
    do {                                                                                                          \
        if constexpr (BWD)                                                                                        \
            kpconv_wf_backward_kernel<I, C, TI><<<g, 256, 0, st>>>(qp, sp, ns, static_cast<const TI*>(nbr), n, nb, \
                                                                   in, cin, kp, K, kpq, extent, out);             \
        else                                                                                                      \
            kpconv_wf_kernel<I, C, TI><<<g, 256, 0, st>>>(qp, sp, ns, static_cast<const TI*>(nbr), n, nb, in, cin, \
                                                          kp, K, kpq, extent, mod, out);                          \
    } while (0)
    if (influence == 0) {
        if (closest) O3DML_KP(0, true); else O3DML_KP(0, false);
    } else if (influence == 1) {
        if (closest) O3DML_KP(1, true); else O3DML_KP(1, false);
    } else {
        if (closest) O3DML_KP(2, true); else O3DML_KP(2, false);
    }
#undef O3DML_KP
    O3DML_LAUNCH_CHECK();
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int o3dml_kpconv_weighted_features(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                             const void* neighbors, int index_bits, int nb, const float* features,
                                             int cin, const float* kernel_points, int K, int kp_per_query,
                                             float extent, int influence, int closest, const float* modulations,
                                             float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= kKpMaxK, "KPConv: kernel points must be in [1, %d]", kKpMaxK);
    O3DML_REQUIRE(nb >= 0, "KPConv: negative neighbour count");
    O3DML_REQUIRE(influence >= 0 && influence <= 2, "KPConv: influence must be constant, linear or gaussian");
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n == 0) return 0;
    if (!closest && !kp_per_query && !modulations && K <= kKpMfmaK && kp_mfma_enabled()) {
        if (index_bits == 32)
            launch_kp_mfma<false, int32_t>(influence, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                           features, cin, kernel_points, K, extent, out);
        else
            launch_kp_mfma<false, int64_t>(influence, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                           features, cin, kernel_points, K, extent, out);
        return 0;
    }
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n, 4), 1 << 20));
    if (index_bits == 32)
        launch_kp<false, int32_t>(influence, closest, g, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                  features, cin, kernel_points, K, kp_per_query, extent, modulations, out);
    else
        launch_kp<false, int64_t>(influence, closest, g, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                  features, cin, kernel_points, K, kp_per_query, extent, modulations, out);
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_weighted_features_backward(const float* q_pts, int64_t n, const float* s_pts,
                                                      int64_t n_support, const void* neighbors, int index_bits, int nb,
                                                      const float* grad_wf, int cin, const float* kernel_points, int K,
                                                      int kp_per_query, float extent, int influence, int closest,
                                                      float* grad_features, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= kKpMaxK, "KPConv: kernel points must be in [1, %d]", kKpMaxK);
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n == 0) return 0;
    if (!closest && !kp_per_query && K <= kKpMfmaK && kp_mfma_enabled()) {
        if (index_bits == 32)
            launch_kp_mfma<true, int32_t>(influence, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                          grad_wf, cin, kernel_points, K, extent, grad_features);
        else
            launch_kp_mfma<true, int64_t>(influence, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                          grad_wf, cin, kernel_points, K, extent, grad_features);
        return 0;
    }
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n, 4), 1 << 20));
    if (index_bits == 32)
        launch_kp<true, int32_t>(influence, closest, g, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                 grad_wf, cin, kernel_points, K, kp_per_query, extent, nullptr, grad_features);
    else
        launch_kp<true, int64_t>(influence, closest, g, as_stream(stream), q_pts, s_pts, n_support, neighbors, n, nb,
                                 grad_wf, cin, kernel_points, K, kp_per_query, extent, nullptr, grad_features);
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_kpconv_inverse_workspace_size(int64_t n, int nb, int64_t n_support) {
    return prim::inverse_workspace_bytes(n * (nb > 0 ? nb : 0), n_support);
}

O3DML_API int o3dml_kpconv_weighted_features_backward_det(const float* q_pts, int64_t n, const float* s_pts,
                                                          int64_t n_support, const void* neighbors, int index_bits,
                                                          int nb, const float* grad_wf, int cin,
                                                          const float* kernel_points, int K, int kp_per_query,
                                                          float extent, int influence, int closest,
                                                          float* grad_features, void* workspace,
                                                          size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= kKpMaxK, "KPConv: kernel points must be in [1, %d]", kKpMaxK);
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    O3DML_REQUIRE(nb >= 0, "KPConv: negative neighbour count");
    if (n_support == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const prim::Inverse inv = index_bits == 32 ? kp_inverse<int32_t>(neighbors, nb, n, nb, n_support, ws, st)
                                               : kp_inverse<int64_t>(neighbors, nb, n, nb, n_support, ws, st);
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_support, 4), 1 << 20));
#define O3DML_KPD(I, C)                                                                                         \
    kpconv_wf_backward_det_kernel<I, C><<<g, 256, 0, st>>>(q_pts, s_pts, n_support, inv.pairs, inv.off, nb,     \
                                                           grad_wf, cin, kernel_points, K, kp_per_query, extent, \
                                                           grad_features)
    if (influence == 0) {
        if (closest) O3DML_KPD(0, true); else O3DML_KPD(0, false);
    } else if (influence == 1) {
        if (closest) O3DML_KPD(1, true); else O3DML_KPD(1, false);
    } else {
        if (closest) O3DML_KPD(2, true); else O3DML_KPD(2, false);
    }
#undef O3DML_KPD
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_kernel_point_grad(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                             const void* neighbors, int index_bits, int nb, const float* features,
                                             int cin, const float* grad_wf, const float* kernel_points, int K,
                                             float extent, int influence, int closest, const float* modulations,
                                             float* grad_kp, float* grad_mod, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(K >= 1 && K <= kKpMaxK, "KPConv: kernel points must be in [1, %d]", kKpMaxK);
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    O3DML_REQUIRE(influence >= 0 && influence <= 2, "KPConv: influence must be constant, linear or gaussian");
    if (n == 0) return 0;
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n, 4), 1 << 20));
    hipStream_t st = as_stream(stream);
#define O3DML_KPG(I, C, T)                                                                                       \
    kpconv_kp_grad_kernel<I, C, T><<<g, 256, 0, st>>>(q_pts, s_pts, n_support, static_cast<const T*>(neighbors), \
                                                      n, nb, features, cin, grad_wf, kernel_points, K, extent,   \
                                                      modulations, grad_kp, grad_mod)
#define O3DML_KPG_T(I, C)                                        \
    do {                                                         \
        if (index_bits == 32) O3DML_KPG(I, C, int32_t);          \
        else O3DML_KPG(I, C, int64_t);                           \
    } while (0)
    if (influence == 0) {
        if (closest) O3DML_KPG_T(0, true); else O3DML_KPG_T(0, false);
    } else if (influence == 1) {
        if (closest) O3DML_KPG_T(1, true); else O3DML_KPG_T(1, false);
    } else {
        if (closest) O3DML_KPG_T(2, true); else O3DML_KPG_T(2, false);
    }
#undef O3DML_KPG_T
#undef O3DML_KPG
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_min_d2_columns(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                          const void* neighbors, int index_bits, int nb, const float* kernel_points,
                                          int K, int32_t* columns, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n == 0) return 0;
    const unsigned g = stream_grid(n * K, 256);
    if (index_bits == 32)
        kpconv_min_d2_kernel<int32_t><<<g, 256, 0, as_stream(stream)>>>(
                q_pts, s_pts, n_support, static_cast<const int32_t*>(neighbors), n, nb, kernel_points, K, columns);
    else
        kpconv_min_d2_kernel<int64_t><<<g, 256, 0, as_stream(stream)>>>(
                q_pts, s_pts, n_support, static_cast<const int64_t*>(neighbors), n, nb, kernel_points, K, columns);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_pool_max(const float* x, int64_t n_support, int c, const void* inds, int index_bits,
                                    int64_t ld, int64_t n, int nb, float* out, int32_t* argmax, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(c > 0, "pool: channels must be > 0");
    O3DML_REQUIRE(nb >= 0 && nb <= ld, "pool: columns (%d) must be in [0, row stride %lld]", nb, (long long)ld);
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n == 0) return 0;
    const unsigned g = stream_grid(n * c, 256, 256 * 16);
    if (index_bits == 32)
        pool_max_kernel<int32_t><<<g, 256, 0, as_stream(stream)>>>(x, n_support, c, static_cast<const int32_t*>(inds),
                                                                   ld, n, nb, out, argmax);
    else
        pool_max_kernel<int64_t><<<g, 256, 0, as_stream(stream)>>>(x, n_support, c, static_cast<const int64_t*>(inds),
                                                                   ld, n, nb, out, argmax);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_pool_max_backward(const float* grad_out, const int32_t* argmax, int64_t n, int c,
                                             int64_t n_support, float* grad_x, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(c > 0, "pool: channels must be > 0");
    if (n == 0) return 0;
    pool_max_backward_kernel<<<stream_grid(n * c, 256, 256 * 16), 256, 0, as_stream(stream)>>>(grad_out, argmax, n, c,
                                                                                            n_support, grad_x);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_kpconv_pool_max_backward_det(const float* grad_out, const int32_t* argmax, const void* inds,
                                                 int index_bits, int64_t ld, int64_t n, int nb, int c,
                                                 int64_t n_support, float* grad_x, void* workspace,
                                                 size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(c > 0, "pool: channels must be > 0");
    O3DML_REQUIRE(nb >= 0 && nb <= ld, "pool: columns (%d) must be in [0, row stride %lld]", nb, (long long)ld);
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n_support == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const prim::Inverse inv = index_bits == 32 ? kp_inverse<int32_t>(inds, ld, n, nb, n_support, ws, st)
                                               : kp_inverse<int64_t>(inds, ld, n, nb, n_support, ws, st);
    pool_max_backward_det_kernel<<<stream_grid(n_support * c, 256, 256 * 16), 256, 0, st>>>(
            grad_out, argmax, inv.pairs, inv.off, nb > 0 ? nb : 1, c, n_support, grad_x);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
