// pointnet2.hip — PointNet++ ops, replacing
// open3d.ml.torch.ops.{furthest_point_sampling, ball_query, three_nn,
// three_interpolate, three_interpolate_grad} as bound by
// ml3d/torch/utils/pointnet/pointnet2_utils.py:33-36 (FPS :55,94; three_nn
// :129; three_interpolate :162; grad :184; ball_query :212) and
// point_transformer.py:518.
//
// FPS is inherently sequential: one 1024-lane workgroup per cloud keeps its
// points AND their running min-distances in registers (ITEMS per lane), so an
// iteration touches no memory except the winner's coordinates; the argmax is a
// wave shuffle tree + one LDS exchange (ties -> smallest index).
// ball_query / three_nn stream the support cloud through LDS tiles shared by
// the 256 queries of a workgroup.
#include "common.hpp"
#include "primitives.hpp"

namespace o3dml {

constexpr int kFpsThreads = 1024;

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

template <int ITEMS>
__global__ void __launch_bounds__(kFpsThreads) fps_kernel(const float* __restrict__ xyz, int n, int m,
                                                          int32_t* __restrict__ out) {
    const int b = blockIdx.x;
    const float* p = xyz + static_cast<int64_t>(b) * n * 3;
    int32_t* o = out + static_cast<int64_t>(b) * m;
    const int t = threadIdx.x;
    float px[ITEMS], py[ITEMS], pz[ITEMS], md[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const int k = t + r * kFpsThreads;
        const bool ok = k < n;
        px[r] = ok ? p[3 * k] : 0.f;
        py[r] = ok ? p[3 * k + 1] : 0.f;
        pz[r] = ok ? p[3 * k + 2] : 0.f;
        md[r] = ok ? 1e10f : -1.f;
    }
    __shared__ float sv[kFpsThreads / 64];
    __shared__ int si[kFpsThreads / 64];
    __shared__ int s_old;
    if (m <= 0) return;
    int old = 0;
    if (t == 0) o[0] = 0;
    for (int j = 1; j < m; ++j) {
        const float x1 = p[3 * old], y1 = p[3 * old + 1], z1 = p[3 * old + 2];
        float best = -1.f;
        int besti = 0;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const int k = t + r * kFpsThreads;
            const float d = dist_l2(px[r], py[r], pz[r], x1, y1, z1);
            const float d2 = d < md[r] ? d : md[r];
            if (k < n) md[r] = d2;
            if (k < n && d2 > best) {
                best = d2;
                besti = k;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float v2 = __shfl_xor(best, off, 64);
            const int i2 = __shfl_xor(besti, off, 64);
            argmax_merge(best, besti, v2, i2);
        }
        if (lane_id() == 0) {
            sv[wave_id()] = best;
            si[wave_id()] = besti;
        }
        __syncthreads();
        if (t < 64) {
            float v = t < kFpsThreads / 64 ? sv[t] : -2.f;
            int i = t < kFpsThreads / 64 ? si[t] : 0x7fffffff;
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1) {
                const float v2 = __shfl_xor(v, off, 64);
                const int i2 = __shfl_xor(i, off, 64);
                argmax_merge(v, i, v2, i2);
            }
            if (t == 0) {
                s_old = i;
                o[j] = i;
            }
        }
        __syncthreads();
        old = s_old;
    }
}

// Fallback for very large clouds: min-distances in global memory.
__global__ void __launch_bounds__(kFpsThreads) fps_global_kernel(const float* __restrict__ xyz, int n, int m,
                                                                 float* __restrict__ temp, int32_t* __restrict__ out) {
    const int b = blockIdx.x;
    const float* p = xyz + static_cast<int64_t>(b) * n * 3;
    float* md = temp + static_cast<int64_t>(b) * n;
    int32_t* o = out + static_cast<int64_t>(b) * m;
    const int t = threadIdx.x;
    __shared__ float sv[kFpsThreads / 64];
    __shared__ int si[kFpsThreads / 64];
    __shared__ int s_old;
    for (int k = t; k < n; k += kFpsThreads) md[k] = 1e10f;
    if (m <= 0) return;
    int old = 0;
    if (t == 0) o[0] = 0;
    __syncthreads();
    for (int j = 1; j < m; ++j) {
        const float x1 = p[3 * old], y1 = p[3 * old + 1], z1 = p[3 * old + 2];
        float best = -1.f;
        int besti = 0;
        for (int k = t; k < n; k += kFpsThreads) {
            const float d = dist_l2(p[3 * k], p[3 * k + 1], p[3 * k + 2], x1, y1, z1);
            const float d2 = d < md[k] ? d : md[k];
            md[k] = d2;
            if (d2 > best) {
                best = d2;
                besti = k;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float v2 = __shfl_xor(best, off, 64);
            const int i2 = __shfl_xor(besti, off, 64);
            argmax_merge(best, besti, v2, i2);
        }
        if (lane_id() == 0) {
            sv[wave_id()] = best;
            si[wave_id()] = besti;
        }
        __syncthreads();
        if (t < 64) {
            float v = t < kFpsThreads / 64 ? sv[t] : -2.f;
            int i = t < kFpsThreads / 64 ? si[t] : 0x7fffffff;
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1) {
                const float v2 = __shfl_xor(v, off, 64);
                const int i2 = __shfl_xor(i, off, 64);
                argmax_merge(v, i, v2, i2);
            }
            if (t == 0) {
                s_old = i;
                o[j] = i;
            }
        }
        __syncthreads();
        old = s_old;
    }
}

constexpr int kTile = 256;

// ball_query: first nsample points (index order) with d2 < r2; pad with the
// first hit; 0 when none.
__global__ void __launch_bounds__(kTile) ball_query_kernel(const float* __restrict__ xyz, const float* __restrict__ ctr,
                                                           int n, int m, float r2, int nsample,
                                                           int32_t* __restrict__ out) {
    const int b = blockIdx.y;
    const int j = blockIdx.x * kTile + threadIdx.x;
    const float* p = xyz + static_cast<int64_t>(b) * n * 3;
    __shared__ float tx[kTile], ty[kTile], tz[kTile];
    const bool active = j < m;
    float cx = 0.f, cy = 0.f, cz = 0.f;
    int32_t* o = out + (static_cast<int64_t>(b) * m + (active ? j : 0)) * nsample;
    if (active) {
        const float* c = ctr + (static_cast<int64_t>(b) * m + j) * 3;
        cx = c[0];
        cy = c[1];
        cz = c[2];
    }
    int cnt = 0;
    for (int base = 0; base < n; base += kTile) {
        if (__syncthreads_and(!active || cnt >= nsample)) break;
        const int k = base + threadIdx.x;
        if (k < n) {
            tx[threadIdx.x] = p[3 * k];
            ty[threadIdx.x] = p[3 * k + 1];
            tz[threadIdx.x] = p[3 * k + 2];
        }
        __syncthreads();
        const int lim = min(kTile, n - base);
        if (active) {
            for (int kk = 0; kk < lim && cnt < nsample; ++kk) {
                const float d2 = dist_l2(tx[kk], ty[kk], tz[kk], cx, cy, cz);
                if (d2 < r2) {
                    if (cnt == 0)
                        for (int l = 0; l < nsample; ++l) o[l] = base + kk;
                    o[cnt++] = base + kk;
                }
            }
        }
        __syncthreads();
    }
    if (active && cnt == 0)
        for (int l = 0; l < nsample; ++l) o[l] = 0;
}

// three_nn: 3 smallest (d2, index) with strict-< insertion in index order.
__global__ void __launch_bounds__(kTile) three_nn_kernel(const float* __restrict__ unknown, const float* __restrict__ known,
                                                         int n, int m, float* __restrict__ dist2,
                                                         int32_t* __restrict__ idx) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * kTile + threadIdx.x;
    const float* kp = known + static_cast<int64_t>(b) * m * 3;
    __shared__ float tx[kTile], ty[kTile], tz[kTile];
    const bool active = i < n;
    float ux = 0.f, uy = 0.f, uz = 0.f;
    if (active) {
        const float* u = unknown + (static_cast<int64_t>(b) * n + i) * 3;
        ux = u[0];
        uy = u[1];
        uz = u[2];
    }
    float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
    int i1 = 0, i2 = 0, i3 = 0;
    for (int base = 0; base < m; base += kTile) {
        const int k = base + threadIdx.x;
        if (k < m) {
            tx[threadIdx.x] = kp[3 * k];
            ty[threadIdx.x] = kp[3 * k + 1];
            tz[threadIdx.x] = kp[3 * k + 2];
        }
        __syncthreads();
        const int lim = min(kTile, m - base);
        for (int kk = 0; kk < lim; ++kk) {
            const float d = dist_l2(tx[kk], ty[kk], tz[kk], ux, uy, uz);
            const int id = base + kk;
            if (d < b1) {
                b3 = b2; i3 = i2; b2 = b1; i2 = i1; b1 = d; i1 = id;
            } else if (d < b2) {
                b3 = b2; i3 = i2; b2 = d; i2 = id;
            } else if (d < b3) {
                b3 = d; i3 = id;
            }
        }
        __syncthreads();
    }
    if (active) {
        const int64_t o = (static_cast<int64_t>(b) * n + i) * 3;
        dist2[o] = b1; dist2[o + 1] = b2; dist2[o + 2] = b3;
        idx[o] = i1; idx[o + 1] = i2; idx[o + 2] = i3;
    }
}

__global__ void three_interpolate_kernel(const float* __restrict__ feat, const int32_t* __restrict__ idx,
                                         const float* __restrict__ w, int B, int C, int m, int n,
                                         float* __restrict__ out) {
    const int64_t total = static_cast<int64_t>(B) * C * n;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e % n;
        const int64_t bc = e / n;
        const int64_t b = bc / C;
        const int32_t* ii = idx + (b * n + i) * 3;
        const float* ww = w + (b * n + i) * 3;
        const float* f = feat + bc * m;
        out[e] = __builtin_fmaf(ww[2], f[ii[2]], __builtin_fmaf(ww[1], f[ii[1]], ww[0] * f[ii[0]]));
    }
}

__global__ void three_interpolate_grad_kernel(const float* __restrict__ grad, const int32_t* __restrict__ idx,
                                              const float* __restrict__ w, int B, int C, int n, int m,
                                              float* __restrict__ out) {
    const int64_t total = static_cast<int64_t>(B) * C * n;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e % n;
        const int64_t bc = e / n;
        const int64_t b = bc / C;
        const int32_t* ii = idx + (b * n + i) * 3;
        const float* ww = w + (b * n + i) * 3;
        const float g = grad[e];
        float* o = out + bc * m;
        atomicAdd(o + ii[0], g * ww[0]);
        atomicAdd(o + ii[1], g * ww[1]);
        atomicAdd(o + ii[2], g * ww[2]);
    }
}

// deterministic gradient (torch.use_deterministic_algorithms(True)): the
// 3 n pairs of each batch are grouped by source point (prim::build_inverse,
// key b * m + idx) and each grad_features element sums its pairs in
// ascending (i, j) order instead of 3 fp32 atomics per pair.
__global__ void three_interp_keys_kernel(const int32_t* __restrict__ idx, int64_t B, int64_t n, int64_t m,
                                         uint32_t* __restrict__ keys) {
    const int64_t total = B * n * 3;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t b = e / (3 * n);
        const int64_t v = idx[e];
        keys[e] = static_cast<uint32_t>(v >= 0 && v < m ? b * m + v : B * m);
    }
}

__global__ void three_interpolate_grad_det_kernel(const float* __restrict__ grad, const float* __restrict__ w,
                                                  const uint32_t* __restrict__ pairs, const int64_t* __restrict__ off,
                                                  int64_t B, int64_t C, int64_t n, int64_t m,
                                                  float* __restrict__ out) {
    const int64_t total = B * C * m;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t t = e % m;
        const int64_t bc = e / m;
        const int64_t b = bc / C;
        const int64_t key = b * m + t;
        const float* g = grad + bc * n - b * n;  // g[b * n + i] = grad[b, c, i]
        float acc = 0.f;
        for (int64_t p = off[key]; p < off[key + 1]; ++p) {
            const uint32_t pr = pairs[p];
            acc += g[pr / 3] * w[pr];
        }
        out[e] = acc;
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_furthest_point_sampling_workspace_size(int64_t B, int64_t n) {
    return n > 32 * kFpsThreads ? ws_bytes<float>(B * n) : 0;
}

// xyz f32 [B,N,3] -> out int32 [B,m]
O3DML_API int o3dml_furthest_point_sampling(const float* xyz, int64_t B, int64_t n, int64_t m, int32_t* out,
                                            void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(n > 0 || m == 0, "furthest_point_sampling: empty cloud");
    O3DML_REQUIRE(n < (int64_t(1) << 31) && m < (int64_t(1) << 31), "furthest_point_sampling: too large");
    if (B == 0 || m == 0) return 0;
    hipStream_t st = as_stream(stream);
    const int ni = static_cast<int>(n), mi = static_cast<int>(m);
    const int items = static_cast<int>(ceil_div(n, kFpsThreads));
    dim3 g(static_cast<unsigned>(B));
    if (items <= 1) fps_kernel<1><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else if (items <= 2) fps_kernel<2><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else if (items <= 4) fps_kernel<4><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else if (items <= 8) fps_kernel<8><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else if (items <= 16) fps_kernel<16><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else if (items <= 32) fps_kernel<32><<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, out);
    else {
        Workspace ws(workspace, workspace_bytes);
        float* temp = ws.take<float>(B * n);
        fps_global_kernel<<<g, kFpsThreads, 0, st>>>(xyz, ni, mi, temp, out);
    }
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// xyz [B,N,3], center [B,M,3] -> out int32 [B,M,nsample]
O3DML_API int o3dml_ball_query(const float* xyz, const float* center, int64_t B, int64_t n, int64_t m, float radius,
                               int64_t nsample, int32_t* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(nsample >= 1, "ball_query: nsample must be >= 1");
    if (B == 0 || m == 0) return 0;
    dim3 g(static_cast<unsigned>(ceil_div(m, kTile)), static_cast<unsigned>(B));
    ball_query_kernel<<<g, kTile, 0, as_stream(stream)>>>(xyz, center, static_cast<int>(n), static_cast<int>(m),
                                                          radius * radius, static_cast<int>(nsample), out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// unknown [B,n,3], known [B,m,3] -> dist2 f32 [B,n,3], idx int32 [B,n,3]
O3DML_API int o3dml_three_nn(const float* unknown, const float* known, int64_t B, int64_t n, int64_t m, float* dist2,
                             int32_t* idx, void* stream) {
    O3DML_GUARD_BEGIN
    if (B == 0 || n == 0) return 0;
    dim3 g(static_cast<unsigned>(ceil_div(n, kTile)), static_cast<unsigned>(B));
    three_nn_kernel<<<g, kTile, 0, as_stream(stream)>>>(unknown, known, static_cast<int>(n), static_cast<int>(m), dist2,
                                                        idx);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// features [B,C,m], idx [B,n,3], weight [B,n,3] -> out [B,C,n]
O3DML_API int o3dml_three_interpolate(const float* features, const int32_t* idx, const float* weight, int64_t B,
                                      int64_t C, int64_t m, int64_t n, float* out, void* stream) {
    O3DML_GUARD_BEGIN
    const int64_t total = B * C * n;
    if (total == 0) return 0;
    three_interpolate_kernel<<<stream_grid(total, 256), 256, 0, as_stream(stream)>>>(
            features, idx, weight, (int)B, (int)C, (int)m, (int)n, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// grad_out [B,C,n] -> grad_features [B,C,m] (zeroed here, then fp32 atomics)
O3DML_API int o3dml_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight, int64_t B,
                                           int64_t C, int64_t n, int64_t m, float* grad_features, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    if (B * C * m > 0) fill_async(grad_features, 0, sizeof(float) * B * C * m, st);
    const int64_t total = B * C * n;
    if (total == 0) return 0;
    three_interpolate_grad_kernel<<<stream_grid(total, 256), 256, 0, st>>>(grad_out, idx, weight, (int)B, (int)C,
                                                                          (int)n, (int)m, grad_features);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_three_interpolate_grad_workspace_size(int64_t B, int64_t n, int64_t m) {
    return prim::inverse_workspace_bytes(B * n * 3, B * m);
}

// deterministic three_interpolate_grad (fixed summation order; no memset needed)
O3DML_API int o3dml_three_interpolate_grad_det(const float* grad_out, const int32_t* idx, const float* weight,
                                               int64_t B, int64_t C, int64_t n, int64_t m, float* grad_features,
                                               void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    const int64_t total = B * C * m;
    if (total == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    uint32_t* keys = ws.take<uint32_t>(B * n * 3);
    if (n > 0) {
        three_interp_keys_kernel<<<stream_grid(B * n * 3, 256), 256, 0, st>>>(idx, B, n, m, keys);
        O3DML_LAUNCH_CHECK();
    }
    const prim::Inverse inv = prim::build_inverse(keys, B * n * 3, B * m, ws, st);
    three_interpolate_grad_det_kernel<<<stream_grid(total, 256, 256 * 16), 256, 0, st>>>(grad_out, weight, inv.pairs,
                                                                                       inv.off, B, C, n, m,
                                                                                       grad_features);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
