// dense.hip — the per-point 1x1 convolutions of RandLA-Net (SharedMLP,
// ml3d/torch/models/randlanet.py:469-512: Conv2d 1x1 + BatchNorm2d +
// LeakyReLU) as ONE launch each in eval mode:
//
//   out[r, :] = act([a1[r, :] | a2[r, :]] @ W^T + bias),   act = LeakyReLU(slope) or identity
//
// with BatchNorm folded into W / bias on the host, and the second operand a2
// covering two cases with no extra pass: LocalFeatureAggregation's tail
// lrelu(mlp2(x) + shortcut(feat)) (randlanet.py:689-692) as one GEMM over the
// concatenated K = [x | feat] with [W2 | Ws], and the decoder's
// [skip | upsampled] concatenation (randlanet.py:281-290, a2 gathered through
// an index: a2_index[r] selects the row of a2).  Replaces a rocBLAS GEMM + a
// LeakyReLU launch (+ an add) per layer: 25 GEMMs and 25 element-wise
// launches per 45,056-point patch before.
//
// Shapes are small (K <= 768, M <= 512) and N is 176 .. 45,056 rows: the
// kernel is launch/HBM-bound at the wide levels and VALU-bound at the deep
// ones; f32 FMA accumulation in K order (parity: logits within 2e-4 of the
// reference, tests/test_gpu_randla.py).  Tile: 256 threads = 16 x 16, each
// thread TR rows x TC columns (rows ty + 16 i, columns tx + 16 j), K staged
// through LDS in chunks of 16 (A chunk [16][16 TR], W chunk [16][16 TC]).
#include <algorithm>

#include "common.hpp"

namespace o3dml {

constexpr int kDenseKC = 16;

template <int TR, int TC>
__global__ void __launch_bounds__(256) dense_act_kernel(const float* __restrict__ a1, int k1,
                                                        const float* __restrict__ a2, int k2,
                                                        const int64_t* __restrict__ a2_index,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        int64_t n, int m, float slope, int act,
                                                        float* __restrict__ out) {
    constexpr int RB = 16 * TR, CB = 16 * TC;
    __shared__ float As[kDenseKC][RB + 1];
    __shared__ float Ws[kDenseKC][CB + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * RB;
    const int c0 = blockIdx.y * CB;
    const int K = k1 + k2;
    float acc[TR][TC];
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[i][j] = 0.f;
    for (int kb = 0; kb < K; kb += kDenseKC) {
        // A chunk: RB rows x 16 k (thread t loads k = t % 16 of rows t / 16 + 16 i)
        {
            const int kk = threadIdx.x & 15;
            const int k = kb + kk;
#pragma unroll
            for (int i = 0; i < TR; ++i) {
                const int rr = (threadIdx.x >> 4) + 16 * i;
                const int64_t r = r0 + rr;
                float v = 0.f;
                if (r < n && k < K) {
                    if (k < k1) {
                        v = a1[r * k1 + k];
                    } else {
                        const int64_t ra = a2_index ? a2_index[r] : r;
                        v = a2[ra * k2 + (k - k1)];
                    }
                }
                As[kk][rr] = v;
            }
            // W chunk: 16 k x CB columns, W is [m, K] row-major (torch Linear layout)
#pragma unroll
            for (int j = 0; j < TC; ++j) {
                const int cc = (threadIdx.x >> 4) + 16 * j;
                const int c = c0 + cc;
                Ws[kk][cc] = (c < m && k < K) ? w[static_cast<int64_t>(c) * K + k] : 0.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kDenseKC; ++kk) {
            float av[TR], bv[TC];
#pragma unroll
            for (int i = 0; i < TR; ++i) av[i] = As[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < TC; ++j) bv[j] = Ws[kk][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < TR; ++i)
#pragma unroll
                for (int j = 0; j < TC; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        const int64_t r = r0 + ty + 16 * i;
        if (r >= n) continue;
#pragma unroll
        for (int j = 0; j < TC; ++j) {
            const int c = c0 + tx + 16 * j;
            if (c >= m) continue;
            float v = acc[i][j] + (bias ? bias[c] : 0.f);
            if (act) v = v >= 0.f ? v : v * slope;
            out[r * m + c] = v;
        }
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int o3dml_dense_act(const float* a1, int k1, const float* a2, int k2, const int64_t* a2_index,
                              const float* weight, const float* bias, int64_t n, int m, int act, float slope,
                              float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k1 >= 0 && k2 >= 0 && k1 + k2 > 0 && m > 0, "dense: bad shape (k1 %d, k2 %d, m %d)", k1, k2, m);
    O3DML_REQUIRE(k2 == 0 || a2, "dense: second operand missing");
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    // column tile: the output width rounded to 16 (<= 64 per block); row
    // tile: 64 rows (4 per thread), 32 when the grid would be small
    const int tc = m <= 16 ? 1 : (m <= 32 ? 2 : 4);
    const unsigned gy = static_cast<unsigned>((m + 16 * tc - 1) / (16 * tc));
    const bool small = ceil_div(n, 64) * gy < 512;
    const int rows = small ? 32 : 64;
    const unsigned gx = static_cast<unsigned>(ceil_div(n, rows));
    const dim3 grid(gx, gy);
#define O3DML_DENSE(TR, TC) \
    dense_act_kernel<TR, TC><<<grid, 256, 0, st>>>(a1, k1, a2, k2, a2_index, weight, bias, n, m, slope, act, out)
    if (small) {
        if (tc == 1) O3DML_DENSE(2, 1); else if (tc == 2) O3DML_DENSE(2, 2); else O3DML_DENSE(2, 4);
    } else {
        if (tc == 1) O3DML_DENSE(4, 1); else if (tc == 2) O3DML_DENSE(4, 2); else O3DML_DENSE(4, 4);
    }
#undef O3DML_DENSE
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
