// dense.hip — the per-point 1x1 convolutions of RandLA-Net (SharedMLP,
// ml3d/torch/models/randlanet.py:469-512: Conv2d 1x1 + BatchNorm2d +
// LeakyReLU) as ONE launch each in eval mode:
//
//   out[r, :] = act([a1[r, :] | a2[r', :]] @ W^T + bias),   act = LeakyReLU(slope) or identity
//
// with BatchNorm folded into W / bias on the host, and the second operand a2
// covering two cases with no extra pass: LocalFeatureAggregation's tail
// lrelu(mlp2(x) + shortcut(feat)) (randlanet.py:689-692) as one GEMM over the
// concatenated K = [x | feat] with [W2 | Ws], and the decoder's
// [skip | upsampled] concatenation (randlanet.py:281-290: r' = a2_index[r]).
// Replaces a rocBLAS GEMM + a LeakyReLU launch (+ an add) per layer.
//
// Shapes: K <= 768, M <= 512, N = 176 .. 45,056 rows.  The deep levels have
// few rows (704 x 768 -> 512), so the K loop is split over blocks until the
// grid holds ~4 blocks per CU (deterministic reduction: per-split f32 partial
// slabs summed in split order by dense_split_reduce_kernel, which adds the
// bias and applies the activation; optionally the last block of each tile
// does it instead, see fused_reduce); the K loop
// itself keeps the next 32-wide chunk in registers while the current one is
// consumed from LDS, so one barrier pair per chunk and the global loads are in
// flight during the FMAs.  f32 FMA accumulation in K order within a split.
// Tile: 256 threads = 16 x 16, each thread TR rows x TC columns (rows
// ty + 16 i, columns tx + 16 j); A chunk [32][16 TR + 1], W chunk [32][16 TC + 1]
// (k-major, conflict-free stores: the +1 row pitch rotates the banks).
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "counters.hpp"

namespace o3dml {

constexpr int kDenseKC = 32;

template <int TR, int TC, bool SPLIT>
__global__ void __launch_bounds__(256) dense_act_kernel(const float* __restrict__ a1, int k1,
                                                        const float* __restrict__ a2, int k2,
                                                        const int64_t* __restrict__ a2_index,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        int64_t n, int m, int k_per_split, float slope, int act,
                                                        float* __restrict__ out, float* __restrict__ part,
                                                        uint32_t* __restrict__ counters) {
    constexpr int RB = 16 * TR, CB = 16 * TC;
    constexpr int LA = TR * kDenseKC / 16, LW = TC * kDenseKC / 16;  // loads per thread per chunk
    __shared__ float As[kDenseKC][RB + 1];
    __shared__ float Ws[kDenseKC][CB + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int lk = threadIdx.x & (kDenseKC - 1), lr = threadIdx.x / kDenseKC;  // load lanes: k fastest
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * RB;
    const int c0 = blockIdx.y * CB;
    const int K = k1 + k2;
    const int kbeg = blockIdx.z * k_per_split, kend = min(K, kbeg + k_per_split);
    // rows this thread loads: lr + 8 i; their a2 row (gathered decoder operand)
    int64_t arow[LA], a2row[LA];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
        arow[i] = r0 + lr + 8 * i;
        a2row[i] = arow[i] < n ? (a2_index ? a2_index[arow[i]] : arow[i]) : 0;
    }
    float ra[LA], rw[LW];
    auto load = [&](int kb) {
        const int k = kb + lk;
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            float v = 0.f;
            if (arow[i] < n && k < kend) v = k < k1 ? a1[arow[i] * k1 + k] : a2[a2row[i] * k2 + (k - k1)];
            ra[i] = v;
        }
#pragma unroll
        for (int j = 0; j < LW; ++j) {
            const int c = c0 + lr + 8 * j;
            rw[j] = (c < m && k < kend) ? w[static_cast<int64_t>(c) * K + k] : 0.f;
        }
    };
    float acc[TR][TC];
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[i][j] = 0.f;
    if (kbeg < kend) load(kbeg);
    for (int kb = kbeg; kb < kend; kb += kDenseKC) {
#pragma unroll
        for (int i = 0; i < LA; ++i) As[lk][lr + 8 * i] = ra[i];
#pragma unroll
        for (int j = 0; j < LW; ++j) Ws[lk][lr + 8 * j] = rw[j];
        __syncthreads();
        if (kb + kDenseKC < kend) load(kb + kDenseKC);  // next chunk in flight during the FMAs
        const int kn = min(kDenseKC, kend - kb);
        for (int kk = 0; kk < kn; ++kk) {
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
    float* dst = SPLIT ? part + static_cast<int64_t>(blockIdx.z) * n * m : out;
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        const int64_t r = r0 + ty + 16 * i;
        if (r >= n) continue;
#pragma unroll
        for (int j = 0; j < TC; ++j) {
            const int c = c0 + tx + 16 * j;
            if (c >= m) continue;
            float v = acc[i][j];
            if (!SPLIT) {
                v += bias ? bias[c] : 0.f;
                if (act) v = v >= 0.f ? v : v * slope;
                dst[r * m + c] = v;
            } else if (counters) {
                // slab entries as agent-scope stores: written through to the
                // device-coherent level, no L2 write-back fence needed
                __hip_atomic_store(dst + r * m + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                dst[r * m + c] = v;
            }
        }
    }
    if constexpr (SPLIT) {
        if (!counters) return;  // dense_split_reduce_kernel finishes
        // arrival once this block's slab stores are complete; the last of the
        // tile's gridDim.z blocks sums the slabs in split order, reading them
        // with agent-scope loads (past the non-coherent caches).  A device-
        // scope fence here would write back the whole L2 per block (8 XCDs:
        // measured 2x slower RandLA frames).
        __shared__ uint32_t s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t tile = blockIdx.y * gridDim.x + blockIdx.x;
        if (threadIdx.x == 0) s_last = atomicAdd(counters + tile, 1u) == gridDim.z - 1;
        __syncthreads();
        if (!s_last) return;
#pragma unroll
        for (int i = 0; i < TR; ++i) {
            const int64_t r = r0 + ty + 16 * i;
            if (r >= n) continue;
#pragma unroll
            for (int j = 0; j < TC; ++j) {
                const int c = c0 + tx + 16 * j;
                if (c >= m) continue;
                float v = 0.f;
                for (unsigned sp = 0; sp < gridDim.z; ++sp)
                    v += __hip_atomic_load(part + sp * n * m + r * m + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v += bias ? bias[c] : 0.f;
                if (act) v = v >= 0.f ? v : v * slope;
                out[r * m + c] = v;
            }
        }
        if (threadIdx.x == 0) atomicExch(counters + tile, 0u);  // ready for the next launch
    }
}

// out = act(sum_s part[s] + bias), splits summed in order
__global__ void dense_split_reduce_kernel(const float* __restrict__ part, int splits, int64_t n, int m,
                                          const float* __restrict__ bias, float slope, int act,
                                          float* __restrict__ out) {
    const int64_t total = n * m;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float v = sum_slabs(part, splits, total, e);
        v += bias ? bias[e % m] : 0.f;
        if (act) v = v >= 0.f ? v : v * slope;
        out[e] = v;
    }
}

struct DensePlan {
    int tr, tc, splits, k_per_split;
    unsigned gx, gy;
};

static DensePlan dense_plan(int64_t n, int k, int m) {
    DensePlan p;
    p.tc = m <= 16 ? 1 : (m <= 32 ? 2 : 4);
    p.gy = static_cast<unsigned>((m + 16 * p.tc - 1) / (16 * p.tc));
    p.tr = ceil_div(n, 64) * p.gy < 1024 ? 2 : 4;
    p.gx = static_cast<unsigned>(ceil_div(n, 16 * p.tr));
    // split K until ~4 blocks per CU (1024), each split >= 2 chunks
    // (O3DML_DENSE_TARGET / O3DML_DENSE_MIN_CHUNKS: A/B of the split plan)
    static const int64_t target = [] {
        const char* e = std::getenv("O3DML_DENSE_TARGET");
        return e ? std::atoll(e) : 1024;
    }();
    static const int min_chunks = [] {
        const char* e = std::getenv("O3DML_DENSE_MIN_CHUNKS");
        return e ? std::max(1, std::atoi(e)) : 2;
    }();
    const int64_t blocks = static_cast<int64_t>(p.gx) * p.gy;
    int s = static_cast<int>(std::min<int64_t>(ceil_div(target, blocks), ceil_div(k, min_chunks * kDenseKC)));
    s = std::max(1, std::min(s, 16));
    p.k_per_split = static_cast<int>(ceil_div(ceil_div(k, s), kDenseKC) * kDenseKC);
    p.splits = static_cast<int>(ceil_div(k, p.k_per_split));
    return p;
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_dense_act_workspace_size(int64_t n, int k, int m) {
    const DensePlan p = dense_plan(n, k, m);
    return p.splits > 1 ? ws_bytes<float>(static_cast<int64_t>(p.splits) * n * m) : 0;
}

O3DML_API int o3dml_dense_act(const float* a1, int k1, const float* a2, int k2, const int64_t* a2_index,
                              const float* weight, const float* bias, int64_t n, int m, int act, float slope,
                              float* out, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k1 >= 0 && k2 >= 0 && k1 + k2 > 0 && m > 0, "dense: bad shape (k1 %d, k2 %d, m %d)", k1, k2, m);
    O3DML_REQUIRE(k2 == 0 || a2, "dense: second operand missing");
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    const DensePlan p = dense_plan(n, k1 + k2, m);
    float* part = nullptr;
    if (p.splits > 1) {
        Workspace ws(workspace, workspace_bytes);
        part = ws.take<float>(static_cast<int64_t>(p.splits) * n * m);
    }
    const dim3 grid(p.gx, p.gy, static_cast<unsigned>(p.splits));
    // Split-K finished by each tile's last block (O3DML_DENSE_FUSED_REDUCE=1):
    // bit-identical, but OFF by default — measured on RandLA (same-session
    // A/B, graph-replayed patches) 15.8-16.0 vs 14.6-14.9 ms/frame: the
    // agent-scope (write-through) slab traffic costs more than the reduce
    // launch it saves, and a device-scope fence instead is 2x slower still.
    static const bool fused_reduce = [] {
        const char* e = std::getenv("O3DML_DENSE_FUSED_REDUCE");
        return e ? std::atoi(e) != 0 : false;
    }();
    uint32_t* counters =
            p.splits > 1 && fused_reduce ? tile_counters(st, static_cast<int64_t>(p.gx) * p.gy) : nullptr;
#define O3DML_DENSE(TR, TC, S)                                                                                   \
    dense_act_kernel<TR, TC, S><<<grid, 256, 0, st>>>(a1, k1, a2, k2, a2_index, weight, bias, n, m,             \
                                                      p.k_per_split, slope, act, out, part, counters)
#define O3DML_DENSE_S(TR, TC)                          \
    do {                                               \
        if (p.splits > 1) O3DML_DENSE(TR, TC, true);   \
        else O3DML_DENSE(TR, TC, false);               \
    } while (0)
    if (p.tr == 2) {
        if (p.tc == 1) O3DML_DENSE_S(2, 1); else if (p.tc == 2) O3DML_DENSE_S(2, 2); else O3DML_DENSE_S(2, 4);
    } else {
        if (p.tc == 1) O3DML_DENSE_S(4, 1); else if (p.tc == 2) O3DML_DENSE_S(4, 2); else O3DML_DENSE_S(4, 4);
    }
#undef O3DML_DENSE_S
#undef O3DML_DENSE
    O3DML_LAUNCH_CHECK();
    if (p.splits > 1 && !counters) {
        dense_split_reduce_kernel<<<stream_grid(n * m, 256), 256, 0, st>>>(part, p.splits, n, m, bias, slope, act,
                                                                          out);
        O3DML_LAUNCH_CHECK();
    }
    O3DML_GUARD_END
}
