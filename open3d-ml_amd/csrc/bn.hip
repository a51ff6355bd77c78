// bn.hip — BatchNorm1d over the point axis (+ the LeakyReLU that follows it)
// for KPFCNN (ml3d/torch/models/kpconv.py:1213-1295, BatchNormBlock /
// UnaryBlock / SimpleBlock / ResnetBottleneckBlock: nn.BatchNorm1d on the
// [1, C, N] view, i.e. per-channel statistics over the N rows of [N, C]).
//
// torch runs a BN + LeakyReLU pair as 4 launches forward (statistics, running
// update, transform, activation) and 3 backward (activation, reduce,
// element-wise), and its channels-last statistics kernel reads a 40,000 x 128
// layer at ~0.25 TB/s.  Here: forward = a reduce launch (per-block partial
// sums of x and x^2 in double), a finalize launch (a workgroup per channel
// sums the partials in a fixed order — deterministic — and finalises mean,
// invstd, the running statistics and num_batches_tracked) and an apply launch
// (normalise, affine, LeakyReLU); backward = the same three for sum dz and
// dz * xhat (dz the activation's gradient, recomputed from x; finalised into
// grad_weight, grad_bias and the dx coefficients).  The statistics are
// accumulated in double (closer to the fp64 reference than fp32 Welford).
//
// save [4C] = (mean, invstd, k = weight * invstd, bias): forward output,
// backward input.  y = (x - mean) * k + bias, then LeakyReLU when act.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "counters.hpp"

namespace o3dml {

constexpr int kBnThreads = 256;
constexpr int kBnMaxBlocks = 128;  // partials the finishing block sums

struct BnArgs {
    const float* x;
    const float* dy;      // backward only
    int64_t n;
    int c;
    int64_t rows_per_block;
    const float* weight;  // nullable (affine off)
    const float* bias;    // nullable
    float* running_mean;  // nullable (no tracking)
    float* running_var;
    int64_t* num_batches;  // nullable
    float momentum, eps, slope;
    int act, training;
    float* save;          // [4C]
    float* coef;          // [2C] backward dx coefficients
    float* grad_weight;   // nullable
    float* grad_bias;     // nullable
    double* part;         // [2][G][C] ([2][C][G] when part_t)
    int part_t;           // tree finalize: channel-major partials
};

// accumulate (s, q) of one element for channel ch: forward x, x^2;
// backward dz, dz * xhat (dyv: the gradient element)
template <int MODE>
__device__ __forceinline__ void bn_accum_v(const BnArgs& a, float x, float dyv, int ch, double& s, double& q) {
    if (MODE == 0) {
        s += x;
        q += static_cast<double>(x) * x;
    } else {
        const float mean = a.save[ch], inv = a.save[a.c + ch], k = a.save[2 * a.c + ch], b = a.save[3 * a.c + ch];
        const float d = x - mean;
        float dz = dyv;
        if (a.act) {
            const float z = d * k + b;
            if (!(z > 0.f)) dz = dz * a.slope;
        }
        const float xhat = d * inv;
        s += dz;
        q += static_cast<double>(dz) * xhat;
    }
}

// rows r0 + ro, r0 + ro + step, ... < r1 of channel ch, 8 rows' loads in
// flight per thread (a load-use chain per row left this latency-bound)
template <int MODE>
__device__ __forceinline__ void bn_rows(const BnArgs& a, int64_t r0, int64_t r1, int64_t step, int ch, double& s,
                                        double& q) {
    constexpr int U = 8;
    const int64_t c = a.c;
    int64_t r = r0;
    for (; r + (U - 1) * step < r1; r += U * step) {
        float xv[U], gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            xv[u] = a.x[(r + u * step) * c + ch];
            gv[u] = MODE == 1 ? a.dy[(r + u * step) * c + ch] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) bn_accum_v<MODE>(a, xv[u], gv[u], ch, s, q);
    }
    for (; r < r1; r += step) bn_accum_v<MODE>(a, a.x[r * c + ch], MODE == 1 ? a.dy[r * c + ch] : 0.f, ch, s, q);
}

// the per-channel finish from the totals S, Q
template <int MODE>
__device__ __forceinline__ void bn_finish(const BnArgs& a, int ch, double S, double Q) {
    const int c = a.c;
    const double n = static_cast<double>(a.n);
    if (MODE == 0) {
        const float w = a.weight ? a.weight[ch] : 1.f, b = a.bias ? a.bias[ch] : 0.f;
        if (a.training) {
            const double mean = S / n;
            const double var = fmax(Q / n - mean * mean, 0.0);
            const float inv = static_cast<float>(1.0 / sqrt(var + static_cast<double>(a.eps)));
            a.save[ch] = static_cast<float>(mean);
            a.save[c + ch] = inv;
            a.save[2 * c + ch] = w * inv;
            a.save[3 * c + ch] = b;
            if (a.running_mean) {
                const float m = a.momentum;
                a.running_mean[ch] = (1.f - m) * a.running_mean[ch] + m * static_cast<float>(mean);
                a.running_var[ch] = (1.f - m) * a.running_var[ch] + m * static_cast<float>(var * n / (n - 1.0));
            }
        }
    } else {
        if (a.grad_weight) a.grad_weight[ch] = static_cast<float>(Q);
        if (a.grad_bias) a.grad_bias[ch] = static_cast<float>(S);
        a.coef[ch] = a.training ? static_cast<float>(S / n) : 0.f;
        a.coef[c + ch] = a.training ? static_cast<float>(Q / n) : 0.f;
    }
}

// index of partial (which: 0 = S, 1 = Q) of block b, channel ch
__device__ __forceinline__ int64_t bn_pidx(const BnArgs& a, int G, int which, int b, int ch) {
    return a.part_t ? (static_cast<int64_t>(which) * a.c + ch) * G + b
                    : (static_cast<int64_t>(which) * G + b) * a.c + ch;
}

// partial store: agent scope when the last-arriving block reads it in this
// launch, plain when a separate finalize launch does
__device__ __forceinline__ void bn_store(double* p, double v, bool agent) {
    if (agent) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

__device__ __forceinline__ double bn_load(const double* p, bool agent) {
    return agent ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

// the totals of the G partials, every thread busy (packed: 256 / C threads
// per channel, partials strided over them, then summed in thread order
// through LDS; wide C: a thread per channel), 8 agent-scope loads in flight
// per thread; fixed order throughout (deterministic)
template <int MODE>
__device__ void bn_finalize_block(const BnArgs& a, int G, bool agent) {
    __shared__ double fs[kBnThreads], fq[kBnThreads];
    const int tid = threadIdx.x, c = a.c;
    const int per = c <= kBnThreads ? kBnThreads / c : 1;
    for (int cb = 0; cb < c; cb += kBnThreads) {
        const int ch = c <= kBnThreads ? tid % c : cb + tid, ro = c <= kBnThreads ? tid / c : 0;
        double S = 0.0, Q = 0.0;
        if (ro < per && ch < c) {
            int b = ro;
            for (; b + 7 * per < G; b += 8 * per) {
                double vs[8], vq[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    vs[u] = bn_load(a.part + static_cast<int64_t>(b + u * per) * c + ch, agent);
                    vq[u] = bn_load(a.part + (static_cast<int64_t>(G) + b + u * per) * c + ch, agent);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    S += vs[u];
                    Q += vq[u];
                }
            }
            for (; b < G; b += per) {
                S += bn_load(a.part + static_cast<int64_t>(b) * c + ch, agent);
                Q += bn_load(a.part + (static_cast<int64_t>(G) + b) * c + ch, agent);
            }
        }
        if (c <= kBnThreads) {
            fs[tid] = S;
            fq[tid] = Q;
            __syncthreads();
            if (tid < c) {
                S = 0.0;
                Q = 0.0;
                for (int k = 0; k < per; ++k) {
                    S += fs[k * c + tid];
                    Q += fq[k * c + tid];
                }
                bn_finish<MODE>(a, tid, S, Q);
            }
            break;
        }
        if (ch < c) bn_finish<MODE>(a, ch, S, Q);
    }
    if (MODE == 0 && a.training && a.num_batches && threadIdx.x == 0) a.num_batches[0] += 1;
}

// partial sums per block (rows [blockIdx * rpb, +rpb)); the last-arriving
// block (counter != nullptr) finalises
template <int MODE>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_kernel(BnArgs a, uint32_t* __restrict__ counter) {
    __shared__ double sh_s[kBnThreads], sh_q[kBnThreads];
    const int tid = threadIdx.x, G = gridDim.x, c = a.c;
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * a.rows_per_block;
    const int64_t r1 = min(a.n, r0 + a.rows_per_block);
    if (c <= kBnThreads) {
        // rows packed: thread -> (row offset tid / c, channel tid % c)
        const int per = kBnThreads / c, ch = tid % c, ro = tid / c;
        double s = 0.0, q = 0.0;
        if (ro < per)
            bn_rows<MODE>(a, r0 + ro, r1, per, ch, s, q);
        sh_s[tid] = s;
        sh_q[tid] = q;
        __syncthreads();
        if (tid < c) {
            double S = 0.0, Q = 0.0;
            for (int k = 0; k < per; ++k) {
                S += sh_s[k * c + tid];
                Q += sh_q[k * c + tid];
            }
            bn_store(a.part + bn_pidx(a, G, 0, blockIdx.x, tid), S, counter != nullptr);
            bn_store(a.part + bn_pidx(a, G, 1, blockIdx.x, tid), Q, counter != nullptr);
        }
    } else {
        // channel blocks of 256: thread -> channel cb + tid over every row
        for (int cb = 0; cb < c; cb += kBnThreads) {
            const int ch = cb + tid;
            if (ch >= c) break;
            double s = 0.0, q = 0.0;
            bn_rows<MODE>(a, r0, r1, 1, ch, s, q);
            bn_store(a.part + bn_pidx(a, G, 0, blockIdx.x, ch), s, counter != nullptr);
            bn_store(a.part + bn_pidx(a, G, 1, blockIdx.x, ch), q, counter != nullptr);
        }
    }
    if (!counter) return;  // bn_finalize_kernel finishes
    // arrival once this block's partial stores are complete (the pattern of
    // dense.hip's split-K tiles: agent-scope stores and loads, no L2 flush)
    __shared__ uint32_t s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(counter, 1u) == static_cast<uint32_t>(G) - 1;
    __syncthreads();
    if (!s_last) return;
    bn_finalize_block<MODE>(a, G, true);
    if (tid == 0) atomicExch(counter, 0u);  // ready for the next launch
}

template <int MODE>
__global__ void __launch_bounds__(kBnThreads) bn_finalize_kernel(BnArgs a, int G) {
    bn_finalize_block<MODE>(a, G, false);
}

// tree finalize: one workgroup per channel sums its G (<= 1,024) channel-major
// partials (coalesced, <= 4 loads per thread, all in flight) and reduces them
// through LDS in a fixed order (deterministic)
template <int MODE>
__global__ void __launch_bounds__(kBnThreads) bn_finalize_tree_kernel(BnArgs a, int G) {
    __shared__ double fs[kBnThreads], fq[kBnThreads];
    const int ch = blockIdx.x, tid = threadIdx.x;
    const double* ps = a.part + static_cast<int64_t>(ch) * G;
    const double* pq = a.part + (static_cast<int64_t>(a.c) + ch) * G;
    double S = 0.0, Q = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int b = tid + u * kBnThreads;
        if (b < G) {
            S += ps[b];
            Q += pq[b];
        }
    }
    fs[tid] = S;
    fq[tid] = Q;
    __syncthreads();
    for (int h = kBnThreads / 2; h > 0; h >>= 1) {
        if (tid < h) {
            fs[tid] += fs[tid + h];
            fq[tid] += fq[tid + h];
        }
        __syncthreads();
    }
    if (tid == 0) {
        bn_finish<MODE>(a, ch, fs[0], fq[0]);
        if (MODE == 0 && ch == 0 && a.training && a.num_batches) a.num_batches[0] += 1;
    }
}

// eval forward: save from the running statistics
__global__ void bn_eval_save_kernel(BnArgs a) {
    for (int ch = blockIdx.x * blockDim.x + threadIdx.x; ch < a.c; ch += gridDim.x * blockDim.x) {
        const float w = a.weight ? a.weight[ch] : 1.f, b = a.bias ? a.bias[ch] : 0.f;
        const float inv = 1.f / sqrtf(a.running_var[ch] + a.eps);
        a.save[ch] = a.running_mean[ch];
        a.save[a.c + ch] = inv;
        a.save[2 * a.c + ch] = w * inv;
        a.save[3 * a.c + ch] = b;
    }
}

// forward apply: y = act((x - mean) * k + b); MODE 1: dx
template <int MODE>
__global__ void __launch_bounds__(kBnThreads) bn_apply_kernel(BnArgs a, float* __restrict__ out) {
    const int64_t total = a.n * a.c;
    const int c = a.c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(kBnThreads) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * kBnThreads) {
        const int ch = static_cast<int>(e % c);
        const float mean = a.save[ch], k = a.save[2 * c + ch], b = a.save[3 * c + ch];
        const float d = a.x[e] - mean;
        float z = d * k + b;
        if (MODE == 0) {
            if (a.act && !(z > 0.f)) z = z * a.slope;
            out[e] = z;
        } else {
            float dz = a.dy[e];
            if (a.act && !(z > 0.f)) dz = dz * a.slope;
            const float xhat = d * a.save[c + ch];
            out[e] = k * (dz - a.coef[ch] - xhat * a.coef[c + ch]);
        }
    }
}

// finalize of the partial sums (O3DML_BN_FINALIZE): 2 (default) = tree:
// <= 1,024 partials (8 elements per thread: one round of loads in flight) and
// a separate launch with a workgroup per channel; 0 = the last-arriving block
// of the reduce launch (<= 128 partials, 64 elements per thread); 1 = a
// separate one-workgroup launch over those.  Measured on the C3 step (kernel
// trace, last 5 steps, gpurun_out/r4s10): reduce + finalize 22.3 -> 10.2 +
// 4.8 us backward, 17.5 -> 7.4 + 5.1 us forward; 9.74 -> 9.19 ms of kernel
// time per step for 92 more launches.  Per-channel sums in a fixed order in
// every mode (deterministic).
static int bn_finalize_mode() {
    static const int m = [] {
        const char* e = std::getenv("O3DML_BN_FINALIZE");
        return e ? std::atoi(e) : 2;
    }();
    return m;
}

static int64_t bn_blocks(int64_t n, int c) {
    const bool tree = bn_finalize_mode() == 2;
    return std::max<int64_t>(1, std::min<int64_t>(tree ? 1024 : kBnMaxBlocks,
                                                  ceil_div(n * c, kBnThreads * (tree ? 8 : 64))));
}

template <int MODE>
static void bn_reduce(BnArgs& a, hipStream_t st) {
    const int64_t G = bn_blocks(a.n, a.c);
    a.rows_per_block = ceil_div(a.n, G);
    const int g = static_cast<int>(ceil_div(a.n, a.rows_per_block));
    const int fm = bn_finalize_mode();
    a.part_t = fm == 2;
    uint32_t* counter = fm == 0 ? tile_counters(st, 1) : nullptr;
    bn_reduce_kernel<MODE><<<g, kBnThreads, 0, st>>>(a, counter);
    O3DML_LAUNCH_CHECK();
    if (fm == 2) {
        bn_finalize_tree_kernel<MODE><<<a.c, kBnThreads, 0, st>>>(a, g);
        O3DML_LAUNCH_CHECK();
    } else if (!counter) {
        bn_finalize_kernel<MODE><<<1, kBnThreads, 0, st>>>(a, g);
        O3DML_LAUNCH_CHECK();
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_batch_norm_workspace_size(int64_t n, int c) {
    return ws_bytes<double>(2 * bn_blocks(n, c) * static_cast<int64_t>(c)) + ws_bytes<float>(2 * c);
}

O3DML_API int o3dml_batch_norm_forward(const float* x, int64_t n, int c, const float* weight, const float* bias,
                                       float* running_mean, float* running_var, int64_t* num_batches_tracked,
                                       float momentum, float eps, int training, int act, float slope, float* y,
                                       float* save, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(c > 0, "batch_norm: channels must be > 0");
    O3DML_REQUIRE(n >= 0, "batch_norm: negative row count");
    O3DML_REQUIRE(!training || n > 1, "batch_norm: expected more than 1 value per channel when training");
    O3DML_REQUIRE(training || (running_mean && running_var), "batch_norm: eval mode needs running statistics");
    O3DML_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "batch_norm: running mean / var pair");
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    BnArgs a{};
    a.x = x;
    a.n = n;
    a.c = c;
    a.weight = weight;
    a.bias = bias;
    a.running_mean = running_mean;
    a.running_var = running_var;
    a.num_batches = num_batches_tracked;
    a.momentum = momentum;
    a.eps = eps;
    a.slope = slope;
    a.act = act;
    a.training = training;
    a.save = save;
    a.part = ws.take<double>(2 * bn_blocks(n, c) * static_cast<int64_t>(c));
    if (training) {
        bn_reduce<0>(a, st);
    } else {
        bn_eval_save_kernel<<<static_cast<unsigned>(ceil_div(c, 256)), 256, 0, st>>>(a);
        O3DML_LAUNCH_CHECK();
    }
    bn_apply_kernel<0><<<stream_grid(n * c, kBnThreads), kBnThreads, 0, st>>>(a, y);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_batch_norm_backward(const float* grad_y, const float* x, int64_t n, int c, const float* save,
                                        int training, int act, float slope, float* grad_x, float* grad_weight,
                                        float* grad_bias, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(c > 0, "batch_norm: channels must be > 0");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    BnArgs a{};
    a.x = x;
    a.dy = grad_y;
    a.n = n;
    a.c = c;
    a.slope = slope;
    a.act = act;
    a.training = training;
    a.save = const_cast<float*>(save);
    a.grad_weight = grad_weight;
    a.grad_bias = grad_bias;
    a.part = ws.take<double>(2 * bn_blocks(n, c) * static_cast<int64_t>(c));
    a.coef = ws.take<float>(2 * c);
    if (n == 0) {
        if (grad_weight) fill_async(grad_weight, 0, sizeof(float) * c, st);
        if (grad_bias) fill_async(grad_bias, 0, sizeof(float) * c, st);
        return 0;
    }
    bn_reduce<1>(a, st);
    if (grad_x) {
        bn_apply_kernel<1><<<stream_grid(n * c, kBnThreads), kBnThreads, 0, st>>>(a, grad_x);
        O3DML_LAUNCH_CHECK();
    }
    O3DML_GUARD_END
}
