// randla_sampler.hip — the per-patch bookkeeping of RandLA-Net inference
// (SemSegSpatiallyRegularSampler, ml3d/datasets/samplers/
// semseg_spatially_regular.py:79-109; RandLANet.transform, randlanet.py:
// 156-239) as three small kernels instead of ~20 torch launches and
// reductions per patch, plus the up-sampling indices derived from the k = 16
// lists instead of a second kNN search.
//
//  * possibility_min: min and FIRST argmin of the float64 possibilities (as
//    np.argmin), the centre point, the minimum also into pinned host memory
//    (the loop test `min > 0.5` is the one host read per patch);
//  * patch_prep / patch_apply: pc = sub[idxs], d = (dx^2 + dy^2) + dz^2 in
//    float32 (the reference's np.sum of np.square over the float32 differences,
//    no contraction), d_max, delta = (1 - d / d_max)^2 (float32), the float64
//    possibility update, and the augmenter's recentring of x, y (mean over the
//    patch: per-block partial sums in a fixed order, so every run gives the
//    same bits);
//  * up_from_knn: level i+1 is the first N_{i+1} points of level i
//    (randlanet.py:222-224), so the nearest level-(i+1) point of p is the first
//    entry of p's (distance, index)-sorted k = 16 list that lies in that prefix
//    — exactly knn_search(level i+1, level i, 1) whenever one does (the order
//    and the distances are the same); the ~(3/4)^16 = 1 % of points with none
//    in their list are searched by brute force over the prefix (one wave each).
#include <cfloat>

#include <hip/hip_fp16.h>

#include "common.hpp"

namespace o3dml {

constexpr int kPatchBlocks = 64;

constexpr int kMinBlocks = 128;

__device__ __forceinline__ void min_pair(double& v, int64_t& i, double ov, int64_t oi) {
    if (ov < v || (ov == v && oi < i)) {  // the first minimum, as np.argmin
        v = ov;
        i = oi;
    }
}

// per-block (min, first argmin) of a contiguous chunk
__global__ void __launch_bounds__(256) possibility_min_partial_kernel(const double* __restrict__ p, int64_t n,
                                                                      double* __restrict__ pv,
                                                                      int64_t* __restrict__ pi) {
    __shared__ double sv[4];
    __shared__ int64_t si[4];
    const int64_t per = ceil_div(n, kMinBlocks);
    const int64_t s = blockIdx.x * per, e = min(n, s + per);
    double best = DBL_MAX;
    int64_t bi = INT64_MAX;
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) min_pair(best, bi, p[i], i);
    for (int o = 32; o >= 1; o >>= 1) min_pair(best, bi, __shfl_xor(best, o, 64), __shfl_xor(bi, o, 64));
    if ((threadIdx.x & 63) == 0) {
        sv[threadIdx.x >> 6] = best;
        si[threadIdx.x >> 6] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) min_pair(best, bi, sv[w], si[w]);
        pv[blockIdx.x] = best;
        pi[blockIdx.x] = bi;
    }
}

__global__ void __launch_bounds__(64) possibility_min_final_kernel(const double* __restrict__ pv,
                                                                   const int64_t* __restrict__ pi, int64_t n,
                                                                   const float* __restrict__ sub,
                                                                   int64_t* __restrict__ arg,
                                                                   float* __restrict__ center,
                                                                   double* __restrict__ host_min) {
    double best = DBL_MAX;
    int64_t bi = INT64_MAX;
    for (int b = threadIdx.x; b < kMinBlocks; b += 64) min_pair(best, bi, pv[b], pi[b]);
    for (int o = 32; o >= 1; o >>= 1) min_pair(best, bi, __shfl_xor(best, o, 64), __shfl_xor(bi, o, 64));
    if (threadIdx.x == 0) {
        *arg = n ? bi : 0;
        if (n) {
            center[0] = sub[3 * bi];
            center[1] = sub[3 * bi + 1];
            center[2] = sub[3 * bi + 2];
        }
        if (host_min) *host_min = n ? best : DBL_MAX;
    }
}

// partials[b] = (max d, sum x, sum y) of block b's chunk
__global__ void __launch_bounds__(256) patch_prep_kernel(const float* __restrict__ sub,
                                                         const int64_t* __restrict__ idxs, int64_t n,
                                                         const float* __restrict__ center, float* __restrict__ pc,
                                                         float* __restrict__ d, float* __restrict__ partials) {
    __shared__ float red[3][4];
    const int64_t per = ceil_div(n, kPatchBlocks);
    const int64_t s = blockIdx.x * per, e = min(n, s + per);
    const float cx = center[0], cy = center[1], cz = center[2];
    float mx = 0.f, sx = 0.f, sy = 0.f;
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        const int64_t j = idxs[i];
        const float x = sub[3 * j], y = sub[3 * j + 1], z = sub[3 * j + 2];
        pc[3 * i] = x;
        pc[3 * i + 1] = y;
        pc[3 * i + 2] = z;
        const float dx = x - cx, dy = y - cy, dz = z - cz;
        const float di = (dx * dx + dy * dy) + dz * dz;
        d[i] = di;
        mx = fmaxf(mx, di);
        sx += x;
        sy += y;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        sx += __shfl_xor(sx, o, 64);
        sy += __shfl_xor(sy, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mx;
        red[1][threadIdx.x >> 6] = sx;
        red[2][threadIdx.x >> 6] = sy;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partials[3 * blockIdx.x] = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
        partials[3 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        partials[3 * blockIdx.x + 2] = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
    }
}

__global__ void __launch_bounds__(256) patch_apply_kernel(const int64_t* __restrict__ idxs, int64_t n,
                                                          const uint8_t* __restrict__ keep,
                                                          const float* __restrict__ partials,
                                                          const float* __restrict__ d, double* __restrict__ poss,
                                                          float* __restrict__ pc) {
    // every block reduces the partials in the same order: same bits everywhere
    float mx = 0.f, sx = 0.f, sy = 0.f;
    for (int b = 0; b < kPatchBlocks; ++b) {
        mx = fmaxf(mx, partials[3 * b]);
        sx += partials[3 * b + 1];
        sy += partials[3 * b + 2];
    }
    const float inv_n = 1.0f / static_cast<float>(n);
    const float mxx = sx * inv_n, myy = sy * inv_n;
    const int64_t per = ceil_div(n, kPatchBlocks);
    const int64_t s = blockIdx.x * per, e = min(n, s + per);
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        const float t = 1.0f - d[i] / mx;
        if (!keep || keep[i]) poss[idxs[i]] += static_cast<double>(t * t);
        pc[3 * i] -= mxx;
        pc[3 * i + 1] -= myy;
    }
}

struct UpLevels {
    int64_t rs[5];    // level starts in the concatenated levels 0..L-1
    int64_t nxt[4];   // size of level i + 1 (the prefix of level i)
    int64_t srs[4];   // level i + 1 start in the concatenated levels 1..L
    int nlev;
};

__device__ __forceinline__ int up_level(int64_t q, const UpLevels& L) {
    int i = 0;
    while (i + 1 < L.nlev && q >= L.rs[i + 1]) ++i;
    return i;
}

// up[q] = position of q's nearest point in level i + 1 (relative to that
// level); the k-list row is rewritten relative to q's own level in the same
// pass (the network consumes level-relative indices)
__global__ void up_from_knn_kernel(int32_t* __restrict__ nb, int k, int64_t total, UpLevels L,
                                   int64_t* __restrict__ up, uint32_t* __restrict__ fallback,
                                   uint32_t* __restrict__ n_fallback) {
    for (int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; q < total;
         q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int i = up_level(q, L);
        const int64_t base = L.rs[i], lim = L.nxt[i];
        int64_t r = -1;
        for (int j = 0; j < k; ++j) {
            const int64_t rel = static_cast<int64_t>(nb[q * k + j]) - base;
            nb[q * k + j] = static_cast<int32_t>(rel);
            if (r < 0 && rel < lim) r = rel;
        }
        if (r >= 0) up[q] = r;
        else fallback[atomicAdd(n_fallback, 1u)] = static_cast<uint32_t>(q);
    }
}

// one workgroup per listed query: (distance bits, index) minimum over the
// prefix, 4 independent loads in flight per thread
__global__ void __launch_bounds__(256) up_fallback_kernel(const float* __restrict__ cat, UpLevels L,
                                                          const uint32_t* __restrict__ fallback,
                                                          const uint32_t* __restrict__ n_fallback,
                                                          int64_t* __restrict__ up) {
    __shared__ uint64_t red[4];
    const int64_t cnt = *n_fallback;
    for (int64_t w = blockIdx.x; w < cnt; w += gridDim.x) {
        const int64_t q = fallback[w];
        const int i = up_level(q, L);
        const float qx = cat[3 * q], qy = cat[3 * q + 1], qz = cat[3 * q + 2];
        const float* base = cat + 3 * L.rs[i];
        const int64_t m = L.nxt[i];
        uint64_t best = ~0ull;
        constexpr int U = 4;
        for (int64_t r0 = threadIdx.x; r0 < m; r0 += U * 256) {
            float px[U], py[U], pz[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = r0 + u * 256;
                const bool ok = r < m;
                px[u] = ok ? base[3 * r] : 0.f;
                py[u] = ok ? base[3 * r + 1] : 0.f;
                pz[u] = ok ? base[3 * r + 2] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = r0 + u * 256;
                if (r < m) {
                    const float d = dist_l2(px[u], py[u], pz[u], qx, qy, qz);
                    const uint64_t key = (static_cast<uint64_t>(__float_as_uint(d)) << 32) | static_cast<uint32_t>(r);
                    best = key < best ? key : best;
                }
            }
        }
        for (int o = 32; o >= 1; o >>= 1) {
            const uint64_t other = __shfl_xor(best, o, 64);
            best = other < best ? other : best;
        }
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int j = 1; j < 4; ++j) best = red[j] < best ? red[j] : best;
            if (best != ~0ull) up[q] = static_cast<int64_t>(static_cast<uint32_t>(best));
        }
        __syncthreads();
    }
}

// dst[i] = src[perm(i)], perm a keyed bijection of [0, n): a 4-round Feistel
// network on the smallest even bit width covering n, cycle-walked into range
// (the patch shuffle of semseg_spatially_regular.py:100 — any uniformly
// random order serves; one launch instead of a sort of random keys)
__device__ __forceinline__ uint32_t feistel_mix(uint32_t x, uint32_t key) {
    x ^= key;
    x *= 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA77u;
    x ^= x >> 13;
    return x;
}

// seed_state (device u64 [2]: base, patch counter): the patch's key is
// splitmix64(base + counter), so a captured patch step draws a new
// permutation per replay (seed_advance_kernel bumps the counter after it)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void random_permute_kernel(const int64_t* __restrict__ src, int64_t n, int half, uint64_t seed,
                                      const uint64_t* __restrict__ seed_state, int64_t* __restrict__ dst) {
    if (seed_state) seed = splitmix64(seed_state[0] + seed_state[1]);
    const uint32_t mask = (1u << half) - 1u;
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    const uint32_t keys[4] = {k0, k1, k0 ^ 0xA5A5A5A5u, k1 ^ 0x3C3C3C3Cu};
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        uint32_t v = static_cast<uint32_t>(i);
        do {
            uint32_t l = v >> half, r = v & mask;
#pragma unroll
            for (int rd = 0; rd < 4; ++rd) {
                const uint32_t t = l ^ (feistel_mix(r, keys[rd]) & mask);
                l = r;
                r = t;
            }
            v = (l << half) | r;
        } while (v >= static_cast<uint64_t>(n));
        dst[i] = src[v];
    }
}

// test_probs[idxs[i]] = smooth * test_probs[idxs[i]] + (1 - smooth) * probs[i]
// (randlanet.py:441-465) with the reference's dtypes: a float16 store
// multiplies in float16 (f16(f16(smooth) * p16), exact product rounded once),
// adds the float32 new term in float32 and rounds to the store; keep masks
// duplicate indices to their last occurrence (numpy semantics)
template <bool HALF>
__global__ void update_probs_kernel(const float* __restrict__ probs, const int64_t* __restrict__ idxs,
                                    const uint8_t* __restrict__ keep, int64_t n, int c, float smooth_store,
                                    float new_w, void* __restrict__ store) {
    const int64_t total = n * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e / c;
        if (keep && !keep[i]) continue;
        const int64_t o = idxs[i] * c + (e - i * c);
        const float b = probs[e] * new_w;
        if constexpr (HALF) {
            __half* t = static_cast<__half*>(store);
            const float a = __half2float(__float2half_rn(__half2float(t[o]) * smooth_store));
            t[o] = __float2half_rn(a + b);
        } else {
            float* t = static_cast<float*>(store);
            t[o] = t[o] * smooth_store + b;
        }
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int o3dml_randla_possibility_min(const double* possibility, int64_t n, const float* sub, int64_t* argmin,
                                           float* center, double* host_min, void* workspace, size_t workspace_bytes,
                                           void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    double* pv = ws.take<double>(kMinBlocks);
    int64_t* pi = ws.take<int64_t>(kMinBlocks);
    possibility_min_partial_kernel<<<kMinBlocks, 256, 0, st>>>(possibility, n, pv, pi);
    O3DML_LAUNCH_CHECK();
    possibility_min_final_kernel<<<1, 64, 0, st>>>(pv, pi, n, sub, argmin, center, host_min);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_randla_possibility_min_workspace_size() {
    return ws_bytes<double>(kMinBlocks) + ws_bytes<int64_t>(kMinBlocks);
}

O3DML_API int o3dml_random_permute(const int64_t* src, int64_t n, uint64_t seed, int64_t* dst, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "random_permute: n out of range");
    if (n == 0) return 0;
    int bits = 1;
    while ((int64_t(1) << bits) < n) ++bits;
    const int half = (bits + 1) / 2;
    random_permute_kernel<<<stream_grid(n, 256), 256, 0, as_stream(stream)>>>(src, n, half, seed, nullptr, dst);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

__global__ void seed_advance_kernel(uint64_t* seed_state) {
    if (threadIdx.x == 0) seed_state[1] += 1;
}

// The same permutation keyed from device state (seed_state u64 [2]: base,
// counter; key = splitmix64(base + counter)), then counter += 1 — no host
// argument changes between patches, so the patch step can be a replayed graph.
O3DML_API int o3dml_random_permute_dev(const int64_t* src, int64_t n, uint64_t* seed_state, int64_t* dst,
                                       void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "random_permute: n out of range");
    hipStream_t st = as_stream(stream);
    if (n > 0) {
        int bits = 1;
        while ((int64_t(1) << bits) < n) ++bits;
        random_permute_kernel<<<stream_grid(n, 256), 256, 0, st>>>(src, n, (bits + 1) / 2, 0, seed_state, dst);
        O3DML_LAUNCH_CHECK();
    }
    seed_advance_kernel<<<1, 64, 0, st>>>(seed_state);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_randla_update_probs(const float* probs, const int64_t* idxs, const uint8_t* keep, int64_t n,
                                        int c, double smooth, int store_half, void* test_probs, void* stream) {
    O3DML_GUARD_BEGIN
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    const unsigned g = stream_grid(n * c, 256);
    // (1 - smooth) in double, then float32: the reference's Python scalar
    // times a float32 array (0.050000000000000044 -> 0.05f)
    const float new_w = static_cast<float>(1.0 - smooth);
    if (store_half) {  // the Python scalar becomes the store's dtype (numpy), the new term stays f32
        const float s16 = __half2float(__float2half_rn(static_cast<float>(smooth)));
        update_probs_kernel<true><<<g, 256, 0, st>>>(probs, idxs, keep, n, c, s16, new_w, test_probs);
    } else {
        update_probs_kernel<false><<<g, 256, 0, st>>>(probs, idxs, keep, n, c, static_cast<float>(smooth), new_w,
                                                      test_probs);
    }
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_randla_patch_workspace_size(int64_t n) {
    return ws_bytes<float>(3 * kPatchBlocks) + ws_bytes<float>(n);
}

O3DML_API int o3dml_randla_patch_update(const float* sub, const int64_t* idxs, int64_t n, const float* center,
                                        const uint8_t* keep, double* possibility, float* pc, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    float* partials = ws.take<float>(3 * kPatchBlocks);
    float* d = ws.take<float>(n);
    patch_prep_kernel<<<kPatchBlocks, 256, 0, st>>>(sub, idxs, n, center, pc, d, partials);
    O3DML_LAUNCH_CHECK();
    patch_apply_kernel<<<kPatchBlocks, 256, 0, st>>>(idxs, n, keep, partials, d, possibility, pc);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// levels: nlev (<= 4) entries each of rs (nlev + 1), nxt, srs (host arrays)
O3DML_API int o3dml_randla_up_from_knn(int32_t* nb, int k, const float* cat, int nlev, const int64_t* rs,
                                       const int64_t* nxt, const int64_t* srs, int64_t* up, void* workspace,
                                       size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(nlev >= 1 && nlev <= 4 && k >= 1, "up_from_knn: 1..4 levels, k >= 1");
    hipStream_t st = as_stream(stream);
    UpLevels L{};
    L.nlev = nlev;
    for (int i = 0; i <= nlev; ++i) L.rs[i] = rs[i];
    for (int i = 0; i < nlev; ++i) {
        L.nxt[i] = nxt[i];
        L.srs[i] = srs[i];
        O3DML_REQUIRE(nxt[i] <= rs[i + 1] - rs[i], "up_from_knn: level %d prefix longer than the level", i);
    }
    const int64_t total = rs[nlev];
    if (total == 0) return 0;
    Workspace ws(workspace, workspace_bytes);
    uint32_t* cntr = ws.take<uint32_t>(1);
    uint32_t* list = ws.take<uint32_t>(total);
    fill_async(cntr, 0, sizeof(uint32_t), st);
    up_from_knn_kernel<<<stream_grid(total, 256), 256, 0, st>>>(nb, k, total, L, up, list, cntr);
    O3DML_LAUNCH_CHECK();
    up_fallback_kernel<<<512, 256, 0, st>>>(cat, L, list, cntr, up);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_randla_up_workspace_size(int64_t total) { return ws_bytes<uint32_t>(1) + ws_bytes<uint32_t>(total); }
