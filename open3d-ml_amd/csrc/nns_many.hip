// nns_many.hip — neighbour searches whose rows are long or of per-query size:
//   * ops.radius_search / layers.RadiusSearch (per-query radius; Open3D ml ops
//     API, SURVEY.md §2.2 ★ — no reference model calls it), rows in ascending
//     (distance, index) order;
//   * ops.knn_search for 64 < k <= 2048 without a host loop (the
//     k <= 64 kernels are in nns_knn.hip; larger k, e.g. the sampler's
//     45,056-point patch crop of SURVEY A2, keeps the per-query path there).
//
// Both run on the dense per-batch grid of grid.hpp (points re-laid out as
// float4 (x, y, z, id) in cell order).  One 256-thread workgroup per query:
// its 4 waves take the (y, z) rows of the query's cell cube in turn, a row's
// cells being one contiguous run of the cell-sorted points; every lane tests
// its points and the passing ones are appended to an LDS list of 64-bit
// (distance bits, id) keys (a distance >= +0 orders as its unsigned bits, so
// the unsigned key order is the (distance, index) order) by one LDS atomic
// per wave and step; a bitonic network over the list then gives the row.
//
// radius: the cube covers q +- r (with a margin against float rounding: every
// point that passes the float test lies inside it); count pass, scan, fill.
// Rows longer than the LDS list are written unsorted straight into place and
// sorted afterwards (o3dml_radius_search_sort_long_rows, u64 radix sort).
// kNN: the smallest cell cube C_R around the query holding >= k points is
// collected and sorted; its k-th key bounds the k-th neighbour's key, so the
// answer lies in the ball of that distance — done if the ball is inside C_R
// (the same conservative lower bound on the unvisited region as nns_knn.hip),
// else the cube around the ball is collected with keys <= that bound and
// sorted.  A query whose candidates exceed the list is listed for the
// per-query path.
#include <algorithm>

#include "grid.hpp"

namespace o3dml {

constexpr int kManyThreads = 256;
constexpr int kManyCapSmall = 1024;  // 8 KiB of keys: 8 workgroups per CU
constexpr int kManyCapLarge = 8192;  // 64 KiB: 2 workgroups per CU

__device__ __forceinline__ uint64_t many_key(float d, uint32_t id) {
    return (static_cast<uint64_t>(__float_as_uint(d)) << 32) | id;
}

template <int METRIC>
__device__ __forceinline__ float many_threshold(float r) {
    return METRIC == kL2 ? r * r : r;
}

// Inclusive cell range of one axis covering [c - w, c + w] (w >= 0), margins
// for the float rounding of the distance test and of q -+ w.
__device__ __forceinline__ void axis_range(float c, float w, float o, float inv_h, int n, int& a, int& b) {
    const float m = w * 1.00001f + 1e-6f * fabsf(c) + 1e-30f;
    a = grid_axis(c - m, o, inv_h, n);
    b = grid_axis(c + m, o, inv_h, n);
}

// Bitonic sort of keys[0, N) (N a power of two) by the whole workgroup.
__device__ __forceinline__ void block_bitonic(uint64_t* keys, int N) {
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < N; i += kManyThreads) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = keys[i], b = keys[ixj];
                    if ((a > b) == ((i & k) == 0)) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// Streams the cube [xa, xb] x [ya, yb] x [za, zb] of grid g; f(float4 p) is
// called for every point (each wave takes every 4th (y, z) row, lanes stride
// the row's run).  f returns the key to append or ~0 to skip; appended keys
// get positions from the LDS counter *cnt and go to sink(pos, key).
template <class Test, class Sink>
__device__ __forceinline__ void stream_cube(const float4* __restrict__ sorted, const uint32_t* __restrict__ splits,
                                            const GridBatch& g, int xa, int xb, int ya, int yb, int za, int zb,
                                            uint32_t* cnt, Test test, Sink sink) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ny = yb - ya + 1, rows = ny * (zb - za + 1);
    for (int rr = wv; rr < rows; rr += kManyThreads / 64) {
        const int z = za + rr / ny, y = ya + rr % ny;
        const uint32_t c = g.offset + static_cast<uint32_t>(g.dx * (y + g.dy * z));
        const uint32_t s = splits[c + xa], e = splits[c + xb + 1];
        for (uint32_t j0 = s; j0 < e; j0 += 64) {
            const uint32_t j = j0 + lane;
            uint64_t key = ~0ull;
            if (j < e) key = test(sorted[j]);
            const bool take = key != ~0ull;
            const uint64_t bal = __builtin_amdgcn_ballot_w64(take);
            if (!bal) continue;
            uint32_t base = 0;
            if (lane == __builtin_ctzll(bal)) base = atomicAdd(cnt, static_cast<uint32_t>(__popcll(bal)));
            base = __builtin_amdgcn_readfirstlane(__shfl(base, __builtin_ctzll(bal), 64));
            if (take)
                sink(base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u)),
                     key);
        }
    }
}

// MODE 0: radius count (counts[q], atomic max into *max_row); MODE 1: radius
// fill into [rs[q], rs[q+1]) — sorted through LDS when the row fits CAP, else
// unsorted straight into place (sorted by the long-row pass).
template <int CAP, int METRIC, bool IGNORE, int MODE>
__global__ void __launch_bounds__(kManyThreads) radius_kernel(
        const float4* __restrict__ sorted, const uint32_t* __restrict__ splits, const GridBatch* __restrict__ grids,
        const float* __restrict__ queries, const float* __restrict__ radii, int64_t m,
        const int64_t* __restrict__ qrs, int nb, int64_t* __restrict__ counts, int64_t* __restrict__ max_row,
        const int64_t* __restrict__ rs, int bits, void* __restrict__ out_idx, float* __restrict__ out_dist,
        int normalize) {
    __shared__ uint64_t keys[CAP];
    __shared__ uint32_t s_cnt;
    for (int64_t q = blockIdx.x; q < m; q += gridDim.x) {
        const GridBatch g = grids[batch_of(q, qrs, nb)];
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        const float r = radii[q];
        const float thr = many_threshold<METRIC>(r);
        int xa, xb, ya, yb, za, zb;
        axis_range(qx, r, g.ox, g.inv_h, g.dx, xa, xb);
        axis_range(qy, r, g.oy, g.inv_h, g.dy, ya, yb);
        axis_range(qz, r, g.oz, g.inv_h, g.dz, za, zb);
        const int64_t o = MODE == 1 ? rs[q] : 0;
        const int64_t len = MODE == 1 ? rs[q + 1] - o : 0;
        const bool in_lds = len <= CAP;
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        auto test = [&](const float4& p) -> uint64_t {
            if (IGNORE && p.x == qx && p.y == qy && p.z == qz) return ~0ull;
            const float d = dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz);
            return d <= thr ? many_key(d, __float_as_uint(p.w)) : ~0ull;
        };
        auto write = [&](int64_t pos, uint64_t key) {
            const uint32_t id = static_cast<uint32_t>(key);
            float d = __uint_as_float(static_cast<uint32_t>(key >> 32));
            if (normalize) d = d / thr;
            if (bits == 32)
                static_cast<int32_t*>(out_idx)[pos] = static_cast<int32_t>(id);
            else
                static_cast<int64_t*>(out_idx)[pos] = static_cast<int64_t>(id);
            if (out_dist) out_dist[pos] = d;
        };
        if (m > 0 && g.dx > 0 && (MODE == 0 || len > 0)) {
            if (MODE == 0 || !in_lds)
                stream_cube(sorted, splits, g, xa, xb, ya, yb, za, zb, &s_cnt, test, [&](uint32_t pos, uint64_t key) {
                    if (MODE == 1 && pos < len) write(o + pos, key);
                });
            else
                stream_cube(sorted, splits, g, xa, xb, ya, yb, za, zb, &s_cnt, test, [&](uint32_t pos, uint64_t key) {
                    if (pos < CAP) keys[pos] = key;
                });
        }
        __syncthreads();
        const uint32_t n = MODE == 0 ? s_cnt : min(s_cnt, static_cast<uint32_t>(CAP));  // == len (same test)
        if constexpr (MODE == 0) {
            if (threadIdx.x == 0) {
                counts[q] = n;
                atomicMax(reinterpret_cast<unsigned long long*>(max_row), static_cast<unsigned long long>(n));
            }
        } else if (in_lds && n > 0) {
            int N = 1;
            while (N < static_cast<int>(n)) N <<= 1;
            for (int i = n + threadIdx.x; i < N; i += kManyThreads) keys[i] = ~0ull;
            __syncthreads();
            block_bitonic(keys, N);
            for (int i = threadIdx.x; i < static_cast<int>(n) && i < len; i += kManyThreads) write(o + i, keys[i]);
        }
        __syncthreads();  // keys / s_cnt reused by the next query
    }
}

// kNN, 64 < k <= 2048, into rows [rs[q], rs[q] + min(k, eligible)).
// A query whose candidate list would exceed CAP is listed in over[] for the
// per-query path (nothing written here).
template <int METRIC, bool IGNORE>
__global__ void __launch_bounds__(kManyThreads) knn_many_kernel(
        const float4* __restrict__ sorted, const uint32_t* __restrict__ splits, const GridBatch* __restrict__ grids,
        const float* __restrict__ queries, int64_t m, const int64_t* __restrict__ qrs, int nb, int k,
        const int64_t* __restrict__ rs, int bits, void* __restrict__ out_idx, float* __restrict__ out_dist,
        uint32_t* __restrict__ over, int64_t* __restrict__ n_over) {
    constexpr int CAP = kManyCapLarge;
    __shared__ uint64_t keys[CAP];
    __shared__ uint32_t s_cnt;
    for (int64_t q = blockIdx.x; q < m; q += gridDim.x) {
        const GridBatch g = grids[batch_of(q, qrs, nb)];
        const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
        const int64_t o = rs[q], want = rs[q + 1] - o;  // min(k, eligible points)
        if (want == 0) continue;
        const int cx = grid_axis(qx, g.ox, g.inv_h, g.dx);
        const int cy = grid_axis(qy, g.oy, g.inv_h, g.dy);
        const int cz = grid_axis(qz, g.oz, g.inv_h, g.dz);
        auto write = [&](int64_t pos, uint64_t key) {
            const uint32_t id = static_cast<uint32_t>(key);
            if (bits == 32)
                static_cast<int32_t*>(out_idx)[pos] = static_cast<int32_t>(id);
            else
                static_cast<int64_t*>(out_idx)[pos] = static_cast<int64_t>(id);
            if (out_dist) out_dist[pos] = __uint_as_float(static_cast<uint32_t>(key >> 32));
        };
        bool overflow = false;
        uint64_t bound = ~0ull;  // keys <= bound are kept (pass 2)
        int xa = 0, xb = 0, ya = 0, yb = 0, za = 0, zb = 0;
        bool done = false;
        // pass 1: the smallest cube C_R with >= want eligible points, all of them
        for (int R = 0;; ++R) {
            xa = max(cx - R, 0), xb = min(cx + R, g.dx - 1);
            ya = max(cy - R, 0), yb = min(cy + R, g.dy - 1);
            za = max(cz - R, 0), zb = min(cz + R, g.dz - 1);
            const bool whole = xa == 0 && ya == 0 && za == 0 && xb == g.dx - 1 && yb == g.dy - 1 && zb == g.dz - 1;
            // points in the cube (eligible or not) from the splits alone
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            {
                const int ny = yb - ya + 1, rows = ny * (zb - za + 1);
                uint32_t part = 0;
                for (int rr = threadIdx.x; rr < rows; rr += kManyThreads) {
                    const int z = za + rr / ny, y = ya + rr % ny;
                    const uint32_t c = g.offset + static_cast<uint32_t>(g.dx * (y + g.dy * z));
                    part += splits[c + xb + 1] - splits[c + xa];
                }
                part = wave_sum(part);
                if ((threadIdx.x & 63) == 0 && part) atomicAdd(&s_cnt, part);
            }
            __syncthreads();
            const uint32_t in_cube = s_cnt;
            __syncthreads();
            if (in_cube < want && !whole) continue;
            if (in_cube > CAP) {
                overflow = true;
                break;
            }
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            stream_cube(sorted, splits, g, xa, xb, ya, yb, za, zb, &s_cnt,
                        [&](const float4& p) -> uint64_t {
                            if (IGNORE && p.x == qx && p.y == qy && p.z == qz) return ~0ull;
                            return many_key(dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz), __float_as_uint(p.w));
                        },
                        [&](uint32_t pos, uint64_t key) {
                            if (pos < CAP) keys[pos] = key;  // pos < in_cube <= CAP
                        });
            __syncthreads();
            const uint32_t n = min(s_cnt, static_cast<uint32_t>(CAP));
            if (n < want && !whole) {  // identical points ignored: widen
                __syncthreads();
                continue;
            }
            int N = 1;
            while (N < static_cast<int>(n)) N <<= 1;
            for (int i = n + threadIdx.x; i < N; i += kManyThreads) keys[i] = ~0ull;
            __syncthreads();
            block_bitonic(keys, N);
            bound = keys[static_cast<int>(min<int64_t>(want, static_cast<int64_t>(n))) - 1];  // n >= want here (whole grid: n == want)
            if (whole) {
                done = true;
                break;
            }
            // done if every unvisited point is farther than the want-th key's
            // distance (conservative lower bound as in nns_knn.hip)
            const float kd = __uint_as_float(static_cast<uint32_t>(bound >> 32));
            float lb = INFINITY;
            if (xa > 0) lb = fminf(lb, qx - (g.ox + static_cast<float>(xa) * g.h));
            if (xb < g.dx - 1) lb = fminf(lb, (g.ox + static_cast<float>(xb + 1) * g.h) - qx);
            if (ya > 0) lb = fminf(lb, qy - (g.oy + static_cast<float>(ya) * g.h));
            if (yb < g.dy - 1) lb = fminf(lb, (g.oy + static_cast<float>(yb + 1) * g.h) - qy);
            if (za > 0) lb = fminf(lb, qz - (g.oz + static_cast<float>(za) * g.h));
            if (zb < g.dz - 1) lb = fminf(lb, (g.oz + static_cast<float>(zb + 1) * g.h) - qz);
            lb = lb - 1e-3f * g.h - 1e-6f * (fabsf(qx) + fabsf(qy) + fabsf(qz));
            if (lb > 0.f && kd < (METRIC == kL2 ? lb * lb : lb)) done = true;
            // else: the ball of distance kd around q (for L2 radius sqrt(kd))
            if (!done) {
                const float w = METRIC == kL2 ? sqrtf(kd) : kd;
                axis_range(qx, w, g.ox, g.inv_h, g.dx, xa, xb);
                axis_range(qy, w, g.oy, g.inv_h, g.dy, ya, yb);
                axis_range(qz, w, g.oz, g.inv_h, g.dz, za, zb);
            }
            break;
        }
        if (!overflow && !done) {
            // pass 2: every point of the ball's cube with key <= bound
            __syncthreads();
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            stream_cube(sorted, splits, g, xa, xb, ya, yb, za, zb, &s_cnt,
                        [&](const float4& p) -> uint64_t {
                            if (IGNORE && p.x == qx && p.y == qy && p.z == qz) return ~0ull;
                            const uint64_t key =
                                    many_key(dist_metric<METRIC>(p.x, p.y, p.z, qx, qy, qz), __float_as_uint(p.w));
                            return key <= bound ? key : ~0ull;
                        },
                        [&](uint32_t pos, uint64_t key) {
                            if (pos < CAP) keys[pos] = key;
                        });
            __syncthreads();
            const uint32_t n = s_cnt;
            if (n > CAP) {
                overflow = true;
            } else {
                int N = 1;
                while (N < static_cast<int>(n)) N <<= 1;
                for (int i = n + threadIdx.x; i < N; i += kManyThreads) keys[i] = ~0ull;
                __syncthreads();
                block_bitonic(keys, N);
            }
        }
        if (overflow) {
            if (threadIdx.x == 0)
                over[atomicAdd(reinterpret_cast<unsigned long long*>(n_over), 1ull)] = static_cast<uint32_t>(q);
        } else {
            for (int i = threadIdx.x; i < want && i < CAP; i += kManyThreads) write(o + i, keys[i]);
        }
        __syncthreads();
    }
}

// Eligible points of each query for k > 64: N_b, minus (ignore_query_point)
// the points at the query's exact position — all in the query's grid cell.
__global__ void many_knn_counts_kernel(const float4* __restrict__ sorted, const uint32_t* __restrict__ splits,
                                       const GridBatch* __restrict__ grids, const float* __restrict__ queries,
                                       int64_t m, const int64_t* __restrict__ prs, const int64_t* __restrict__ qrs,
                                       int nb, int64_t k, int ignore, int64_t* __restrict__ counts) {
    for (int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; q < m;
         q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(q, qrs, nb);
        int64_t n = prs[b + 1] - prs[b];
        if (ignore && n > 0) {
            const GridBatch g = grids[b];
            const float qx = queries[3 * q], qy = queries[3 * q + 1], qz = queries[3 * q + 2];
            const int cx = grid_axis(qx, g.ox, g.inv_h, g.dx);
            const int cy = grid_axis(qy, g.oy, g.inv_h, g.dy);
            const int cz = grid_axis(qz, g.oz, g.inv_h, g.dz);
            const uint32_t c = g.offset + static_cast<uint32_t>(cx + g.dx * (cy + g.dy * cz));
            for (uint32_t j = splits[c]; j < splits[c + 1]; ++j) {
                const float4 p = sorted[j];
                n -= (p.x == qx && p.y == qy && p.z == qz) ? 1 : 0;
            }
        }
        counts[q] = n < k ? n : k;
    }
}

// keys of rows to be sorted by (distance, index): one row [s, s + n)
__global__ void row_keys_kernel(const void* __restrict__ idx, const float* __restrict__ dist, int bits, int64_t s,
                                int64_t n, uint64_t* __restrict__ keys) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t id = bits == 32 ? static_cast<uint32_t>(static_cast<const int32_t*>(idx)[s + j])
                                       : static_cast<uint32_t>(static_cast<const int64_t*>(idx)[s + j]);
        keys[j] = many_key(dist[s + j], id);
    }
}

__global__ void row_write_kernel(const uint64_t* __restrict__ keys, int64_t s, int64_t n, int bits,
                                 void* __restrict__ idx, float* __restrict__ dist, int write_dist) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t id = static_cast<uint32_t>(keys[j]);
        if (bits == 32)
            static_cast<int32_t*>(idx)[s + j] = static_cast<int32_t>(id);
        else
            static_cast<int64_t*>(idx)[s + j] = id;
        if (write_dist) dist[s + j] = __uint_as_float(static_cast<uint32_t>(keys[j] >> 32));
    }
}

// Workspace of the radius search (count and fill share it; same layout).
struct RadiusPlan {
    int64_t* scalars;  // [0] max row length
    int64_t* counts;   // [M]
    uint64_t* rkeys;   // [N]
    uint64_t* rskeys;  // [N]
    uint32_t* rvals;   // [N]
    GridIndex gi;
};

static constexpr double kRadiusTarget = 8.0;  // points per grid cell (uniform-fill plan)
static constexpr double kManyCapFactor = 2.0;

static RadiusPlan take_radius_plan(Workspace& ws, const float* pts, int64_t n, int64_t m, const int64_t* prs, int nb,
                                   hipStream_t st, bool build) {
    RadiusPlan p;
    p.scalars = ws.take<int64_t>(4);
    p.counts = ws.take<int64_t>(m);
    p.rkeys = ws.take<uint64_t>(n);
    p.rskeys = ws.take<uint64_t>(n);
    p.rvals = ws.take<uint32_t>(n);
    if (build) {
        p.gi = build_grid(pts, n, prs, nb, kRadiusTarget, kManyCapFactor, ws, st);
    } else {  // same takes as build_grid, nothing launched
        p.gi.params = ws.take<GridBatch>(nb);
        ws.take<float>(6 * nb);
        p.gi.cells = grid_cells_cap(n, nb, kManyCapFactor);
        p.gi.splits = ws.take<uint32_t>(p.gi.cells + 1);
        p.gi.sorted = ws.take<float4>(n);
    }
    return p;
}

template <int CAP, int MODE>
static void launch_radius(int metric, bool ignore, hipStream_t st, const RadiusPlan& p, const float* queries,
                          const float* radii, int64_t m, const int64_t* qrs, int nb, const int64_t* rs, int bits,
                          void* oi, float* od, int normalize) {
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(m, 1 << 20)));
#define O3DML_RAD(M, I)                                                                                        \
    radius_kernel<CAP, M, I, MODE><<<grid, kManyThreads, 0, st>>>(p.gi.sorted, p.gi.splits, p.gi.params,       \
                                                                  queries, radii, m, qrs, nb, p.counts,        \
                                                                  p.scalars, rs, bits, oi, od, normalize)
    if (metric == kL2) {
        if (ignore) O3DML_RAD(kL2, true); else O3DML_RAD(kL2, false);
    } else if (metric == kL1) {
        if (ignore) O3DML_RAD(kL1, true); else O3DML_RAD(kL1, false);
    } else {
        if (ignore) O3DML_RAD(kLinf, true); else O3DML_RAD(kLinf, false);
    }
#undef O3DML_RAD
    O3DML_LAUNCH_CHECK();
}

static size_t radius_plan_bytes(int64_t n, int64_t m, int64_t nb) {
    return ws_bytes<int64_t>(4) + ws_bytes<int64_t>(m) + 2 * ws_bytes<uint64_t>(n) +
           ws_bytes<uint32_t>(n) + grid_workspace_bytes(n, static_cast<int>(nb), kManyCapFactor);
}

// ---- batched kNN, 64 < k <= 2048 (kManyKnnMaxK, called from nns_knn.hip) ----
size_t knn_many_workspace_bytes(int64_t n, int64_t m, int64_t k, int64_t nb) {
    return ws_bytes<int64_t>(4) + ws_bytes<uint32_t>(m) + ws_bytes<int64_t>(m) + ws_bytes<int64_t>(nb + 1) +
           prim::scan_workspace_bytes(m) + grid_workspace_bytes(n, static_cast<int>(nb), kManyCapFactor);
}

static double knn_many_target(int64_t k) { return std::max(2.0, static_cast<double>(k) / 8.0); }

struct KnnManyPlan {
    int64_t* scalars;  // [0] overflow count
    uint32_t* over;    // [M]
    int64_t* counts;   // [M]
    int64_t* prs;      // [B + 1] device copy of the point row splits (the overflow path of the fill)
    GridIndex gi;
};

static KnnManyPlan take_knn_many(Workspace& ws, const float* pts, int64_t n, int64_t m, int64_t k,
                                 const int64_t* prs, int nb, hipStream_t st, bool build) {
    KnnManyPlan p;
    p.scalars = ws.take<int64_t>(4);
    p.over = ws.take<uint32_t>(m);
    p.counts = ws.take<int64_t>(m);
    p.prs = ws.take<int64_t>(nb + 1);
    if (build) {
        p.gi = build_grid(pts, n, prs, nb, knn_many_target(k), kManyCapFactor, ws, st);
    } else {
        p.gi.params = ws.take<GridBatch>(nb);
        ws.take<float>(6 * nb);
        p.gi.cells = grid_cells_cap(n, nb, kManyCapFactor);
        p.gi.splits = ws.take<uint32_t>(p.gi.cells + 1);
        p.gi.sorted = ws.take<float4>(n);
    }
    return p;
}

void knn_many_count(const float* pts, int64_t n, const float* queries, int64_t m, int64_t k, int nb,
                    const int64_t* prs, const int64_t* qrs, int ignore, int64_t* rs, Workspace ws, hipStream_t st) {
    KnnManyPlan p = take_knn_many(ws, pts, n, m, k, prs, nb, st, true);
    fill_async(p.scalars, 0, 4 * sizeof(int64_t), st);
    fill_async(rs, 0, sizeof(int64_t), st);
    copy_async(p.prs, prs, sizeof(int64_t) * (nb + 1), st);
    if (m == 0) return;
    many_knn_counts_kernel<<<stream_grid(m, 256), 256, 0, st>>>(p.gi.sorted, p.gi.splits, p.gi.params, queries, m,
                                                               prs, qrs, nb, k, ignore, p.counts);
    O3DML_LAUNCH_CHECK();
    prim::scan<int64_t, int64_t>(p.counts, rs + 1, m, true, ws, st);
}

void topk_overflow(const float* pts, const float* queries, const int64_t* prs, const int64_t* qrs, int nb,
                   int metric, int ignore, const uint32_t* over, const int64_t* n_over, const int64_t* rs, int bits,
                   void* oi, float* od, int64_t max_over, hipStream_t st);

// Fills the rows; the queries whose candidates overflow the LDS list are
// listed on the device and done by nns_topk.hip's radix selection over their
// whole batch item, queued right behind (no host read of the count).
void knn_many_fill(const float* pts, int64_t n, const float* queries, int64_t m, int64_t k, int nb,
                   const int64_t* qrs, int metric, int ignore, const int64_t* rs, int bits, void* oi, float* od,
                   Workspace ws, hipStream_t st) {
    KnnManyPlan p = take_knn_many(ws, pts, n, m, k, nullptr, nb, st, false);
    if (m == 0) return;
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(m, 1 << 20)));
#define O3DML_KM(M, I)                                                                                        \
    knn_many_kernel<M, I><<<grid, kManyThreads, 0, st>>>(p.gi.sorted, p.gi.splits, p.gi.params, queries, m,    \
                                                        qrs, nb, static_cast<int>(k), rs, bits, oi, od, p.over, \
                                                        p.scalars)
    if (metric == kL2) {
        if (ignore) O3DML_KM(kL2, true); else O3DML_KM(kL2, false);
    } else if (metric == kL1) {
        if (ignore) O3DML_KM(kL1, true); else O3DML_KM(kL1, false);
    } else {
        if (ignore) O3DML_KM(kLinf, true); else O3DML_KM(kLinf, false);
    }
#undef O3DML_KM
    O3DML_LAUNCH_CHECK();
    topk_overflow(pts, queries, p.prs, qrs, nb, metric, ignore, p.over, p.scalars, rs, bits, oi, od, m, st);
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_radius_search_workspace_size(int64_t n_points, int64_t n_queries, int64_t n_batch) {
    return radius_plan_bytes(n_points, n_queries, n_batch) +
           std::max(prim::scan_workspace_bytes(n_queries), prim::radix_sort_workspace_bytes<uint64_t>(n_points));
}

O3DML_API int o3dml_radius_search_count(const float* points, int64_t n_points, const float* queries,
                                        int64_t n_queries, const float* radii, int64_t n_batch,
                                        const int64_t* points_row_splits, const int64_t* queries_row_splits,
                                        int metric, int ignore_query_point, int64_t* neighbors_row_splits,
                                        void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(metric >= 0 && metric <= 2, "metric must be L1(0), L2(1) or Linf(2)");
    O3DML_REQUIRE(n_batch >= 1, "need at least one batch item");
    O3DML_REQUIRE(n_points < (int64_t(1) << 31) && n_queries < (int64_t(1) << 31), "too many points");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    RadiusPlan p = take_radius_plan(ws, points, n_points, n_queries, points_row_splits, static_cast<int>(n_batch), st,
                                    true);
    fill_async(p.scalars, 0, 4 * sizeof(int64_t), st);
    fill_async(neighbors_row_splits, 0, sizeof(int64_t), st);
    if (n_queries == 0) return 0;
    if (n_points == 0) {
        fill_async(neighbors_row_splits, 0, sizeof(int64_t) * (n_queries + 1), st);
        return 0;
    }
    launch_radius<1, 0>(metric, ignore_query_point != 0, st, p, queries, radii, n_queries, queries_row_splits,
                        static_cast<int>(n_batch), nullptr, 32, nullptr, nullptr, 0);
    prim::scan<int64_t, int64_t>(p.counts, neighbors_row_splits + 1, n_queries, true, ws, st);
    O3DML_GUARD_END
}

// [total, max row length] into a host (pinned) buffer
__global__ void radius_totals_kernel(const int64_t* __restrict__ rs, int64_t m, const int64_t* __restrict__ scalars,
                                     int64_t* __restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = rs[m];
        out[1] = scalars[0];
    }
}

O3DML_API int o3dml_radius_search_totals(const int64_t* neighbors_row_splits, int64_t n_queries, void* workspace,
                                         int64_t* totals, void* stream) {
    O3DML_GUARD_BEGIN
    radius_totals_kernel<<<1, 64, 0, as_stream(stream)>>>(neighbors_row_splits, n_queries,
                                                         static_cast<const int64_t*>(workspace), totals);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_radius_search_fill(const float* points, int64_t n_points, const float* queries,
                                       int64_t n_queries, const float* radii, int64_t n_batch,
                                       const int64_t* queries_row_splits, int metric, int ignore_query_point,
                                       int normalize_distances, const int64_t* neighbors_row_splits,
                                       int64_t max_row, int index_bits, void* neighbors_index,
                                       float* neighbors_distance, void* workspace, size_t workspace_bytes,
                                       void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(index_bits == 32 || index_bits == 64, "index_bits must be 32 or 64");
    if (n_queries == 0 || n_points == 0) return 0;
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    RadiusPlan p = take_radius_plan(ws, points, n_points, n_queries, nullptr, static_cast<int>(n_batch), st, false);
    // rows longer than the large list are written unsorted, with their
    // distances (the caller passes a distance buffer then), and sorted by
    // o3dml_radius_search_sort_long_rows
    O3DML_REQUIRE(max_row <= kManyCapLarge || neighbors_distance, "rows longer than %d need a distance buffer",
                  kManyCapLarge);
    if (max_row <= kManyCapSmall)
        launch_radius<kManyCapSmall, 1>(metric, ignore_query_point != 0, st, p, queries, radii, n_queries,
                                        queries_row_splits, static_cast<int>(n_batch), neighbors_row_splits,
                                        index_bits, neighbors_index, neighbors_distance, normalize_distances);
    else
        launch_radius<kManyCapLarge, 1>(metric, ignore_query_point != 0, st, p, queries, radii, n_queries,
                                        queries_row_splits, static_cast<int>(n_batch), neighbors_row_splits,
                                        index_bits, neighbors_index, neighbors_distance, normalize_distances);
    O3DML_GUARD_END
}

// Sorts the rows longer than the LDS list (written unsorted by the fill) by
// (distance, index).  neighbors_distance holds the (possibly normalized)
// distances of those rows; normalization is monotone, so the order is the
// same.  rows_host: the host copy of the row splits.
O3DML_API int o3dml_radius_search_sort_long_rows(int64_t n_points, int64_t n_queries, int64_t n_batch,
                                                 const int64_t* rows_host, int index_bits, void* neighbors_index,
                                                 float* neighbors_distance, void* workspace, size_t workspace_bytes,
                                                 void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    RadiusPlan p = take_radius_plan(ws, nullptr, n_points, n_queries, nullptr, static_cast<int>(n_batch), st, false);
    for (int64_t q = 0; q < n_queries; ++q) {
        const int64_t s = rows_host[q], len = rows_host[q + 1] - s;
        if (len <= kManyCapLarge) continue;
        O3DML_REQUIRE(neighbors_distance, "long rows need the distances");
        row_keys_kernel<<<stream_grid(len, 256), 256, 0, st>>>(neighbors_index, neighbors_distance, index_bits, s,
                                                              len, p.rkeys);
        O3DML_LAUNCH_CHECK();
        Workspace sws = ws;
        prim::radix_sort_pairs<uint64_t>(p.rkeys, nullptr, p.rskeys, p.rvals, len, 64, sws, st);
        row_write_kernel<<<stream_grid(len, 256), 256, 0, st>>>(p.rskeys, s, len, index_bits, neighbors_index,
                                                               neighbors_distance, 1);
        O3DML_LAUNCH_CHECK();
    }
    O3DML_GUARD_END
}
