// voxel.hip — voxelization and grid subsampling.
//   o3dml_voxelize*       replaces open3d.ml.torch.ops.voxelize
//                         (point_pillars.py:352-357, sparseconvnet.py:293-298)
//   o3dml_grid_subsample* replaces open3d.ml.contrib.subsample / subsample_batch
//                         (dataprocessing.py:33-49 <- randlanet.py:133-139,
//                          kpconv.py:2099-2155 <- concat_batcher.py:245-247)
// Both are: key per point -> stable LSD radix sort (key, id) -> segment heads
// -> scans -> per-segment outputs.  Stability keeps the points of a voxel /
// cell in input order, so per-cell sums run left to right exactly as the
// oracle's and the results are bit-identical.  All HBM-streaming, integer/byte
// work (no MFMA).
#include <limits>
#include <cmath>
#include <vector>

#include "grid.hpp"

namespace o3dml {

constexpr int kMaxVoxDim = 8;

struct VoxParams {
    double mn[kMaxVoxDim];
    double inv[kMaxVoxDim];
    int64_t ext[kMaxVoxDim];
    int64_t stride[kMaxVoxDim];
    int64_t batch_hash;
    int64_t invalid_key;
    int ndim;
    int nb;
};

// OR of a block's keys and of their complements into or_and[0..1] (zeroed by
// the caller): one atomic pair per block, only for bits not yet recorded.
// 256 threads per block.
__device__ __forceinline__ void or_and_block(uint64_t o1, uint64_t o0, unsigned long long* __restrict__ or_and) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        o1 |= static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(o1), d, 64));
        o0 |= static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(o0), d, 64));
    }
    __shared__ unsigned long long part[2][4];
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = o1;
        part[1][threadIdx.x >> 6] = o0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < static_cast<int>(blockDim.x >> 6); ++k) {
            o1 |= part[0][k];
            o0 |= part[1][k];
        }
        const unsigned long long c1 = __hip_atomic_load(&or_and[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c0 = __hip_atomic_load(&or_and[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o1 & ~c1) atomicOr(&or_and[0], static_cast<unsigned long long>(o1));
        if (o0 & ~c0) atomicOr(&or_and[1], static_cast<unsigned long long>(o0));
    }
}

// or_and (nullable, zeroed): OR of the keys and of their complements — the
// bits that vary among them, so the radix sort runs only the digits that do
// (device-planned passes, as calculate_grid); one atomic pair per block, and
// only for bits not yet recorded.  256 threads per block.
__global__ void __launch_bounds__(256) vox_keys_kernel(const float* __restrict__ pts, int64_t n,
                                                       const int64_t* __restrict__ rs, VoxParams vp,
                                                       uint64_t* __restrict__ keys,
                                                       unsigned long long* __restrict__ or_and) {
    uint64_t o1 = 0, o0 = 0;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(i, rs, vp.nb);
        int64_t key = static_cast<int64_t>(b) * vp.batch_hash;
        bool ok = true;
        for (int d = 0; d < vp.ndim; ++d) {
            const double c = floor((static_cast<double>(pts[i * vp.ndim + d]) - vp.mn[d]) * vp.inv[d]);
            if (!(c >= 0.0 && c < static_cast<double>(vp.ext[d]))) {
                ok = false;
                break;
            }
            key += static_cast<int64_t>(c) * vp.stride[d];
        }
        const uint64_t kv = static_cast<uint64_t>(ok ? key : vp.invalid_key);
        keys[i] = kv;
        o1 |= kv;
        o0 |= ~kv;
    }
    if (!or_and) return;  // uniform
    or_and_block(o1, o0, or_and);
}

// head[j] = 1 where a new valid segment starts; also records n_valid.
__global__ void seg_heads_kernel(const uint64_t* __restrict__ sk, int64_t n, uint64_t invalid, int64_t* __restrict__ head,
                                 int64_t* __restrict__ n_valid) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const bool valid = sk[j] != invalid;
        head[j] = (valid && (j == 0 || sk[j] != sk[j - 1])) ? 1 : 0;
        if (valid && (j == n - 1 || sk[j + 1] == invalid)) *n_valid = j + 1;
    }
}

__global__ void seg_start_kernel(const int64_t* __restrict__ head, const int64_t* __restrict__ incl, int64_t n,
                                 int64_t* __restrict__ start) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x)
        if (head[j]) start[incl[j] - 1] = j;
}

// bfirst[b] = first segment of batch item b (segments sorted by batch).
__global__ void seg_batch_first_kernel(const uint64_t* __restrict__ sk, const int64_t* __restrict__ start,
                                       const int64_t* __restrict__ incl, int64_t n, int nb, int shift_or_div_is_shift,
                                       uint64_t div, int64_t* __restrict__ bfirst) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    if (nseg == 0) {
        if (blockIdx.x == 0)
            for (int b = threadIdx.x; b <= nb; b += blockDim.x) bfirst[b] = 0;
        return;
    }
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nseg;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        auto bat = [&](int64_t s) {
            const uint64_t k = sk[start[s]];
            return static_cast<int64_t>(shift_or_div_is_shift ? (k >> div) : (k / div));
        };
        const int64_t b = bat(v);
        const int64_t bp = v == 0 ? -1 : bat(v - 1);
        for (int64_t bb = bp + 1; bb <= b; ++bb) bfirst[bb] = v;
        if (v == nseg - 1)
            for (int64_t bb = b + 1; bb <= nb; ++bb) bfirst[bb] = nseg;
    }
}

// keep[v] (0/1) and npts[v] for voxelize caps.
__global__ void vox_caps_kernel(const uint64_t* __restrict__ sk, const int64_t* __restrict__ start,
                                const int64_t* __restrict__ incl, const int64_t* __restrict__ n_valid, int64_t n,
                                const int64_t* __restrict__ bfirst, int64_t batch_hash, int64_t max_voxels,
                                int64_t max_ppv, int64_t* __restrict__ keep, int64_t* __restrict__ npts) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nseg;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t j0 = start[v];
        const int64_t j1 = v + 1 < nseg ? start[v + 1] : *n_valid;
        const int64_t b = static_cast<int64_t>(sk[j0]) / batch_hash;
        const bool k = (v - bfirst[b]) < max_voxels;
        keep[v] = k ? 1 : 0;
        const int64_t c = j1 - j0;
        npts[v] = k ? (c < max_ppv ? c : max_ppv) : 0;
    }
}

__global__ void vox_totals_kernel(const int64_t* __restrict__ incl, int64_t n, const int64_t* __restrict__ keep_incl,
                                  const int64_t* __restrict__ npts_incl, int64_t* __restrict__ out /*[Vall,V,P]*/) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int64_t nseg = n > 0 ? incl[n - 1] : 0;
        out[0] = nseg;
        out[1] = nseg > 0 ? keep_incl[nseg - 1] : 0;
        out[2] = nseg > 0 ? npts_incl[nseg - 1] : 0;
    }
}

__global__ void vox_fill_kernel(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sidx,
                                const int64_t* __restrict__ start, const int64_t* __restrict__ incl, int64_t n,
                                const int64_t* __restrict__ keep, const int64_t* __restrict__ keep_incl,
                                const int64_t* __restrict__ npts, const int64_t* __restrict__ npts_incl, VoxParams vp,
                                int32_t* __restrict__ coords, int64_t* __restrict__ pidx, int64_t* __restrict__ prs) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nseg;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        if (!keep[v]) continue;
        const int64_t k = keep_incl[v] - 1;
        const int64_t j0 = start[v];
        const int64_t key = static_cast<int64_t>(sk[j0]);
        int64_t rem = key % vp.batch_hash;
        for (int d = vp.ndim - 1; d >= 0; --d) {
            coords[k * vp.ndim + d] = static_cast<int32_t>(rem / vp.stride[d]);
            rem %= vp.stride[d];
        }
        const int64_t c = npts[v];
        const int64_t o = npts_incl[v] - c;
        prs[k] = o;
        for (int64_t j = 0; j < c; ++j) pidx[o + j] = sidx[j0 + j];
    }
}

__global__ void batch_splits_kernel(const int64_t* __restrict__ bfirst, const int64_t* __restrict__ keep_incl, int nb,
                                    const int64_t* __restrict__ totals, int64_t* __restrict__ bsplits,
                                    int64_t* __restrict__ prs, int64_t V_host) {
    for (int b = threadIdx.x; b <= nb; b += blockDim.x) {
        const int64_t f = bfirst[b];
        bsplits[b] = f == 0 ? 0 : keep_incl[f - 1];
    }
    if (threadIdx.x == 0 && prs) prs[V_host] = totals[2];
}

// ---------------------------------------------------------------------------
// grid subsampling
// ---------------------------------------------------------------------------
struct SubBatch {
    float ox, oy, oz, dl;
    uint64_t nx, ny;
};

__global__ void __launch_bounds__(256) sub_keys_kernel(const float* __restrict__ pts, int64_t n,
                                                       const int64_t* __restrict__ rs, int nb,
                                                       const SubBatch* __restrict__ sb, uint64_t* __restrict__ keys,
                                                       unsigned long long* __restrict__ or_and) {
    uint64_t o1 = 0, o0 = 0;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int b = batch_of(i, rs, nb);
        const SubBatch s = sb[b];
        const uint64_t ix = static_cast<uint64_t>(floorf((pts[3 * i] - s.ox) / s.dl));
        const uint64_t iy = static_cast<uint64_t>(floorf((pts[3 * i + 1] - s.oy) / s.dl));
        const uint64_t iz = static_cast<uint64_t>(floorf((pts[3 * i + 2] - s.oz) / s.dl));
        const uint64_t key = ix + s.nx * iy + s.nx * s.ny * iz;
        const uint64_t kv = (static_cast<uint64_t>(b) << 48) | (key & ((uint64_t(1) << 48) - 1));
        keys[i] = kv;
        o1 |= kv;
        o0 |= ~kv;
    }
    or_and_block(o1, o0, or_and);
}

__global__ void sub_caps_kernel(const int64_t* __restrict__ start, const int64_t* __restrict__ incl, int64_t n,
                                const uint64_t* __restrict__ sk, const int64_t* __restrict__ bfirst, int64_t max_p,
                                int64_t* __restrict__ keep) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nseg;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t b = static_cast<int64_t>(sk[start[v]] >> 48);
        keep[v] = (max_p <= 0 || (v - bfirst[b]) < max_p) ? 1 : 0;
    }
}

__global__ void sub_fill_kernel(const float* __restrict__ pts, const float* __restrict__ feat, int fdim,
                                const int32_t* __restrict__ cls, int ldim, const uint32_t* __restrict__ sidx,
                                const int64_t* __restrict__ start, const int64_t* __restrict__ incl, int64_t n,
                                const int64_t* __restrict__ keep, const int64_t* __restrict__ keep_incl,
                                float* __restrict__ out_pts, float* __restrict__ out_feat, int32_t* __restrict__ out_cls) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nseg;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        if (!keep[v]) continue;
        const int64_t k = keep_incl[v] - 1;
        const int64_t j0 = start[v];
        const int64_t j1 = v + 1 < nseg ? start[v + 1] : n;
        const int64_t cnt = j1 - j0;
        float sx = 0.f, sy = 0.f, sz = 0.f;
        for (int64_t j = j0; j < j1; ++j) {
            const int64_t i = sidx[j];
            sx += pts[3 * i];
            sy += pts[3 * i + 1];
            sz += pts[3 * i + 2];
        }
        const float a = static_cast<float>(1.0 / static_cast<double>(cnt));
        out_pts[3 * k] = sx * a;
        out_pts[3 * k + 1] = sy * a;
        out_pts[3 * k + 2] = sz * a;
        for (int c = 0; c < fdim; ++c) {
            float f = 0.f;
            for (int64_t j = j0; j < j1; ++j) f += feat[static_cast<int64_t>(sidx[j]) * fdim + c];
            out_feat[k * fdim + c] = f / static_cast<float>(cnt);
        }
        for (int c = 0; c < ldim; ++c) {
            // majority label; ties -> smallest label
            int32_t best = 0;
            int64_t bestc = 0;
            for (int64_t j = j0; j < j1; ++j) {
                const int32_t l = cls[static_cast<int64_t>(sidx[j]) * ldim + c];
                int64_t cntl = 0;
                for (int64_t jj = j0; jj < j1; ++jj) cntl += cls[static_cast<int64_t>(sidx[jj]) * ldim + c] == l;
                if (cntl > bestc || (cntl == bestc && l < best)) {
                    bestc = cntl;
                    best = l;
                }
            }
            out_cls[k * ldim + c] = best;
        }
    }
}

__global__ void sub_lengths_kernel(const int64_t* __restrict__ bfirst, const int64_t* __restrict__ keep_incl, int nb,
                                   int64_t* __restrict__ lengths) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const int64_t f0 = bfirst[b], f1 = bfirst[b + 1];
        const int64_t k0 = f0 == 0 ? 0 : keep_incl[f0 - 1];
        const int64_t k1 = f1 == 0 ? 0 : keep_incl[f1 - 1];
        lengths[b] = k1 - k0;
    }
}

// Grid of each batch item on the device, in the host's float arithmetic
// (origin = floor(min / dl) * dl, cells = floor((max - origin) / dl) + 1; the
// library builds with -ffp-contract=off and IEEE division, so the same
// roundings): no bbox read-back.  out[1] = 1 if a grid exceeds the 64-bit key
// range (checked by the host with the totals).
__global__ void sub_grid_kernel(const float* __restrict__ bbox, const int64_t* __restrict__ rs, int nb, float dl,
                                SubBatch* __restrict__ sb, int64_t* __restrict__ out) {
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const float inv = 1.0f / dl;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        SubBatch x;
        x.dl = dl;
        if (rs[b + 1] == rs[b]) {
            x.ox = x.oy = x.oz = 0.f;
            x.nx = x.ny = 1;
        } else {
            const float* bb = bbox + 6 * b;
            x.ox = floorf(bb[0] * inv) * dl;
            x.oy = floorf(bb[1] * inv) * dl;
            x.oz = floorf(bb[2] * inv) * dl;
            const float ex = floorf((bb[3] - x.ox) / dl), ey = floorf((bb[4] - x.oy) / dl),
                        ez = floorf((bb[5] - x.oz) / dl);
            if (!(ex < 1e15f && ey < 1e15f && ez < 1e15f)) {
                bad = 1;
                x.nx = x.ny = 1;
            } else {
                x.nx = static_cast<uint64_t>(ex) + 1;
                x.ny = static_cast<uint64_t>(ey) + 1;
                const uint64_t nz = static_cast<uint64_t>(ez) + 1;
                if (static_cast<double>(x.nx) * x.ny * nz >= 2.8e14) bad = 1;
                // power-of-two row / plane pitches when they fit the 48 key
                // bits: the same cell order, each coordinate in whole bits, so
                // the sort runs only the digits the keys vary in (or_and)
                uint64_t px = 1, py = 1, pz = 1;
                while (px < x.nx) px <<= 1;
                while (py < x.ny) py <<= 1;
                while (pz < nz) pz <<= 1;
                if (static_cast<double>(px) * py * pz < 2.8e14) {
                    x.nx = px;
                    x.ny = py;
                }
            }
        }
        sb[b] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) out[1] = bad;
}

// out[0] = output points, out[2 + b] = output points of batch item b
__global__ void sub_totals_kernel(const int64_t* __restrict__ incl, int64_t n, const int64_t* __restrict__ keep_incl,
                                  const int64_t* __restrict__ bfirst, int nb, int64_t* __restrict__ out) {
    const int64_t nseg = n > 0 ? incl[n - 1] : 0;
    if (threadIdx.x == 0) out[0] = nseg > 0 ? keep_incl[nseg - 1] : 0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const int64_t f0 = bfirst[b], f1 = bfirst[b + 1];
        const int64_t k0 = f0 == 0 ? 0 : keep_incl[f0 - 1];
        const int64_t k1 = f1 == 0 ? 0 : keep_incl[f1 - 1];
        out[2 + b] = k1 - k0;
    }
}

// Shared "sorted segments" state in the workspace front (same layout for the
// count and fill phases).
struct SegState {
    uint64_t* sk;
    uint32_t* sidx;
    int64_t* start;
    int64_t* incl;
    int64_t* keep;
    int64_t* keep_incl;
    int64_t* npts;
    int64_t* npts_incl;
    int64_t* bfirst;
    int64_t* scalars;  // [0] n_valid, [1..3] totals
};

inline SegState take_seg_state(Workspace& ws, int64_t n, int nb) {
    SegState s;
    s.sk = ws.take<uint64_t>(n);
    s.sidx = ws.take<uint32_t>(n);
    s.start = ws.take<int64_t>(n);
    s.incl = ws.take<int64_t>(n);
    s.keep = ws.take<int64_t>(n);
    s.keep_incl = ws.take<int64_t>(n);
    s.npts = ws.take<int64_t>(n);
    s.npts_incl = ws.take<int64_t>(n);
    s.bfirst = ws.take<int64_t>(nb + 1);
    s.scalars = ws.take<int64_t>(8);
    return s;
}

inline size_t seg_state_bytes(int64_t n, int nb) {
    return ws_bytes<uint64_t>(n) + ws_bytes<uint32_t>(n) + 6 * ws_bytes<int64_t>(n) + ws_bytes<int64_t>(nb + 1) +
           ws_bytes<int64_t>(8);
}

// keys (unsorted) -> sorted segments, heads, starts, batch firsts.
// or_and (nullable): the keys' OR / complement-OR pair (vox_keys_kernel), in
// s.scalars[6..7], which the caller zeroed before the keys (prefilled)
inline void sort_segments(const uint64_t* keys, int64_t n, int end_bit, uint64_t invalid, int nb, bool batch_shift,
                          uint64_t batch_div, SegState& s, Workspace& ws, hipStream_t st,
                          const uint64_t* or_and = nullptr) {
    if (!or_and) fill_async(s.scalars, 0, sizeof(int64_t) * 8, st);
    const unsigned g = stream_grid(n > 0 ? n : 1, 256);
    if (n > 0) {
        Workspace sws = ws;
        prim::radix_sort_pairs<uint64_t>(keys, nullptr, s.sk, s.sidx, n, end_bit, sws, st, -1, or_and);
        int64_t* head = s.keep;  // reuse as scratch before keep is computed
        seg_heads_kernel<<<g, 256, 0, st>>>(s.sk, n, invalid, head, s.scalars);
        O3DML_LAUNCH_CHECK();
        sws = ws;
        prim::scan<int64_t, int64_t>(head, s.incl, n, true, sws, st);
        seg_start_kernel<<<g, 256, 0, st>>>(head, s.incl, n, s.start);
        O3DML_LAUNCH_CHECK();
    }
    seg_batch_first_kernel<<<g, 256, 0, st>>>(s.sk, s.start, s.incl, n, nb, batch_shift ? 1 : 0, batch_div, s.bfirst);
    O3DML_LAUNCH_CHECK();
}

inline size_t sort_segments_ws_bytes(int64_t n) {
    return prim::radix_sort_workspace_bytes<uint64_t>(n) + ws_bytes<uint64_t>(n) + prim::scan_workspace_bytes(n);
}

inline VoxParams make_vox_params(int ndim, int nb, const float* vs, const float* mn, const float* mx) {
    VoxParams vp{};
    vp.ndim = ndim;
    vp.nb = nb;
    int64_t h = 1, h2 = 1;
    int64_t stride2[kMaxVoxDim];
    for (int d = 0; d < ndim; ++d) {
        vp.inv[d] = 1.0 / static_cast<double>(vs[d]);
        vp.mn[d] = static_cast<double>(mn[d]);
        vp.ext[d] = static_cast<int32_t>((static_cast<double>(mx[d]) - static_cast<double>(mn[d])) * vp.inv[d]);
        if (vp.ext[d] < 0) vp.ext[d] = 0;
        vp.stride[d] = h;
        h *= vp.ext[d];
        // power-of-two strides: the same order of (batch, coordinates) keys,
        // each coordinate in whole bits, so only the digits its values vary in
        // need a sort pass (the keys' OR / AND plan the passes)
        stride2[d] = h2;
        int64_t p2 = 1;
        while (p2 < vp.ext[d] && p2 < (int64_t(1) << 40)) p2 <<= 1;
        h2 = h2 < (int64_t(1) << 56) / p2 ? h2 * p2 : (int64_t(1) << 56);
    }
    if (h2 < (int64_t(1) << 56) / (nb + 1)) {  // fits the 64-bit key budget: use it
        for (int d = 0; d < ndim; ++d) vp.stride[d] = stride2[d];
        h = h2;
    }
    vp.batch_hash = h > 0 ? h : 1;
    vp.invalid_key = vp.batch_hash * nb;
    return vp;
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_voxelize_workspace_size(int64_t n_points, int64_t n_batch) {
    return seg_state_bytes(n_points, static_cast<int>(n_batch)) + ws_bytes<uint64_t>(n_points) +
           sort_segments_ws_bytes(n_points) + 2 * prim::scan_workspace_bytes(n_points);
}

// Phase 1: writes counts_host[0] = V (voxels), counts_host[1] = P (points).
// voxel_size / range_min / range_max are HOST arrays of ndim floats.
O3DML_API int o3dml_voxelize_count(const float* points, int64_t n_points, int ndim, int64_t n_batch,
                                   const int64_t* row_splits, const float* voxel_size_host,
                                   const float* range_min_host, const float* range_max_host,
                                   int64_t max_points_per_voxel, int64_t max_voxels, int64_t* counts_host,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(ndim >= 1 && ndim <= kMaxVoxDim, "voxelize supports 1..%d dims", kMaxVoxDim);
    for (int d = 0; d < ndim; ++d) O3DML_REQUIRE(voxel_size_host[d] > 0.f, "voxel_size must be > 0");
    O3DML_REQUIRE(max_points_per_voxel >= 1 && max_voxels >= 0, "invalid caps");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    VoxParams vp = make_vox_params(ndim, nb, voxel_size_host, range_min_host, range_max_host);
    O3DML_REQUIRE(vp.batch_hash < (int64_t(1) << 56) / (nb + 1), "voxel grid too large for 64-bit keys");
    SegState s = take_seg_state(ws, n_points, nb);
    uint64_t* keys = ws.take<uint64_t>(n_points);
    const unsigned g = stream_grid(n_points > 0 ? n_points : 1, 256);
    TimedRegion tr("voxelize_count", st);  // device time of the phase (bench op roofline)
    // scalars zeroed first: [6..7] collect the keys' OR / complement OR
    fill_async(s.scalars, 0, sizeof(int64_t) * 8, st);
    unsigned long long* or_and = reinterpret_cast<unsigned long long*>(s.scalars + 6);
    if (n_points > 0) {
        vox_keys_kernel<<<g, 256, 0, st>>>(points, n_points, row_splits, vp, keys, or_and);
        O3DML_LAUNCH_CHECK();
    }
    sort_segments(keys, n_points, prim::bits_needed(static_cast<uint64_t>(vp.invalid_key)),
                  static_cast<uint64_t>(vp.invalid_key), nb, false, static_cast<uint64_t>(vp.batch_hash), s, ws, st,
                  reinterpret_cast<const uint64_t*>(or_and));
    if (n_points > 0) {
        vox_caps_kernel<<<g, 256, 0, st>>>(s.sk, s.start, s.incl, s.scalars, n_points, s.bfirst, vp.batch_hash,
                                           max_voxels, max_points_per_voxel, s.keep, s.npts);
        O3DML_LAUNCH_CHECK();
        // only the first n_seg entries matter; scanning n keeps the launch host-sync free
        Workspace sws = ws;
        prim::scan<int64_t, int64_t>(s.keep, s.keep_incl, n_points, true, sws, st);
        sws = ws;
        prim::scan<int64_t, int64_t>(s.npts, s.npts_incl, n_points, true, sws, st);
    }
    vox_totals_kernel<<<1, 64, 0, st>>>(s.incl, n_points, s.keep_incl, s.npts_incl, s.scalars + 1);
    O3DML_LAUNCH_CHECK();
    tr.end();
    int64_t* tot = pinned_scratch();
    O3DML_CHECK_HIP(hipMemcpyAsync(tot, s.scalars + 1, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    O3DML_CHECK_HIP(hipStreamSynchronize(st));
    counts_host[0] = tot[1];
    counts_host[1] = tot[2];
    O3DML_GUARD_END
}

O3DML_API int o3dml_voxelize_fill(int64_t n_points, int ndim, int64_t n_batch, const float* voxel_size_host,
                                  const float* range_min_host, const float* range_max_host, int64_t n_voxels,
                                  int32_t* voxel_coords, int64_t* voxel_point_indices,
                                  int64_t* voxel_point_row_splits, int64_t* voxel_batch_splits, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    VoxParams vp = make_vox_params(ndim, nb, voxel_size_host, range_min_host, range_max_host);
    SegState s = take_seg_state(ws, n_points, nb);
    TimedRegion tr("voxelize_fill", st);
    if (n_points > 0) {
        vox_fill_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(s.sk, s.sidx, s.start, s.incl, n_points, s.keep,
                                                                   s.keep_incl, s.npts, s.npts_incl, vp, voxel_coords,
                                                                   voxel_point_indices, voxel_point_row_splits);
        O3DML_LAUNCH_CHECK();
    }
    batch_splits_kernel<<<1, 256, 0, st>>>(s.bfirst, s.keep_incl, nb, s.scalars + 1, voxel_batch_splits,
                                           voxel_point_row_splits, n_voxels);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// ---------------------------------------------------------------------------
namespace o3dml {
// p' = p R_b (transpose: p R_b^T) for the points of batch item b, in fp32 with
// the reference's rounding: (p0 R0j + p1 R1j) + p2 R2j, every product rounded
// (no contraction; kpconv.py:2087-2090 batch_grid_subsampling's rotations)
__global__ void __launch_bounds__(256) rotate_batched_kernel(const float* __restrict__ pts, int64_t n, int nb,
                                                             const int64_t* __restrict__ rs,
                                                             const float* __restrict__ R, int transpose,
                                                             float* __restrict__ out) {
    __shared__ int64_t s_rs[kLdsSplits];
    const int64_t* rsp = stage_splits(s_rs, rs, nb);
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const float* r = R + 9 * batch_of(i, rsp, nb);
        const float p0 = pts[3 * i], p1 = pts[3 * i + 1], p2 = pts[3 * i + 2];
        float o[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float r0 = transpose ? r[3 * j] : r[j], r1 = transpose ? r[3 * j + 1] : r[3 + j],
                        r2 = transpose ? r[3 * j + 2] : r[6 + j];
            o[j] = (p0 * r0 + p1 * r1) + p2 * r2;
        }
        out[3 * i] = o[0];
        out[3 * i + 1] = o[1];
        out[3 * i + 2] = o[2];
    }
}
}  // namespace o3dml

O3DML_API int o3dml_rotate_batched(const float* points, int64_t n_points, int64_t n_batch,
                                   const int64_t* row_splits, const float* rotations, int transpose, float* out,
                                   void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(n_batch >= 1, "need at least one batch item");
    if (n_points == 0) return 0;
    rotate_batched_kernel<<<stream_grid(n_points, 256), 256, 0, as_stream(stream)>>>(
            points, n_points, (int)n_batch, row_splits, rotations, transpose, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API size_t o3dml_grid_subsample_workspace_size(int64_t n_points, int64_t n_batch) {
    return seg_state_bytes(n_points, static_cast<int>(n_batch)) + ws_bytes<uint64_t>(n_points) +
           ws_bytes<SubBatch>(n_batch) + ws_bytes<float>(6 * n_batch) + sort_segments_ws_bytes(n_points) +
           prim::scan_workspace_bytes(n_points) + ws_bytes<int64_t>(2 + n_batch);
}

// Phase 1 without a host synchronisation: grid per batch item (on the device,
// sub_grid_kernel), sort, caps; out (device int64 [2 + n_batch]) receives the
// number of output points, a grid-too-large flag and the output points per
// batch item — the caller reads them (with other values) in one transfer.
O3DML_API int o3dml_grid_subsample_count_async(const float* points, int64_t n_points, int64_t n_batch,
                                               const int64_t* row_splits, float dl, int64_t max_p, int64_t* out,
                                               void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(dl > 0.f, "sampleDl must be > 0");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    if (n_points == 0) {
        fill_async(out, 0, sizeof(int64_t) * (2 + nb), st);
        return 0;
    }
    SegState s = take_seg_state(ws, n_points, nb);
    uint64_t* keys = ws.take<uint64_t>(n_points);
    SubBatch* sb_d = ws.take<SubBatch>(nb);
    float* bbox_d = ws.take<float>(6 * nb);
    TimedRegion tr("grid_subsample_count", st);  // device time of the phase (bench op roofline)
    launch_bbox(points, row_splits, nb, bbox_d, st);
    O3DML_LAUNCH_CHECK();
    sub_grid_kernel<<<1, 256, 0, st>>>(bbox_d, row_splits, nb, dl, sb_d, out);
    O3DML_LAUNCH_CHECK();
    fill_async(s.scalars, 0, sizeof(int64_t) * 8, st);  // [6..7]: the keys' OR / complement OR
    unsigned long long* or_and = reinterpret_cast<unsigned long long*>(s.scalars + 6);
    sub_keys_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(points, n_points, row_splits, nb, sb_d, keys, or_and);
    O3DML_LAUNCH_CHECK();
    const uint64_t invalid = ~uint64_t(0);
    sort_segments(keys, n_points, 48 + prim::bits_needed(static_cast<uint64_t>(nb > 1 ? nb - 1 : 0)), invalid, nb,
                  true, 48, s, ws, st, reinterpret_cast<const uint64_t*>(or_and));
    sub_caps_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(s.start, s.incl, n_points, s.sk, s.bfirst, max_p,
                                                               s.keep);
    O3DML_LAUNCH_CHECK();
    Workspace sws = ws;
    prim::scan<int64_t, int64_t>(s.keep, s.keep_incl, n_points, true, sws, st);
    sub_totals_kernel<<<1, 256, 0, st>>>(s.incl, n_points, s.keep_incl, s.bfirst, nb, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// Phase 1 with the read-back: writes the number of output points to *n_out_host.
O3DML_API int o3dml_grid_subsample_count(const float* points, int64_t n_points, int64_t n_batch,
                                         const int64_t* row_splits, const int64_t* row_splits_host, float dl,
                                         int64_t max_p, int64_t* n_out_host, void* workspace, size_t workspace_bytes,
                                         void* stream) {
    O3DML_GUARD_BEGIN
    (void)row_splits_host;
    hipStream_t st = as_stream(stream);
    const size_t front = o3dml_grid_subsample_workspace_size(n_points, n_batch) - ws_bytes<int64_t>(2 + n_batch);
    O3DML_REQUIRE(workspace_bytes >= front + ws_bytes<int64_t>(2), "grid_subsample: workspace too small");
    int64_t* out = reinterpret_cast<int64_t*>(static_cast<char*>(workspace) + front);
    const int rc = o3dml_grid_subsample_count_async(points, n_points, n_batch, row_splits, dl, max_p, out, workspace,
                                                    front, stream);
    if (rc != 0) return rc;
    int64_t* tot = pinned_scratch();
    O3DML_CHECK_HIP(hipMemcpyAsync(tot, out, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    O3DML_CHECK_HIP(hipStreamSynchronize(st));
    O3DML_REQUIRE(tot[1] == 0, "grid_subsample: grid too large");
    *n_out_host = tot[0];
    O3DML_GUARD_END
}

// Phase 2: barycentres (fp32, input order), feature means, majority labels,
// lengths per batch item (int64 [B]).
O3DML_API int o3dml_grid_subsample_fill(const float* points, int64_t n_points, int64_t n_batch, const float* features,
                                        int fdim, const int32_t* classes, int ldim, float* out_points,
                                        float* out_features, int32_t* out_classes, int64_t* out_lengths,
                                        void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    const int nb = static_cast<int>(n_batch);
    SegState s = take_seg_state(ws, n_points, nb);
    TimedRegion tr("grid_subsample_fill", st);
    if (n_points > 0) {
        sub_fill_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(points, features, fdim, classes, ldim, s.sidx,
                                                                   s.start, s.incl, n_points, s.keep, s.keep_incl,
                                                                   out_points, out_features, out_classes);
        O3DML_LAUNCH_CHECK();
        sub_lengths_kernel<<<1, 256, 0, st>>>(s.bfirst, s.keep_incl, nb, out_lengths);
    } else {
        fill_async(out_lengths, 0, sizeof(int64_t) * nb, st);
    }
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

// ---------------------------------------------------------------------------
// calculate_grid (ml3d/torch/models/sparseconvnet.py:388-401)
// The reference expands each position by {-1,0}^3, keeps non-negative
// all-even cells and takes torch.unique(dim=0).  Per axis exactly one of
// {c-1, c} is even, so each input has a single candidate parent: c - (c & 1)
// with c = trunc(p) (torch .long()), kept iff every c >= 0.  Parents are
// packed as (x/2, y/2, z/2) 20-bit fields, x most significant, so one radix
// sort + unique gives the lexicographic order torch.unique returns.
// ---------------------------------------------------------------------------
namespace o3dml {
namespace {

constexpr uint64_t kGridInvalid = uint64_t(1) << 60;
constexpr int64_t kGridMax = int64_t(1) << 21;

// or_and[0] / [1]: OR of the keys and of their complements (the bits that
// vary among them, for the device-planned radix passes): one atomic pair per
// wave.
constexpr int kGridBlock = 256;  // grid_parent_kernel block (its LDS partials are sized for it)

__global__ void __launch_bounds__(kGridBlock) grid_parent_kernel(const float* __restrict__ pos, int64_t n, uint64_t* __restrict__ keys,
                                   int64_t* __restrict__ flags, unsigned long long* __restrict__ or_and) {
    uint64_t o1 = 0, o0 = 0;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        uint64_t key = 0;
        bool valid = true;
        for (int d = 0; d < 3; ++d) {
            const float p = pos[3 * i + d];
            if (!(p > -1.0f)) {  // trunc(p) < 0 (or NaN): no non-negative parent
                valid = false;
                continue;
            }
            if (p >= static_cast<float>(kGridMax)) {
                flags[0] = 1;  // out of the packable range -> host raises
                valid = false;
                continue;
            }
            const int64_t c = static_cast<int64_t>(p);  // trunc, as torch .long()
            key = (key << 20) | static_cast<uint64_t>(c >> 1);
        }
        keys[i] = valid ? key : kGridInvalid;
        o1 |= keys[i];
        o0 |= ~keys[i];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        o1 |= static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(o1), d, 64));
        o0 |= static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(o0), d, 64));
    }
    // the block's waves combined in LDS, then one atomic pair per block and
    // only for bits not yet recorded: same-address atomics serialise (one
    // pair per wave cost a 88k-voxel level ~30 us)
    __shared__ unsigned long long part[2][kGridBlock / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[0][w] = o1;
        part[1][w] = o0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < static_cast<int>(blockDim.x >> 6); ++k) {
            o1 |= part[0][k];
            o0 |= part[1][k];
        }
        const unsigned long long c1 = __hip_atomic_load(&or_and[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c0 = __hip_atomic_load(&or_and[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o1 & ~c1) atomicOr(&or_and[0], static_cast<unsigned long long>(o1));
        if (o0 & ~c0) atomicOr(&or_and[1], static_cast<unsigned long long>(o0));
    }
}

__global__ void grid_unique_heads_kernel(const uint64_t* __restrict__ sk, int64_t n, int64_t* __restrict__ head) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        head[i] = (sk[i] != kGridInvalid && (i == 0 || sk[i] != sk[i - 1])) ? 1 : 0;
}

__global__ void grid_unique_write_kernel(const uint64_t* __restrict__ sk, const int64_t* __restrict__ incl, int64_t n,
                                         float* __restrict__ out) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint64_t k = sk[i];
        if (k == kGridInvalid || (i > 0 && k == sk[i - 1])) continue;
        const int64_t o = incl[i] - 1;
        const uint64_t m = (uint64_t(1) << 20) - 1;
        out[3 * o + 0] = static_cast<float>(static_cast<int64_t>((k >> 40) & m) * 2) + 0.5f;
        out[3 * o + 1] = static_cast<float>(static_cast<int64_t>((k >> 20) & m) * 2) + 0.5f;
        out[3 * o + 2] = static_cast<float>(static_cast<int64_t>(k & m) * 2) + 0.5f;
    }
}

struct GridState {
    uint64_t* keys;
    uint64_t* sk;
    uint32_t* sidx;
    int64_t* head;
    int64_t* incl;
    int64_t* flags;
};

inline GridState take_grid_state(Workspace& ws, int64_t n) {
    GridState g;
    g.keys = ws.take<uint64_t>(n);
    g.sk = ws.take<uint64_t>(n);
    g.sidx = ws.take<uint32_t>(n);
    g.head = ws.take<int64_t>(n);
    g.incl = ws.take<int64_t>(n);
    g.flags = ws.take<int64_t>(6);  // [0] range flag, [2..3] (count, flag) for the host read, [4..5] key OR / ~OR
    return g;
}

}  // namespace
}  // namespace o3dml

O3DML_API size_t o3dml_calculate_grid_workspace_size(int64_t n_points) {
    return 2 * ws_bytes<uint64_t>(n_points) + ws_bytes<uint32_t>(n_points) + 2 * ws_bytes<int64_t>(n_points) +
           ws_bytes<int64_t>(6) +
           std::max(prim::radix_sort_workspace_bytes<uint64_t>(n_points), prim::scan_workspace_bytes(n_points));
}

O3DML_API int o3dml_calculate_grid_count(const float* positions, int64_t n_points, int64_t* n_out_host,
                                         void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    GridState g = take_grid_state(ws, n_points);
    int64_t host[2] = {0, 0};
    if (n_points > 0) {
        fill_async(g.flags, 0, 6 * sizeof(int64_t), st);
        const unsigned gr = stream_grid(n_points, 256);
        unsigned long long* or_and = reinterpret_cast<unsigned long long*>(g.flags + 4);
        // one block per CU at most: fewer blocks, fewer same-address atomics
        grid_parent_kernel<<<stream_grid(n_points, kGridBlock, 256), kGridBlock, 0, st>>>(positions, n_points,
                                                                                          g.keys, g.flags, or_and);
        O3DML_LAUNCH_CHECK();
        Workspace sws = ws;
        // three 20-bit fields, 8 passes planned on the host; only the digits
        // that vary among the keys run (a room's parents: 3-4 of the 8)
        prim::radix_sort_pairs<uint64_t>(g.keys, nullptr, g.sk, g.sidx, n_points, 61, sws, st, -1,
                                         reinterpret_cast<const uint64_t*>(or_and));
        grid_unique_heads_kernel<<<gr, 256, 0, st>>>(g.sk, n_points, g.head);
        O3DML_LAUNCH_CHECK();
        sws = ws;
        // the scan's last tile writes (count, range flag) next to each other:
        // one 16-B read into pinned memory instead of two pageable ones
        prim::scan<int64_t, int64_t>(g.head, g.incl, n_points, true, sws, st, g.flags + 2, g.flags);
        int64_t* pinned = pinned_scratch();
        O3DML_CHECK_HIP(hipMemcpyAsync(pinned, g.flags + 2, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        O3DML_CHECK_HIP(hipStreamSynchronize(st));
        host[0] = pinned[1];
        host[1] = pinned[0];
    }
    O3DML_REQUIRE(host[0] == 0, "calculate_grid: positions must be < %lld", (long long)kGridMax);
    *n_out_host = host[1];
    O3DML_GUARD_END
}

O3DML_API int o3dml_calculate_grid_fill(int64_t n_points, float* out_positions, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    GridState g = take_grid_state(ws, n_points);
    if (n_points > 0) {
        grid_unique_write_kernel<<<stream_grid(n_points, 256), 256, 0, st>>>(g.sk, g.incl, n_points, out_positions);
        O3DML_LAUNCH_CHECK();
    }
    O3DML_GUARD_END
}

// ---------------------------------------------------------------------------
// SparseConvUnet eval plan in ONE call (sparseconvnet.py:296-331 InputLayer,
// :388-401 calculate_grid per level): voxelize at vs = 1 in [0, 40960)^3,
// per voxel its first point's position and the mean of its points' features
// (summed in point order, as reduce_subarrays_sum over the voxel-sorted
// features, then divided by the count), the voxel of every input point (0 for
// points outside the range, as the reference's zero-initialised reverse map),
// and the stride-2 grid of every level (level l's input = level l-1's grid
// / 2, exactly).  The host reads each size once (voxel count, one per level),
// with no Python between the launches.  Outputs go to caller buffers sized
// for n_points rows per level (every level has at most as many points as
// the one before), at fixed offsets, so a captured body can read them in place.
// ---------------------------------------------------------------------------
namespace o3dml {
namespace {
__global__ void scn_splits_kernel(int64_t n, int64_t* __restrict__ rs) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        rs[0] = 0;
        rs[1] = n;
    }
}

__global__ void scn_input_kernel(const float* __restrict__ points, const float* __restrict__ features, int fdim,
                                 const int64_t* __restrict__ pidx, const int64_t* __restrict__ prs, int64_t nvox,
                                 float* __restrict__ vpos, float* __restrict__ vfeat,
                                 int64_t* __restrict__ index_map) {
    for (int64_t v = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v < nvox;
         v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t s = prs[v], e = prs[v + 1];
        const int64_t p0 = pidx[s];
        vpos[3 * v] = points[3 * p0];
        vpos[3 * v + 1] = points[3 * p0 + 1];
        vpos[3 * v + 2] = points[3 * p0 + 2];
        const float cnt = static_cast<float>(e - s);
        for (int c = 0; c < fdim; ++c) {
            float acc = 0.f;
            for (int64_t j = s; j < e; ++j) acc += features[pidx[j] * fdim + c];
            vfeat[v * fdim + c] = acc / cnt;
        }
        for (int64_t j = s; j < e; ++j) index_map[pidx[j]] = v;
    }
}

__global__ void scn_half_kernel(const float* __restrict__ in, int64_t n3, float* __restrict__ out) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n3;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[i] = in[i] / 2.f;
}
}  // namespace
}  // namespace o3dml

// The deep levels of the eval plan in ONE workgroup: once a level's input has
// <= kDeepMax points (a room: from level 2 on, ~5k, then ~1.3k, ~400, ~130),
// every remaining level's calculate_grid runs here — parent keys (grid_parent
// arithmetic), a bitonic sort in LDS, the unique keys compacted — each
// level's grid and grid / 2 written at its offset, the counts to sizes_dev;
// the next level's keys are the unique keys' fields >> 1 (its positions are
// k + 0.25, whose trunc is k).  Same keys, same order, same floats as
// calculate_grid level by level, in one launch and one host read instead of
// ~7 launches and a read per level.
constexpr int kDeepMax = 8192;
constexpr int kDeepThreads = 1024;

__device__ __forceinline__ void deep_write(uint64_t k, int64_t o, float* __restrict__ out, float* __restrict__ half) {
    const uint64_t m = (uint64_t(1) << 20) - 1;
    const float x = static_cast<float>(static_cast<int64_t>((k >> 40) & m) * 2) + 0.5f;
    const float y = static_cast<float>(static_cast<int64_t>((k >> 20) & m) * 2) + 0.5f;
    const float z = static_cast<float>(static_cast<int64_t>(k & m) * 2) + 0.5f;
    out[3 * o] = x;
    out[3 * o + 1] = y;
    out[3 * o + 2] = z;
    if (half) {
        half[3 * o] = x / 2.f;
        half[3 * o + 1] = y / 2.f;
        half[3 * o + 2] = z / 2.f;
    }
}

__global__ void __launch_bounds__(kDeepThreads) scn_deep_levels_kernel(const float* __restrict__ in_pos, int m, int l0,
                                                                        int n_levels, int64_t cap,
                                                                        float* __restrict__ grids,
                                                                        float* __restrict__ halves,
                                                                        int64_t* __restrict__ sizes_dev) {
    __shared__ uint64_t a[kDeepMax];
    __shared__ uint64_t b[kDeepMax];
    __shared__ int wsum[kDeepThreads / 64];
    const int t = threadIdx.x;
    const uint64_t kPad = ~uint64_t(0);  // sorts after every key, kGridInvalid included
    for (int i = t; i < m; i += kDeepThreads) {  // grid_parent_kernel's keys (in range by construction)
        uint64_t key = 0;
        bool valid = true;
        for (int d = 0; d < 3; ++d) {
            const float p = in_pos[3 * i + d];
            if (!(p > -1.0f) || p >= static_cast<float>(kGridMax)) {
                valid = false;
                continue;
            }
            key = (key << 20) | static_cast<uint64_t>(static_cast<int64_t>(p) >> 1);
        }
        a[i] = valid ? key : kGridInvalid;
    }
    int n = m;
    for (int l = l0; l < n_levels; ++l) {
        if (n == 0) {
            if (t == 0) sizes_dev[l] = 0;
            continue;
        }
        int P = 1;
        while (P < n) P <<= 1;
        for (int i = n + t; i < P; i += kDeepThreads) a[i] = kPad;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1) {  // bitonic sort, ascending
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = t; i < P; i += kDeepThreads) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const uint64_t x = a[i], y = a[ixj];
                        if ((x > y) == ((i & k) == 0)) {
                            a[i] = y;
                            a[ixj] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        // unique: thread t owns the contiguous items [t c, t c + c)
        const int c = (P + kDeepThreads - 1) / kDeepThreads;
        const int i0 = t * c;
        int h = 0;
        for (int i = i0; i < i0 + c && i < P; ++i) {
            const uint64_t k = a[i];
            h += (k != kGridInvalid && k != kPad && (i == 0 || k != a[i - 1])) ? 1 : 0;
        }
        const int incl = wave_inclusive_scan(h);
        if ((t & 63) == 63) wsum[t >> 6] = incl;
        __syncthreads();
        int o = incl - h, tot = 0;
        for (int w = 0; w < kDeepThreads / 64; ++w) {
            o += w < (t >> 6) ? wsum[w] : 0;
            tot += wsum[w];
        }
        float* out = grids + static_cast<int64_t>(l) * cap * 3;
        float* hl = halves ? halves + static_cast<int64_t>(l) * cap * 3 : nullptr;
        for (int i = i0; i < i0 + c && i < P; ++i) {
            const uint64_t k = a[i];
            if (k != kGridInvalid && k != kPad && (i == 0 || k != a[i - 1])) {
                b[o] = k;
                deep_write(k, o, out, hl);
                ++o;
            }
        }
        if (t == 0) sizes_dev[l] = tot;
        __syncthreads();
        const uint64_t f = (uint64_t(1) << 20) - 1;
        for (int i = t; i < tot; i += kDeepThreads) {  // next level: the fields >> 1
            const uint64_t k = b[i];
            a[i] = ((((k >> 40) & f) >> 1) << 40) | ((((k >> 20) & f) >> 1) << 20) | ((k & f) >> 1);
        }
        n = tot;
        __syncthreads();
    }
}

// O3DML_SCN_DEEP=0: every level through calculate_grid (A/B)
static bool scn_deep_on() {
    static const bool v = [] {
        const char* e = std::getenv("O3DML_SCN_DEEP");
        return !(e && e[0] == '0');
    }();
    return v;
}

O3DML_API size_t o3dml_scn_plan_workspace_size(int64_t n_points) {
    const int64_t n = std::max<int64_t>(n_points, 1);
    return ws_bytes<int64_t>(2) + ws_bytes<int32_t>(3 * n) + ws_bytes<int64_t>(n) + ws_bytes<int64_t>(n + 1) +
           ws_bytes<int64_t>(2) + ws_bytes<float>(3 * n) +
           std::max(o3dml_voxelize_workspace_size(n, 1), o3dml_calculate_grid_workspace_size(n));
}

// points / features: f32 [n, 3] / [n, fdim]; buffers of cap >= n rows: vox_pos
// [cap, 3], vox_feat [cap, fdim], index_map int64 [cap], grids f32
// [n_levels][cap][3] (level l's grid at row l * cap); sizes_host int64
// [1 + n_levels] = voxels, then each level's grid points.
O3DML_API int o3dml_scn_plan(const float* points, const float* features, int64_t n_points, int64_t cap, int fdim,
                             int n_levels,
                             float* vox_pos, float* vox_feat, int64_t* index_map, float* grids, float* halves,
                             int64_t* sizes_host, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(fdim >= 1 && fdim <= 64 && n_levels >= 0, "scn_plan: bad fdim / n_levels");
    O3DML_REQUIRE(cap >= n_points, "scn_plan: capacity %lld < %lld points", (long long)cap, (long long)n_points);
    O3DML_REQUIRE(workspace_bytes >= o3dml_scn_plan_workspace_size(n_points), "scn_plan: workspace too small");
    hipStream_t st = as_stream(stream);
    const int64_t n = std::max<int64_t>(n_points, 1);
    Workspace ws(workspace, workspace_bytes);
    int64_t* rs = ws.take<int64_t>(2);
    int32_t* coords = ws.take<int32_t>(3 * n);
    int64_t* pidx = ws.take<int64_t>(n);
    int64_t* prs = ws.take<int64_t>(n + 1);
    int64_t* bsp = ws.take<int64_t>(2);
    float* half = ws.take<float>(3 * n);
    void* sub = ws.base + ws.used;
    const size_t sub_bytes = ws.size - ws.used;
    for (int l = 0; l <= n_levels; ++l) sizes_host[l] = 0;
    fill_async(index_map, 0, sizeof(int64_t) * n_points, st);
    if (n_points == 0) return 0;
    scn_splits_kernel<<<1, 64, 0, st>>>(n_points, rs);
    O3DML_LAUNCH_CHECK();
    const float vs[3] = {1.f, 1.f, 1.f}, mn[3] = {0.f, 0.f, 0.f}, mx[3] = {40960.f, 40960.f, 40960.f};
    const int64_t big = std::numeric_limits<int64_t>::max();
    int64_t counts[2] = {0, 0};
    int rc = o3dml_voxelize_count(points, n_points, 3, 1, rs, vs, mn, mx, big, big, counts, sub, sub_bytes, stream);
    if (rc) return rc;
    const int64_t nvox = counts[0];
    rc = o3dml_voxelize_fill(n_points, 3, 1, vs, mn, mx, nvox, coords, pidx, prs, bsp, sub, sub_bytes, stream);
    if (rc) return rc;
    sizes_host[0] = nvox;
    if (nvox > 0) {
        scn_input_kernel<<<stream_grid(nvox, 256), 256, 0, st>>>(points, features, fdim, pidx, prs, nvox, vox_pos,
                                                                  vox_feat, index_map);
        O3DML_LAUNCH_CHECK();
    }
    const float* in = vox_pos;
    int64_t m = nvox;
    for (int l = 0; l < n_levels && m > 0; ++l) {
        if (scn_deep_on() && m <= kDeepMax && n_levels - l <= 8) {  // the rest in one workgroup, one host read
            int64_t* sizes_dev = reinterpret_cast<int64_t*>(sub);
            scn_deep_levels_kernel<<<1, kDeepThreads, 0, st>>>(in, static_cast<int>(m), l, n_levels, cap, grids,
                                                               halves, sizes_dev);
            O3DML_LAUNCH_CHECK();
            int64_t* pinned = pinned_scratch();
            O3DML_CHECK_HIP(hipMemcpyAsync(pinned, sizes_dev + l, (n_levels - l) * sizeof(int64_t),
                                           hipMemcpyDeviceToHost, st));
            O3DML_CHECK_HIP(hipStreamSynchronize(st));
            for (int q = l; q < n_levels; ++q) sizes_host[1 + q] = pinned[q - l];
            break;
        }
        int64_t m_out = 0;
        rc = o3dml_calculate_grid_count(in, m, &m_out, sub, sub_bytes, stream);
        if (rc) return rc;
        float* out = grids + static_cast<int64_t>(l) * cap * 3;
        rc = o3dml_calculate_grid_fill(m, out, sub, sub_bytes, stream);
        if (rc) return rc;
        sizes_host[1 + l] = m_out;
        // the next level's positions: into `halves` at the level's offset when
        // given (the body reads them in place), else a workspace temp
        float* hl = halves ? halves + static_cast<int64_t>(l) * cap * 3 : half;
        if ((l + 1 < n_levels || halves) && m_out > 0) {
            scn_half_kernel<<<stream_grid(3 * m_out, 256), 256, 0, st>>>(out, 3 * m_out, hl);
            O3DML_LAUNCH_CHECK();
        }
        in = hl;
        m = m_out;
    }
    O3DML_GUARD_END
}
