// grid.hpp — dense per-batch uniform grid over a point cloud, used by the
// kNN / radius / ball-query kernels (not by fixed_radius_search, which must
// use Open3D's hash-table semantics).
//
// Build: per-batch bounding box (one workgroup per batch item) -> host picks a
// cell size h giving ~`target` points per cell, capped at `cap_factor*N_b+64`
// cells -> cell key per point -> stable radix sort (key, id) -> CSR
// cell_splits + points re-laid out as float4 (x,y,z,id) in cell order, so a
// cell scan is one contiguous 16-B-per-point stream.
#pragma once

#include <cmath>
#include <vector>

#include "primitives.hpp"

namespace o3dml {

struct GridBatch {
    float ox, oy, oz, h;   // origin, cell size
    float inv_h;
    int dx, dy, dz;        // cells per axis
    uint32_t offset;       // first global cell id of this batch item
    uint32_t pad[3];
};

// Kernels defined in this header get internal linkage (one copy per TU).
namespace {

// Per-batch bounding boxes [B][6] (min xyz, max xyz).  gridDim = (kBBoxParts,
// B): block (p, b) reduces a 1/kBBoxParts slice of batch item b and folds it
// into the item's box with integer atomics on an order-preserving encoding of
// the floats (so one launch fills the chip even for a single large cloud);
// bbox_init / bbox_decode bracket it.  Use launch_bbox().
constexpr int kBBoxParts = 32;

__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void bbox_init_kernel(uint32_t* __restrict__ out, int nb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 6 * nb) out[i] = (i % 6) < 3 ? f2ord(INFINITY) : f2ord(-INFINITY);
}

__global__ void __launch_bounds__(256) bbox_kernel(const float* __restrict__ pts, const int64_t* __restrict__ rs,
                                                   uint32_t* __restrict__ out /*[B][6] encoded*/) {
    const int b = blockIdx.y;
    const int64_t s0 = rs[b], n = rs[b + 1] - s0;
    const int64_t chunk = (n + kBBoxParts - 1) / kBBoxParts;
    const int64_t hi = (blockIdx.x + 1) * chunk;
    const int64_t s = s0 + blockIdx.x * chunk, e = s0 + (hi < n ? hi : n);
    if (s >= e) return;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float v = pts[3 * i + d];
            mn[d] = fminf(mn[d], v);
            mx[d] = fmaxf(mx[d], v);
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mn[d] = fminf(mn[d], __shfl_xor(mn[d], o, 64));
            mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o, 64));
        }
    }
    // block reduction in LDS, then one set of atomics per block (few per address)
    __shared__ float red[6][4];
    if (lane_id() == 0) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            red[d][wave_id()] = mn[d];
            red[3 + d][wave_id()] = mx[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int d = threadIdx.x;
        float v = red[d][0];
        for (int w = 1; w < static_cast<int>(blockDim.x / 64); ++w) v = d < 3 ? fminf(v, red[d][w]) : fmaxf(v, red[d][w]);
        if (d < 3 ? v < INFINITY : v > -INFINITY) {
            if (d < 3) atomicMin(out + 6 * b + d, f2ord(v));
            else atomicMax(out + 6 * b + d, f2ord(v));
        }
    }
}

__global__ void bbox_decode_kernel(uint32_t* __restrict__ io, int nb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 6 * nb) reinterpret_cast<float*>(io)[i] = ord2f(io[i]);
}

// bbox[6 * nb] floats (empty items: +inf / -inf) of the points of each batch item.
inline void launch_bbox(const float* pts, const int64_t* rs_dev, int nb, float* bbox, hipStream_t st) {
    uint32_t* enc = reinterpret_cast<uint32_t*>(bbox);
    const unsigned g6 = static_cast<unsigned>((6 * nb + 255) / 256);
    bbox_init_kernel<<<g6, 256, 0, st>>>(enc, nb);
    bbox_kernel<<<dim3(kBBoxParts, static_cast<unsigned>(nb)), 256, 0, st>>>(pts, rs_dev, enc);
    bbox_decode_kernel<<<g6, 256, 0, st>>>(enc, nb);
}

__device__ __forceinline__ int grid_axis(float p, float o, float inv_h, int n) {
    int c = static_cast<int>(floorf((p - o) * inv_h));
    return c < 0 ? 0 : (c >= n ? n - 1 : c);
}

__global__ void grid_key_kernel(const float* __restrict__ pts, int64_t n, const int64_t* __restrict__ rs, int nb,
                                const GridBatch* __restrict__ g, uint32_t* __restrict__ keys) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const GridBatch gb = g[batch_of(i, rs, nb)];
        const int cx = grid_axis(pts[3 * i], gb.ox, gb.inv_h, gb.dx);
        const int cy = grid_axis(pts[3 * i + 1], gb.oy, gb.inv_h, gb.dy);
        const int cz = grid_axis(pts[3 * i + 2], gb.oz, gb.inv_h, gb.dz);
        keys[i] = gb.offset + static_cast<uint32_t>(cx + gb.dx * (cy + gb.dy * cz));
    }
}

// CSR splits from sorted keys: splits[c] = first position with key >= c —
// one thread per cell, binary search (balanced however many cells are empty).
__global__ void key_boundaries_kernel(const uint32_t* __restrict__ skeys, int64_t n, int64_t n_cells,
                                      uint32_t* __restrict__ splits) {
    for (int64_t c = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; c <= n_cells;
         c += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (static_cast<int64_t>(skeys[mid]) < c) lo = mid + 1; else hi = mid;
        }
        splits[c] = static_cast<uint32_t>(lo);
    }
}

__global__ void gather_float4_kernel(const float* __restrict__ pts, const uint32_t* __restrict__ order, int64_t n,
                                     float4* __restrict__ out) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = order[j];
        out[j] = make_float4(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], __uint_as_float(static_cast<uint32_t>(i)));
    }
}

}  // namespace

// Choose per-batch grids from the bounding boxes (~target points per cell
// for a uniform fill of the box, at most cap_factor * n_b + 64 cells per item):
// one device thread walks the batch items, so building a grid needs no host
// round trip.  Any grid gives exact results; the plan only sets the cost.
namespace {
__global__ void plan_grid_kernel(const float* __restrict__ bbox, const int64_t* __restrict__ rs, int nb,
                                 double target, double cap_factor, GridBatch* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t off = 0;
    for (int b = 0; b < nb; ++b) {
        const int64_t n = rs[b + 1] - rs[b];
        double ext[3];
        double vol = 1.0, maxe = 0.0;
        for (int d = 0; d < 3; ++d) {
            const double lo = n > 0 ? bbox[6 * b + d] : 0.0, hi = n > 0 ? bbox[6 * b + 3 + d] : 0.0;
            ext[d] = isfinite(hi - lo) ? (hi - lo) : 0.0;
            maxe = fmax(maxe, ext[d]);
        }
        if (maxe <= 0.0) maxe = 1.0;
        for (int d = 0; d < 3; ++d) vol *= fmax(ext[d], maxe * 1e-3);
        double h = cbrt(vol * target / static_cast<double>(n > 1 ? n : 1));
        h = fmax(h, maxe / 1024.0);
        const int64_t cap = static_cast<int64_t>(cap_factor * static_cast<double>(n)) + 64;
        int64_t dims[3], cells = 1;
        for (int it = 0; it < 64; ++it) {
            cells = 1;
            for (int d = 0; d < 3; ++d) {
                dims[d] = static_cast<int64_t>(floor(ext[d] / h)) + 1;
                cells *= dims[d];
            }
            if (cells <= cap) break;
            h *= cbrt(static_cast<double>(cells) / static_cast<double>(cap)) * 1.01;
        }
        GridBatch gb;
        gb.ox = n > 0 ? bbox[6 * b] : 0.f;
        gb.oy = n > 0 ? bbox[6 * b + 1] : 0.f;
        gb.oz = n > 0 ? bbox[6 * b + 2] : 0.f;
        gb.h = static_cast<float>(h);
        gb.inv_h = static_cast<float>(1.0 / h);
        gb.dx = static_cast<int>(dims[0]);
        gb.dy = static_cast<int>(dims[1]);
        gb.dz = static_cast<int>(dims[2]);
        gb.offset = static_cast<uint32_t>(off);
        gb.pad[0] = gb.pad[1] = gb.pad[2] = 0;
        out[b] = gb;
        off += cells;
    }
}
}  // namespace

inline int64_t grid_cells_cap(int64_t n, int nb, double cap_factor) {
    return static_cast<int64_t>(cap_factor * static_cast<double>(n)) + 64 * static_cast<int64_t>(nb) + 64;
}

// Device-side index produced by build_grid().
struct GridIndex {
    GridBatch* params;    // [nb]
    uint32_t* splits;     // [cells+1]
    float4* sorted;       // [n] (x,y,z,id) in cell order
    uint32_t* order;      // [n] point ids in cell order
    int64_t cells;
};

inline size_t grid_workspace_bytes(int64_t n, int nb, double cap_factor) {
    return ws_bytes<GridBatch>(nb) + ws_bytes<float>(6 * nb) + ws_bytes<uint32_t>(grid_cells_cap(n, nb, cap_factor) + 1) +
           ws_bytes<float4>(n) + 3 * ws_bytes<uint32_t>(n) + prim::radix_sort_workspace_bytes<uint32_t>(n);
}

// Builds the grid entirely on the device (bounding boxes -> plan -> cell keys
// -> radix sort -> cell boundaries); no host synchronisation.  Cell ids are
// bounded by the capacity, which sizes the sort and the boundary array.
inline GridIndex build_grid(const float* pts, int64_t n, const int64_t* rs_dev, int nb, double target,
                            double cap_factor, Workspace& ws, hipStream_t st) {
    GridIndex gi;
    gi.params = ws.take<GridBatch>(nb);
    float* bbox_d = ws.take<float>(6 * nb);
    const int64_t cap = grid_cells_cap(n, nb, cap_factor);
    gi.cells = cap;
    gi.splits = ws.take<uint32_t>(cap + 1);
    gi.sorted = ws.take<float4>(n);
    uint32_t* keys = ws.take<uint32_t>(n);
    uint32_t* skeys = ws.take<uint32_t>(n);
    gi.order = ws.take<uint32_t>(n);
    launch_bbox(pts, rs_dev, nb, bbox_d, st);
    O3DML_LAUNCH_CHECK();
    plan_grid_kernel<<<1, 64, 0, st>>>(bbox_d, rs_dev, nb, target, cap_factor, gi.params);
    O3DML_LAUNCH_CHECK();
    if (n > 0) {
        grid_key_kernel<<<stream_grid(n, 256), 256, 0, st>>>(pts, n, rs_dev, nb, gi.params, keys);
        O3DML_LAUNCH_CHECK();
        prim::radix_sort_pairs<uint32_t>(keys, nullptr, skeys, gi.order, n,
                                         prim::bits_needed(static_cast<uint64_t>(cap - 1)), ws, st);
        gather_float4_kernel<<<stream_grid(n, 256), 256, 0, st>>>(pts, gi.order, n, gi.sorted);
        O3DML_LAUNCH_CHECK();
    }
    key_boundaries_kernel<<<stream_grid(cap + 1, 256, 1 << 16), 256, 0, st>>>(skeys, n, cap, gi.splits);
    O3DML_LAUNCH_CHECK();
    return gi;
}

}  // namespace o3dml
