// spatial_hash.hpp — Open3D spatial-hash arithmetic shared by the table build
// (nns_hash.hip) and the fixed-radius search (nns_frs.hip).  Bit-identical to
// oracle/o3d_oracle.c (orc_spatial_hash / orc_voxel_index / orc_query_bins).
#pragma once

#include "common.hpp"

namespace o3dml {

// Open3D SpatialHash: 32-bit int products XOR-ed, converted to size_t (sign
// extension), reduced modulo the table size.
__device__ __forceinline__ uint32_t spatial_bin(int32_t x, int32_t y, int32_t z, uint32_t tsize) {
    const uint32_t h = (static_cast<uint32_t>(x) * 73856096u) ^ (static_cast<uint32_t>(y) * 193649663u) ^
                       (static_cast<uint32_t>(z) * 83492791u);
    const uint64_t u = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(h)));
    return static_cast<uint32_t>(u % tsize);
}

__device__ __forceinline__ uint32_t point_bin(float x, float y, float z, float inv, uint32_t tsize) {
    return spatial_bin(static_cast<int32_t>(floorf(x * inv)), static_cast<int32_t>(floorf(y * inv)),
                       static_cast<int32_t>(floorf(z * inv)), tsize);
}

// Same bucket as spatial_bin, with the 64-bit modulo split into 32-bit ones:
// for h < 0 the size_t value is 2^64 - |h|, so the bucket is
// (2^64 mod T - |h| mod T) mod T; k64 = 2^64 mod T is computed once per table.
__device__ __forceinline__ uint32_t pow64_mod(uint32_t tsize) {
    const uint32_t r32 = static_cast<uint32_t>((0xffffffffu % tsize + 1u) % tsize);  // 2^32 mod T
    return static_cast<uint32_t>((static_cast<uint64_t>(r32) * r32) % tsize);
}

__device__ __forceinline__ uint32_t spatial_bin_k(int32_t x, int32_t y, int32_t z, uint32_t tsize, uint32_t k64) {
    const uint32_t h = (static_cast<uint32_t>(x) * 73856096u) ^ (static_cast<uint32_t>(y) * 193649663u) ^
                       (static_cast<uint32_t>(z) * 83492791u);
    if ((tsize & (tsize - 1u)) == 0u) return h & (tsize - 1u);  // 2^k table: the low k bits
    const int32_t hs = static_cast<int32_t>(h);
    if (hs >= 0) return static_cast<uint32_t>(hs) % tsize;
    const uint32_t a = static_cast<uint32_t>(-static_cast<int64_t>(hs)) % tsize;
    const uint64_t v = static_cast<uint64_t>(k64) + tsize - a;
    return static_cast<uint32_t>(v >= tsize ? v - tsize : v);
}

__device__ __forceinline__ uint32_t point_bin_k(float x, float y, float z, float inv, uint32_t tsize, uint32_t k64) {
    return spatial_bin_k(static_cast<int32_t>(floorf(x * inv)), static_cast<int32_t>(floorf(y * inv)),
                         static_cast<int32_t>(floorf(z * inv)), tsize, k64);
}

__device__ __forceinline__ void cswap(uint32_t& a, uint32_t& b) {
    const uint32_t lo = a < b ? a : b;
    const uint32_t hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// The 9 bins a query visits (own voxel + the 8 corners q ± r), sorted
// ascending; duplicates are skipped by the caller (bins[k] == bins[k-1]).
struct QueryBins {
    uint32_t b[9];
};

__device__ __forceinline__ QueryBins query_bins(float qx, float qy, float qz, float r, float inv, uint32_t first,
                                                uint32_t tsize) {
    QueryBins s;
    const float xs[2] = {qx - r, qx + r};
    const float ys[2] = {qy - r, qy + r};
    const float zs[2] = {qz - r, qz + r};
    if ((tsize & (tsize - 1u)) == 0u) {
        // power-of-two table (Open3D's default factor 1/64 on 2^k-point items,
        // e.g. C1): the sign-extended 64-bit value mod 2^k is its low k bits
        const uint32_t m = tsize - 1u;
        auto pb = [&](float x, float y, float z) {
            const uint32_t h = (static_cast<uint32_t>(static_cast<int32_t>(floorf(x * inv))) * 73856096u) ^
                               (static_cast<uint32_t>(static_cast<int32_t>(floorf(y * inv))) * 193649663u) ^
                               (static_cast<uint32_t>(static_cast<int32_t>(floorf(z * inv))) * 83492791u);
            return h & m;
        };
        s.b[0] = pb(qx, qy, qz);
#pragma unroll
        for (int c = 0; c < 8; ++c) s.b[1 + c] = pb(xs[c & 1], ys[(c >> 1) & 1], zs[c >> 2]);
    } else {
        const uint32_t k64 = pow64_mod(tsize);
        s.b[0] = point_bin_k(qx, qy, qz, inv, tsize, k64);
#pragma unroll
        for (int c = 0; c < 8; ++c) s.b[1 + c] = point_bin_k(xs[c & 1], ys[(c >> 1) & 1], zs[c >> 2], inv, tsize, k64);
    }
    // a 25-comparator sorting network for 9 inputs (checked on all 2^9 0-1
    // inputs; the odd-even transposition network it replaced took 36)
    constexpr int kNet[25][2] = {{0, 1}, {3, 4}, {6, 7}, {1, 2}, {4, 5}, {7, 8}, {0, 1}, {3, 4}, {6, 7},
                                 {0, 3}, {3, 6}, {0, 3}, {1, 4}, {4, 7}, {1, 4}, {2, 5}, {5, 8}, {2, 5},
                                 {1, 3}, {5, 7}, {2, 6}, {4, 6}, {2, 4}, {2, 3}, {5, 6}};
#pragma unroll
    for (int i = 0; i < 25; ++i) cswap(s.b[kNet[i][0]], s.b[kNet[i][1]]);
#pragma unroll
    for (int i = 0; i < 9; ++i) s.b[i] += first;
    return s;
}

}  // namespace o3dml
