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
    const uint32_t k64 = pow64_mod(tsize);
    s.b[0] = point_bin_k(qx, qy, qz, inv, tsize, k64);
    const float xs[2] = {qx - r, qx + r};
    const float ys[2] = {qy - r, qy + r};
    const float zs[2] = {qz - r, qz + r};
#pragma unroll
    for (int c = 0; c < 8; ++c) s.b[1 + c] = point_bin_k(xs[c & 1], ys[(c >> 1) & 1], zs[c >> 2], inv, tsize, k64);
    // odd-even transposition network, 9 stages -> fully sorted
#pragma unroll
    for (int st = 0; st < 9; ++st) {
#pragma unroll
        for (int i = (st & 1); i + 1 < 9; i += 2) cswap(s.b[i], s.b[i + 1]);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) s.b[i] += first;
    return s;
}

}  // namespace o3dml
