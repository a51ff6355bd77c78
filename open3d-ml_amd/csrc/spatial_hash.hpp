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
    s.b[0] = point_bin(qx, qy, qz, inv, tsize);
    const float xs[2] = {qx - r, qx + r};
    const float ys[2] = {qy - r, qy + r};
    const float zs[2] = {qz - r, qz + r};
#pragma unroll
    for (int c = 0; c < 8; ++c) s.b[1 + c] = point_bin(xs[c & 1], ys[(c >> 1) & 1], zs[c >> 2], inv, tsize);
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
