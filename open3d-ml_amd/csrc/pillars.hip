// pillars.hip — PointPillars pillar decoration and BEV scatter (SURVEY.md §8a
// A9 consumers, §8f rank 3; reference ml3d/torch/models/point_pillars.py
// PointPillarsVoxelization.forward :352-380, PillarFeatureNet.forward
// :509-552, PointPillarsScatter.forward :567-601).
//
// The reference densifies every pillar to [V, M, 3+C] with a gather through a
// prepended zero row (ragged_to_dense + 1), then builds the decorations with
// five torch ops and masks the padded rows.  Here one thread owns one
// (pillar, slot) row and writes the whole decorated row once:
//   [p (C values), p.xyz - mean(xyz of the pillar), p.x - (ix*vx + x_off),
//    p.y - (iy*vy + y_off)]   for slots < count, zeros for the padding.
// The pillar mean is the fp32 sum of the pillar's points in slot order
// divided by the count (the reference's sum over the zero-padded slots gives
// the same value up to summation order).
//
// Scatter: canvas[b, c, iy, ix] = feat[v, c] (NCHW, the layout the SECOND
// backbone convolutions read); lanes walk pillars of one channel so the
// feature reads of a wave are 64 pillars x 4 B.  The backward is the same
// index map as a gather.
#include "common.hpp"

namespace o3dml {

__global__ void __launch_bounds__(256) pillar_decorate_kernel(const float* __restrict__ pts, int cdim,
                                                              const int64_t* __restrict__ pidx,
                                                              const int64_t* __restrict__ prs,
                                                              const int32_t* __restrict__ coords_xyz, int64_t V, int M,
                                                              float vx, float vy, float x_off, float y_off,
                                                              float* __restrict__ out) {
    const int width = cdim + 5;
    const int64_t rows = V * M;
    for (int64_t r = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; r < rows;
         r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t v = r / M;
        const int slot = static_cast<int>(r - v * M);
        const int64_t beg = prs[v];
        int64_t cnt = prs[v + 1] - beg;
        if (cnt > M) cnt = M;
        float* o = out + r * width;
        if (slot >= cnt) {
            for (int k = 0; k < width; ++k) o[k] = 0.f;
            continue;
        }
        float sx = 0.f, sy = 0.f, sz = 0.f;
        for (int64_t j = 0; j < cnt; ++j) {
            const float* q = pts + pidx[beg + j] * cdim;
            sx += q[0];
            sy += q[1];
            sz += q[2];
        }
        const float fc = static_cast<float>(cnt);
        const float* p = pts + pidx[beg + slot] * cdim;
        for (int k = 0; k < cdim; ++k) o[k] = p[k];
        o[cdim] = p[0] - sx / fc;
        o[cdim + 1] = p[1] - sy / fc;
        o[cdim + 2] = p[2] - sz / fc;
        const float cx = static_cast<float>(coords_xyz[3 * v]) * vx + x_off;
        const float cy = static_cast<float>(coords_xyz[3 * v + 1]) * vy + y_off;
        o[cdim + 3] = p[0] - cx;
        o[cdim + 4] = p[1] - cy;
    }
}

template <bool GATHER>
__global__ void __launch_bounds__(256) pillar_scatter_kernel(float* __restrict__ feat, const int32_t* __restrict__ bzyx,
                                                             int64_t V, int C, int ny, int nx,
                                                             float* __restrict__ canvas) {
    const int64_t total = V * C;
    const int64_t plane = static_cast<int64_t>(ny) * nx;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int c = static_cast<int>(e / V);
        const int64_t v = e - static_cast<int64_t>(c) * V;
        const int32_t* k = bzyx + 4 * v;
        const int64_t at = (static_cast<int64_t>(k[0]) * C + c) * plane + static_cast<int64_t>(k[2]) * nx + k[3];
        if constexpr (GATHER)
            feat[v * C + c] = canvas[at];
        else
            canvas[at] = feat[v * C + c];
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int o3dml_pillar_features(const float* points, int64_t n_points, int cdim,
                                    const int64_t* voxel_point_indices, const int64_t* voxel_point_row_splits,
                                    const int32_t* voxel_coords_xyz, int64_t n_voxels, int max_points, float vx,
                                    float vy, float x_offset, float y_offset, float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(cdim >= 3, "pillar features: points need at least 3 channels, got %d", cdim);
    O3DML_REQUIRE(max_points > 0, "pillar features: max_points must be > 0");
    (void)n_points;
    if (n_voxels == 0) return 0;
    pillar_decorate_kernel<<<stream_grid(n_voxels * max_points, 256, 256 * 16), 256, 0, as_stream(stream)>>>(
        points, cdim, voxel_point_indices, voxel_point_row_splits, voxel_coords_xyz, n_voxels, max_points, vx, vy,
        x_offset, y_offset, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_pillar_scatter(const float* features, const int32_t* coords_bzyx, int64_t n_voxels, int channels,
                                   int ny, int nx, float* canvas, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(channels > 0 && ny > 0 && nx > 0, "pillar scatter: bad canvas shape");
    if (n_voxels == 0) return 0;
    pillar_scatter_kernel<false><<<stream_grid(n_voxels * channels, 256, 256 * 16), 256, 0, as_stream(stream)>>>(
        const_cast<float*>(features), coords_bzyx, n_voxels, channels, ny, nx, canvas);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_pillar_gather(const float* canvas, const int32_t* coords_bzyx, int64_t n_voxels, int channels,
                                  int ny, int nx, float* features, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(channels > 0 && ny > 0 && nx > 0, "pillar gather: bad canvas shape");
    if (n_voxels == 0) return 0;
    pillar_scatter_kernel<true><<<stream_grid(n_voxels * channels, 256, 256 * 16), 256, 0, as_stream(stream)>>>(
        features, coords_bzyx, n_voxels, channels, ny, nx, const_cast<float*>(canvas));
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
