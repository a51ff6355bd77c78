// ragged.hip — ragged-tensor helpers on the path:
//   ops.ragged_to_dense      (kpconv.py:2030-2032, point_pillars.py:364-366)
//   ops.reduce_subarrays_sum (sparseconvnet.py:319-324)
// Both are HBM-streaming; reduce_subarrays_sum keeps the reference CPU
// left-to-right fp32 summation order (one lane per row) so results are
// bit-identical to the oracle.
#include "common.hpp"

namespace o3dml {

template <class T>
__global__ void ragged_to_dense_kernel(const T* __restrict__ values, const int64_t* __restrict__ rs, int64_t n_rows,
                                       int64_t out_col, int64_t inner, const T* __restrict__ dflt,
                                       T* __restrict__ out) {
    const int64_t total = n_rows * out_col * inner;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = e / (out_col * inner);
        const int64_t rem = e - r * out_col * inner;
        const int64_t c = rem / inner;
        const int64_t k = rem - c * inner;
        const int64_t s = rs[r];
        const int64_t len = rs[r + 1] - s;
        out[e] = c < len ? values[(s + c) * inner + k] : dflt[k];
    }
}

__global__ void reduce_subarrays_sum_kernel(const float* __restrict__ values, const int64_t* __restrict__ rs,
                                            int64_t n_rows, float* __restrict__ out) {
    for (int64_t r = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; r < n_rows;
         r += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float s = 0.f;
        for (int64_t j = rs[r], e = rs[r + 1]; j < e; ++j) s += values[j];
        out[r] = s;
    }
}

}  // namespace o3dml

using namespace o3dml;

// values: [P, inner] elements of elem_bytes (1,2,4,8); default_value: [inner].
O3DML_API int o3dml_ragged_to_dense(const void* values, const int64_t* row_splits, int64_t n_rows,
                                    int64_t out_col_size, int64_t inner, int elem_bytes, const void* default_value,
                                    void* out, void* stream) {
    O3DML_GUARD_BEGIN
    hipStream_t st = as_stream(stream);
    const int64_t total = n_rows * out_col_size * inner;
    if (total == 0) return 0;
    const unsigned g = stream_grid(total, 256);
#define O3DML_R2D(T)                                                                                        \
    ragged_to_dense_kernel<T><<<g, 256, 0, st>>>(static_cast<const T*>(values), row_splits, n_rows, out_col_size, \
                                                 inner, static_cast<const T*>(default_value), static_cast<T*>(out))
    switch (elem_bytes) {
        case 1: O3DML_R2D(uint8_t); break;
        case 2: O3DML_R2D(uint16_t); break;
        case 4: O3DML_R2D(uint32_t); break;
        case 8: O3DML_R2D(uint64_t); break;
        default: O3DML_REQUIRE(false, "unsupported element size %d", elem_bytes);
    }
#undef O3DML_R2D
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_reduce_subarrays_sum(const float* values, const int64_t* row_splits, int64_t n_rows,
                                         float* out, void* stream) {
    O3DML_GUARD_BEGIN
    if (n_rows == 0) return 0;
    reduce_subarrays_sum_kernel<<<stream_grid(n_rows, 256), 256, 0, as_stream(stream)>>>(values, row_splits,
                                                                                         n_rows, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
