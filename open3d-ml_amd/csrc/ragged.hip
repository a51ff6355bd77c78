// ragged.hip — ragged-tensor helpers on the path:
//   ops.ragged_to_dense      (kpconv.py:2030-2032, point_pillars.py:364-366)
//   ops.reduce_subarrays_sum (sparseconvnet.py:319-324)
// Both are HBM-streaming; reduce_subarrays_sum keeps the reference CPU
// left-to-right fp32 summation order (one lane per row) so results are
// bit-identical to the oracle.
#include "common.hpp"
#include "primitives.hpp"

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

// The stable LSD radix sort every op of the path uses (primitives.hpp), as an
// entry point of its own for tests and callers that sort ids by a key:
// (keys, vals) sorted by key, ties in input order, for keys < 2^end_bit;
// vals_in == nullptr means the element index.  key_bytes 4 or 8; small_kind picks the one-workgroup sort
// for n <= 8,192 (-1 default, 0 LSD radix, 1 bitonic).
O3DML_API size_t o3dml_sort_pairs_workspace_size(int64_t n, int key_bytes) {
    return key_bytes == 8 ? prim::radix_sort_workspace_bytes<uint64_t>(n)
                          : prim::radix_sort_workspace_bytes<uint32_t>(n);
}

O3DML_API int o3dml_sort_pairs(const void* keys_in, const uint32_t* vals_in, void* keys_out, uint32_t* vals_out,
                               int64_t n, int key_bytes, int end_bit, int small_kind, void* workspace,
                               size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(key_bytes == 4 || key_bytes == 8, "sort_pairs: key_bytes must be 4 or 8, got %d", key_bytes);
    O3DML_REQUIRE(end_bit >= 0 && end_bit <= 8 * key_bytes, "sort_pairs: end_bit %d out of range", end_bit);
    O3DML_REQUIRE(n < (int64_t(1) << 32), "sort_pairs: %lld keys exceed 32-bit ids", (long long)n);
    O3DML_REQUIRE(workspace_bytes >= o3dml_sort_pairs_workspace_size(n, key_bytes), "sort_pairs: workspace too small");
    hipStream_t st = as_stream(stream);
    Workspace ws(workspace, workspace_bytes);
    if (key_bytes == 8)
        prim::radix_sort_pairs<uint64_t>(static_cast<const uint64_t*>(keys_in), vals_in,
                                         static_cast<uint64_t*>(keys_out), vals_out, n, end_bit, ws, st, small_kind);
    else
        prim::radix_sort_pairs<uint32_t>(static_cast<const uint32_t*>(keys_in), vals_in,
                                         static_cast<uint32_t*>(keys_out), vals_out, n, end_bit, ws, st, small_kind);
    O3DML_GUARD_END
}
