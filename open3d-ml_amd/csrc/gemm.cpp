// gemm.cpp — plain fp32 GEMMs of the KPFCNN layers (UnaryBlock Linear and the
// rigid KPConv's WF @ W, forward and backward) through rocBLAS.  These are
// library GEMMs (no fusion to gain at these shapes), and rocBLAS's host cost
// per call is a fraction of hipBLASLt's heuristic query, which torch issues
// per matmul: the C3 train step runs ~140 of them (measured 19.3 -> 14.5 ms
// per step with torch's backend switched; here the ops call rocBLAS
// themselves, whatever torch's preference).  One rocBLAS handle per (host
// thread, device), its stream set per call.
#include <rocblas/rocblas.h>

#include <algorithm>
#include <unordered_map>

#include "common.hpp"

namespace o3dml {

static rocblas_handle gemm_handle(hipStream_t st) {
    thread_local std::unordered_map<int, rocblas_handle> handles;
    int dev = 0;
    if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) {
        set_error("gemm: cannot resolve the stream's device");
        throw Error{1};
    }
    auto it = handles.find(dev);
    if (it == handles.end()) {
        rocblas_handle h = nullptr;
        if (rocblas_create_handle(&h) != rocblas_status_success) {
            set_error("gemm: rocblas_create_handle failed");
            throw Error{1};
        }
        it = handles.emplace(dev, h).first;
    }
    if (rocblas_set_stream(it->second, st) != rocblas_status_success) {
        set_error("gemm: rocblas_set_stream failed");
        throw Error{1};
    }
    return it->second;
}

}  // namespace o3dml

using namespace o3dml;

// Row-major C[m, n] = alpha op(A) op(B) + beta C, op(A) [m, k], op(B) [k, n]
// (trans_a: A stored [k, m]; trans_b: B stored [n, k]); leading dimensions in
// elements of the stored row-major matrices.  As column-major rocBLAS:
// C^T = op(B)^T op(A)^T.
O3DML_API int o3dml_sgemm(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, float alpha, const float* a,
                          int64_t lda, const float* b, int64_t ldb, float beta, float* c, int64_t ldc, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(m >= 0 && n >= 0 && k >= 0, "sgemm: negative size");
    O3DML_REQUIRE(m < (int64_t(1) << 31) && n < (int64_t(1) << 31) && k < (int64_t(1) << 31) &&
                      lda < (int64_t(1) << 31) && ldb < (int64_t(1) << 31) && ldc < (int64_t(1) << 31),
                  "sgemm: sizes past rocBLAS's 32-bit dimensions");
    if (m == 0 || n == 0) return 0;
    rocblas_handle h = gemm_handle(as_stream(stream));
    const rocblas_operation ob = trans_b ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_operation oa = trans_a ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_status s = rocblas_sgemm(h, ob, oa, static_cast<rocblas_int>(n), static_cast<rocblas_int>(m),
                                           static_cast<rocblas_int>(k), &alpha, b, static_cast<rocblas_int>(ldb), a,
                                           static_cast<rocblas_int>(lda), &beta, c, static_cast<rocblas_int>(ldc));
    O3DML_REQUIRE(s == rocblas_status_success, "sgemm: rocblas_sgemm failed (status %d)", static_cast<int>(s));
    O3DML_GUARD_END
}

namespace o3dml {

constexpr int64_t kSplitChunk = 2048;  // reduction rows per split
constexpr int64_t kSplitMax = 64;

static int64_t splitk_parts(int64_t k) { return std::min<int64_t>(kSplitMax, (k + kSplitChunk - 1) / kSplitChunk); }

// C[m, n] = sum of the s slabs [s][m][n], in slab order (deterministic)
__global__ void splitk_reduce_kernel(const float* __restrict__ part, int64_t s, int64_t mn, float* __restrict__ c,
                                     int64_t n, int64_t ldc) {
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < mn;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        float v = 0.f;
        for (int64_t i = 0; i < s; ++i) v += part[i * mn + e];
        c[(e / n) * ldc + e % n] = v;
    }
}

}  // namespace o3dml

O3DML_API size_t o3dml_sgemm_splitk_workspace_size(int64_t m, int64_t n, int64_t k) {
    return ws_bytes<float>(splitk_parts(k) * m * n);
}

// o3dml_sgemm (alpha 1, beta 0) with a long reduction k split into up to 64
// parts of >= 2,048 (one strided-batched rocBLAS call over the equal parts,
// one more for the tail), the parts' [m, n] slabs summed in order
// (deterministic).  For the KPFCNN GEMMs with few output tiles and a long k:
// the weight gradients (k = points, up to 40,000) and the deep layers' KPConv
// WF @ W (k = 15 x 512 over 150 rows) — as one GEMM, rocBLAS runs those on a
// handful of workgroups.
O3DML_API int o3dml_sgemm_splitk(int trans_a, int trans_b, int64_t m, int64_t n, int64_t k, const float* a,
                                 int64_t lda, const float* b, int64_t ldb, float* c, int64_t ldc, void* workspace,
                                 size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(m >= 0 && n >= 0 && k >= 0, "sgemm_splitk: negative size");
    O3DML_REQUIRE(m < (int64_t(1) << 31) && n < (int64_t(1) << 31) && k < (int64_t(1) << 31),
                  "sgemm_splitk: sizes past rocBLAS's 32-bit dimensions");
    if (m == 0 || n == 0) return 0;
    hipStream_t st = as_stream(stream);
    const int64_t s = splitk_parts(k);
    if (s <= 1) return o3dml_sgemm(trans_a, trans_b, m, n, k, 1.f, a, lda, b, ldb, 0.f, c, ldc, stream);
    Workspace ws(workspace, workspace_bytes);
    float* part = ws.take<float>(s * m * n);
    const int64_t kc = k / s, full = s - (k % s ? 1 : 0);  // equal parts of kc; the tail in the last
    // the offset of reduction index r in each stored operand
    const int64_t sa = trans_a ? lda : 1, sb = trans_b ? 1 : ldb;
    const rocblas_operation ob = trans_b ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_operation oa = trans_a ? rocblas_operation_transpose : rocblas_operation_none;
    rocblas_handle h = gemm_handle(st);
    const float one = 1.f, zero = 0.f;
    // column-major: part_i^T [n, m] = op(B_i)^T op(A_i)^T
    rocblas_status rs = rocblas_sgemm_strided_batched(
            h, ob, oa, static_cast<rocblas_int>(n), static_cast<rocblas_int>(m), static_cast<rocblas_int>(kc), &one,
            b, static_cast<rocblas_int>(ldb), kc * sb, a, static_cast<rocblas_int>(lda), kc * sa, &zero, part,
            static_cast<rocblas_int>(n), m * n, static_cast<rocblas_int>(full));
    O3DML_REQUIRE(rs == rocblas_status_success, "sgemm_splitk: strided-batched GEMM failed (%d)", static_cast<int>(rs));
    if (full < s) {
        const int64_t r0 = full * kc;
        rs = rocblas_sgemm(h, ob, oa, static_cast<rocblas_int>(n), static_cast<rocblas_int>(m),
                           static_cast<rocblas_int>(k - r0), &one, b + r0 * sb, static_cast<rocblas_int>(ldb),
                           a + r0 * sa, static_cast<rocblas_int>(lda), &zero, part + full * m * n,
                           static_cast<rocblas_int>(n));
        O3DML_REQUIRE(rs == rocblas_status_success, "sgemm_splitk: tail GEMM failed (%d)", static_cast<int>(rs));
    }
    splitk_reduce_kernel<<<stream_grid(m * n, 256), 256, 0, st>>>(part, s, m * n, c, n, ldc);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
