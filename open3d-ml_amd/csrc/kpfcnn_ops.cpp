// kpfcnn_ops.cpp — the KPFCNN layer pairs as single C-ABI calls: UnaryBlock
// (Linear without bias + BatchNorm1d + LeakyReLU, ml3d/torch/models/kpconv.py:
// 1255-1295) and the rigid KPConv (aggregation + the WF @ W GEMM,
// kpconv.py:1005-1159), forward and backward.  Each composes the existing
// entry points (o3dml_sgemm*, o3dml_batch_norm_*, o3dml_kpconv_weighted_*) on
// one stream: the training step issues one host call per layer and direction
// instead of two or three (the C3 step is host-bound: ~14 us of Python + ctypes
// per call, tools/kp_host.py).  Workspaces are used one sub-call at a time.
#include <algorithm>

#include "common.hpp"

namespace o3dml {

// the long-reduction rule of the Python layer (o3dml_amd/_util.mm): split-K
// for k >= 4,096 with at most 2^20 outputs
static bool gemm_split(int64_t m, int64_t n, int64_t k) { return k >= 4096 && m * n <= (int64_t(1) << 20); }

static size_t gemm_ws(int64_t m, int64_t n, int64_t k) {
    return gemm_split(m, n, k) ? o3dml_sgemm_splitk_workspace_size(m, n, k) : 0;
}

static int gemm_auto(int ta, int tb, int64_t m, int64_t n, int64_t k, const float* a, int64_t lda, const float* b,
                     int64_t ldb, float* c, int64_t ldc, void* ws, size_t wsb, void* stream) {
    if (gemm_split(m, n, k)) return o3dml_sgemm_splitk(ta, tb, m, n, k, a, lda, b, ldb, c, ldc, ws, wsb, stream);
    return o3dml_sgemm(ta, tb, m, n, k, 1.f, a, lda, b, ldb, 0.f, c, ldc, stream);
}

#define O3DML_TRY(expr)          \
    do {                         \
        const int _rc = (expr);  \
        if (_rc != 0) return _rc; \
    } while (0)

}  // namespace o3dml

using namespace o3dml;

O3DML_API size_t o3dml_linear_bn_workspace_size(int64_t n, int cin, int cout) {
    return std::max({o3dml_batch_norm_workspace_size(n, cout), gemm_ws(n, cout, cin), gemm_ws(n, cin, cout),
                     gemm_ws(cout, cin, n)});
}

// z = x @ w^T ([n, cout], w [cout, cin]), y = act(bn(z)) (o3dml_batch_norm_forward
// semantics, save [4 cout])
O3DML_API int o3dml_linear_bn_forward(const float* x, int64_t n, int cin, const float* w, int cout,
                                      const float* gamma, const float* beta, float* running_mean, float* running_var,
                                      int64_t* num_batches_tracked, float momentum, float eps, int training, int act,
                                      float slope, float* z, float* y, float* save, void* workspace,
                                      size_t workspace_bytes, void* stream) {
    O3DML_TRY(gemm_auto(0, 1, n, cout, cin, x, cin, w, cin, z, cout, workspace, workspace_bytes, stream));
    return o3dml_batch_norm_forward(z, n, cout, gamma, beta, running_mean, running_var, num_batches_tracked, momentum,
                                    eps, training, act, slope, y, save, workspace, workspace_bytes, stream);
}

// dz = bn-act backward of gy (scratch [n, cout]); dx = dz @ w, dw = dz^T x
// (each output nullable)
O3DML_API int o3dml_linear_bn_backward(const float* gy, const float* x, int64_t n, int cin, const float* w, int cout,
                                       const float* z, const float* save, int training, int act, float slope,
                                       float* dz, float* dx, float* dw, float* dgamma, float* dbeta, void* workspace,
                                       size_t workspace_bytes, void* stream) {
    O3DML_TRY(o3dml_batch_norm_backward(gy, z, n, cout, save, training, act, slope, dz, dgamma, dbeta, workspace,
                                        workspace_bytes, stream));
    if (dx) O3DML_TRY(gemm_auto(0, 0, n, cin, cout, dz, cout, w, cin, dx, cin, workspace, workspace_bytes, stream));
    if (dw) O3DML_TRY(gemm_auto(1, 0, cout, cin, n, dz, cout, x, cin, dw, cin, workspace, workspace_bytes, stream));
    return 0;
}

O3DML_API size_t o3dml_kpconv_rigid_workspace_size(int64_t n, int nb, int64_t n_support, int K, int cin, int cout,
                                                   int deterministic) {
    const int64_t kc = static_cast<int64_t>(K) * cin;
    size_t s = std::max({gemm_ws(n, cout, kc), gemm_ws(n, kc, cout), gemm_ws(kc, cout, n)});
    if (deterministic) s = std::max(s, o3dml_kpconv_inverse_workspace_size(n, nb, n_support));
    return s;
}

// wf [n, K, cin] = the weighted neighbour features, out [n, cout] = wf @ w
// (w [K cin, cout])
O3DML_API int o3dml_kpconv_rigid_forward(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                         const void* neighbors, int index_bits, int nb, const float* x, int cin,
                                         const float* kernel_points, int K, float extent, int influence, int closest,
                                         const float* w, int cout, float* wf, float* out, void* workspace,
                                         size_t workspace_bytes, void* stream) {
    O3DML_TRY(o3dml_kpconv_weighted_features(q_pts, n, s_pts, n_support, neighbors, index_bits, nb, x, cin,
                                             kernel_points, K, 0, extent, influence, closest, nullptr, wf, stream));
    const int64_t kc = static_cast<int64_t>(K) * cin;
    return gemm_auto(0, 0, n, cout, kc, wf, kc, w, cout, out, cout, workspace, workspace_bytes, stream);
}

// dw = wf^T g, gwf = g w^T (scratch [n, K cin]), dx = the aggregation's
// backward of gwf (zeroed here; fp32 atomics, or the fixed-order gather when
// deterministic)
O3DML_API int o3dml_kpconv_rigid_backward(const float* q_pts, int64_t n, const float* s_pts, int64_t n_support,
                                          const void* neighbors, int index_bits, int nb, const float* g, int cin,
                                          const float* kernel_points, int K, float extent, int influence, int closest,
                                          const float* w, int cout, const float* wf, float* gwf, float* dx, float* dw,
                                          int deterministic, void* workspace, size_t workspace_bytes, void* stream) {
    const int64_t kc = static_cast<int64_t>(K) * cin;
    if (dw) O3DML_TRY(gemm_auto(1, 0, kc, cout, n, wf, kc, g, cout, dw, cout, workspace, workspace_bytes, stream));
    if (!dx) return 0;
    O3DML_TRY(gemm_auto(0, 1, n, kc, cout, g, cout, w, cout, gwf, kc, workspace, workspace_bytes, stream));
    if (deterministic)
        return o3dml_kpconv_weighted_features_backward_det(q_pts, n, s_pts, n_support, neighbors, index_bits, nb, gwf,
                                                           cin, kernel_points, K, 0, extent, influence, closest, dx,
                                                           workspace, workspace_bytes, stream);
    try {
        fill_async(dx, 0, sizeof(float) * n_support * cin, as_stream(stream));
    } catch (const Error& e) {
        return e.code;
    }
    return o3dml_kpconv_weighted_features_backward(q_pts, n, s_pts, n_support, neighbors, index_bits, nb, gwf, cin,
                                                   kernel_points, K, 0, extent, influence, closest, dx, stream);
}
