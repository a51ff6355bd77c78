// randla.hip — RandLA-Net neighbour gathers: the parts of
// ml3d/torch/models/randlanet.py that are pure index work around the 1x1
// convolutions, fused so each (point, neighbour) pair is touched once.
//
// Layout: channels-last rows.  coords f32 [N,3]; neighbour indices int32 [N,K]
// (row-major, K contiguous); per-pair tensors [N,K,C]; per-point [N,C].
//   * relative encoding  (LocalSpatialEncoding, randlanet.py:593-606):
//     [|c-p|, c-p, c, p] for centre c and neighbour p -> [N,K,10]
//   * attentive pooling   (AttentivePooling, randlanet.py:632-650): softmax
//     over K of the score logits, weighted sum of the features -> [N,C]
//   * gather-max          (random_sample, randlanet.py:306-331): max over the
//     K gathered rows -> [M,C]
// All are HBM-bound; one thread per output element, channel-fastest so
// consecutive lanes read consecutive addresses.
#include "common.hpp"

namespace o3dml {

__global__ void relenc_kernel(const float* __restrict__ coords, int64_t n, const int32_t* __restrict__ nbr, int k,
                              float* __restrict__ out) {
    const int64_t total = n * k;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e / k;
        const int64_t j = nbr[e];
        const float cx = coords[3 * i], cy = coords[3 * i + 1], cz = coords[3 * i + 2];
        const float px = coords[3 * j], py = coords[3 * j + 1], pz = coords[3 * j + 2];
        const float rx = cx - px, ry = cy - py, rz = cz - pz;
        float* o = out + e * 10;
        o[0] = sqrtf((rx * rx + ry * ry) + rz * rz);
        o[1] = rx;
        o[2] = ry;
        o[3] = rz;
        o[4] = cx;
        o[5] = cy;
        o[6] = cz;
        o[7] = px;
        o[8] = py;
        o[9] = pz;
    }
}

__global__ void attentive_pool_kernel(const float* __restrict__ x, const float* __restrict__ logits, int64_t n,
                                      int k, int c, float* __restrict__ out) {
    const int64_t total = n * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e / c;
        const int ch = static_cast<int>(e - i * c);
        const float* lg = logits + i * k * c + ch;
        const float* xv = x + i * k * c + ch;
        float mx = -__builtin_huge_valf();
        for (int j = 0; j < k; ++j) mx = fmaxf(mx, lg[static_cast<int64_t>(j) * c]);
        float den = 0.f, num = 0.f;
        for (int j = 0; j < k; ++j) {
            const float w = __expf(lg[static_cast<int64_t>(j) * c] - mx);
            den += w;
            num += w * xv[static_cast<int64_t>(j) * c];
        }
        out[e] = num / den;
    }
}

__global__ void gather_max_kernel(const float* __restrict__ feat, int c, const int32_t* __restrict__ idx, int64_t m,
                                  int k, float* __restrict__ out) {
    const int64_t total = m * c;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = e / c;
        const int ch = static_cast<int>(e - i * c);
        const int32_t* row = idx + i * k;
        float v = -__builtin_huge_valf();
        for (int j = 0; j < k; ++j) v = fmaxf(v, feat[static_cast<int64_t>(row[j]) * c + ch]);
        out[e] = v;
    }
}


// Row concatenation with optional gathers: out[r] = [A[ia[r]] (da), B[ib[r]] (db)]
// (identity when an index array is null).  Replaces the gather + torch.cat
// pairs of LocalSpatialEncoding (neighbour features | relative features,
// randlanet.py:598-606) and of the decoder (skip features | 1-NN
// interpolation, randlanet.py:285-289): one write of the concatenated rows.
template <class TA, class TB>
__global__ void concat_rows_kernel(const float* __restrict__ A, int da, const TA* __restrict__ ia,
                                   const float* __restrict__ B, int db, const TB* __restrict__ ib, int64_t rows,
                                   float* __restrict__ out) {
    const int w = da + db;
    const int64_t total = rows * w;
    for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = e / w;
        const int c = static_cast<int>(e - r * w);
        float v;
        if (c < da) {
            const int64_t src = ia ? static_cast<int64_t>(ia[r]) : r;
            v = A[src * da + c];
        } else {
            const int64_t src = ib ? static_cast<int64_t>(ib[r]) : r;
            v = B[src * db + (c - da)];
        }
        out[e] = v;
    }
}

}  // namespace o3dml

using namespace o3dml;

O3DML_API int o3dml_randla_relative_encoding(const float* coords, int64_t n, const int32_t* neighbors, int k,
                                             float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k > 0, "k must be > 0");
    if (n == 0) return 0;
    relenc_kernel<<<stream_grid(n * k, 256), 256, 0, as_stream(stream)>>>(coords, n, neighbors, k, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_randla_attentive_pool(const float* x, const float* logits, int64_t n, int k, int c, float* out,
                                          void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k > 0 && c > 0, "k and c must be > 0");
    if (n == 0) return 0;
    attentive_pool_kernel<<<stream_grid(n * c, 256), 256, 0, as_stream(stream)>>>(x, logits, n, k, c, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_randla_gather_max(const float* feat, int c, const int32_t* idx, int64_t m, int k, float* out,
                                      void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k > 0 && c > 0, "k and c must be > 0");
    if (m == 0) return 0;
    gather_max_kernel<<<stream_grid(m * c, 256), 256, 0, as_stream(stream)>>>(feat, c, idx, m, k, out);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}

O3DML_API int o3dml_concat_rows(const float* a, int da, const void* ia, int ia_bits, const float* b, int db,
                                const void* ib, int ib_bits, int64_t rows, float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(da >= 0 && db >= 0 && da + db > 0, "concat_rows: widths must be >= 0 and not both 0");
    O3DML_REQUIRE((ia_bits == 32 || ia_bits == 64) && (ib_bits == 32 || ib_bits == 64), "index_bits must be 32 or 64");
    if (rows == 0) return 0;
    const unsigned g = stream_grid(rows * (da + db), 256, 256 * 16);
    hipStream_t st = as_stream(stream);
#define O3DML_CAT(TA, TB)                                                                                  \
    concat_rows_kernel<TA, TB><<<g, 256, 0, st>>>(a, da, static_cast<const TA*>(ia), b, db,                 \
                                                  static_cast<const TB*>(ib), rows, out)
    if (ia_bits == 32) {
        if (ib_bits == 32) O3DML_CAT(int32_t, int32_t); else O3DML_CAT(int32_t, int64_t);
    } else {
        if (ib_bits == 32) O3DML_CAT(int64_t, int32_t); else O3DML_CAT(int64_t, int64_t);
    }
#undef O3DML_CAT
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
