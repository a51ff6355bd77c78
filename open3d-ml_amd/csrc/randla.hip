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
#include <algorithm>
#include <cstdlib>

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


// ---------------------------------------------------------------------------
// Fused LocalSpatialEncoding + AttentivePooling (randlanet.py:540-650): per
// point n with neighbours j < K,
//   rel_j = leaky_0.2(Wr . r_j + br)            r_j = relative encoding of
//           (n, nbr_j) (first pass, 10 values) or the previous pass's rel_j
//   F_j   = [x[nbr_j] (D/2), rel_j (D/2)]
//   s_j   = Ws . F_j + bs                       (score_fn Linear, D x D)
//   out   = sum_j softmax_j(s_j) * F_j          (per channel)
// The reference materialises every [N, K, *] tensor (relative encoding, MLP
// output, gathered features, their concatenation, the scores) in HBM; here F
// lives in LDS (channel-major, K contiguous, so a lane reads the K values of
// one input channel with 128-bit broadcast loads) and each lane owns output
// channels.  Wr / Ws come transposed ([in][out]) so the weight loads of a
// wave are coalesced.  rel_out (nullable) keeps rel_j for the second pass.
// ---------------------------------------------------------------------------
constexpr int kApK = 16;  // neighbours (RandLA num_neighbors)

template <int D, bool RELENC>
__global__ void __launch_bounds__(D > 64 ? D : 64) att_pool_kernel(
        const float* __restrict__ coords, const float* __restrict__ x, const int32_t* __restrict__ nbr, int64_t n,
        const float* __restrict__ rel_in, const float* __restrict__ wrt, const float* __restrict__ br,
        const float* __restrict__ wst, const float* __restrict__ bs, float* __restrict__ rel_out,
        float* __restrict__ out) {
    constexpr int H = D / 2;
    constexpr int IR = RELENC ? 10 : H;  // rel MLP input width
    constexpr int TP = D;                // threads per point: one output channel each
    constexpr int BS = D > 64 ? D : 64;  // block size
    constexpr int PPB = BS / TP;         // points per block
    __shared__ __attribute__((aligned(16))) float ft[PPB][D][kApK];  // F, channel-major
    __shared__ float rin[PPB][kApK][IR];                              // MLP input rows
    __shared__ int32_t nb_s[PPB][kApK];
    const int ps = threadIdx.x / TP, c = threadIdx.x % TP;
    for (int64_t base = static_cast<int64_t>(blockIdx.x) * PPB; base < n;
         base += static_cast<int64_t>(gridDim.x) * PPB) {
        const int64_t q = base + ps;
        const bool valid = q < n;
        // (a) neighbour ids and the MLP input rows
        if (valid && c < kApK) nb_s[ps][c] = nbr[q * kApK + c];
        __syncthreads();
        if (valid) {
            if constexpr (RELENC) {
                if (c < kApK) {
                    const int64_t j = nb_s[ps][c];
                    const float cx = coords[3 * q], cy = coords[3 * q + 1], cz = coords[3 * q + 2];
                    const float px = coords[3 * j], py = coords[3 * j + 1], pz = coords[3 * j + 2];
                    const float rx = cx - px, ry = cy - py, rz = cz - pz;
                    float* r = rin[ps][c];
                    r[0] = sqrtf((rx * rx + ry * ry) + rz * rz);
                    r[1] = rx;
                    r[2] = ry;
                    r[3] = rz;
                    r[4] = cx;
                    r[5] = cy;
                    r[6] = cz;
                    r[7] = px;
                    r[8] = py;
                    r[9] = pz;
                }
            } else {
                for (int e = c; e < kApK * IR; e += TP) rin[ps][e / IR][e % IR] = rel_in[q * kApK * IR + e];
            }
        }
        __syncthreads();
        // (b) F = [x[nbr] | leaky(Wr . r + br)], channel-major in LDS (consecutive
        //     threads = consecutive channels of one neighbour: coalesced rows)
        if (valid) {
            for (int e = c; e < kApK * H; e += TP) {
                const int j = e / H, cc = e % H;
                ft[ps][cc][j] = x[static_cast<int64_t>(nb_s[ps][j]) * H + cc];
                float acc = br[cc];
#pragma unroll 10
                for (int i = 0; i < IR; ++i) acc = __builtin_fmaf(wrt[i * H + cc], rin[ps][j][i], acc);
                const float v = acc > 0.f ? acc : 0.2f * acc;
                ft[ps][H + cc][j] = v;
                if (rel_out) rel_out[(q * kApK + j) * H + cc] = v;
            }
        }
        __syncthreads();
        // (c) scores s[j] = bs[c] + sum_i Ws[c][i] F[j][i] for this thread's channel c,
        //     softmax over j, weighted sum
        if (valid) {
            float acc[kApK];
#pragma unroll
            for (int j = 0; j < kApK; ++j) acc[j] = bs[c];
            for (int i = 0; i < D; ++i) {
                const float w = wst[i * D + c];
                const float4* fr = reinterpret_cast<const float4*>(ft[ps][i]);
#pragma unroll
                for (int v = 0; v < kApK / 4; ++v) {
                    const float4 f = fr[v];
                    acc[4 * v] = __builtin_fmaf(w, f.x, acc[4 * v]);
                    acc[4 * v + 1] = __builtin_fmaf(w, f.y, acc[4 * v + 1]);
                    acc[4 * v + 2] = __builtin_fmaf(w, f.z, acc[4 * v + 2]);
                    acc[4 * v + 3] = __builtin_fmaf(w, f.w, acc[4 * v + 3]);
                }
            }
            float mx = acc[0];
#pragma unroll
            for (int j = 1; j < kApK; ++j) mx = fmaxf(mx, acc[j]);
            float den = 0.f, num = 0.f;
#pragma unroll
            for (int j = 0; j < kApK; ++j) {
                const float e = __expf(acc[j] - mx);
                den += e;
                num += e * ft[ps][c][j];
            }
            out[q * D + c] = num / den;
        }
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// D >= 64: the same fused pass with both GEMMs on MFMA.  The per-point work is
// two small GEMMs over the K = 16 neighbour rows — the rel MLP (second pass:
// [16 x D/2] x [D/2 x D/2]) and the scores ([16 x D] x [D x D]) — which the
// lane-per-channel kernel runs as VALU FMA chains (7-20 TF/s at D = 256).
// Here a workgroup takes 2 points = 32 rows, one wave per 64 output channels
// (D / 64 waves); every 32 x 32 tile is a chain of v_mfma_f32_32x32x2_f32 with
// A read from the LDS rows (F channel-major [pt][ch][j], rin row-major
// [row][i]) and B = the transposed weights ([in][out], coalesced, L2-resident).
// Accumulator layout: lane l, register r holds column l % 32 of row
// (r & 3) + 8 (r >> 2) + 4 (l >> 5), so point p's 16 rows are registers
// 8p .. 8p+7 of lanes l and l ^ 32 — softmax and the weighted sum combine
// those two lanes with one xor-32 shuffle.
// ---------------------------------------------------------------------------
typedef float ap_f32x16 __attribute__((ext_vector_type(16)));

template <int D, bool RELENC>
__global__ void __launch_bounds__(D) att_pool_mfma_kernel(
        const float* __restrict__ coords, const float* __restrict__ x, const int32_t* __restrict__ nbr, int64_t n,
        const float* __restrict__ rel_in, const float* __restrict__ wrt, const float* __restrict__ br,
        const float* __restrict__ wst, const float* __restrict__ bs, float* __restrict__ rel_out,
        float* __restrict__ out) {
    constexpr int H = D / 2;
    constexpr int IR = RELENC ? 10 : H;
    constexpr int NT = D;  // threads: D / 64 waves
    // F of the two points, point 1 shifted by 32 banks (the MFMA A reads of the
    // two points' rows hit distinct banks)
    constexpr int PS = D * kApK + 32;
    __shared__ __attribute__((aligned(16))) float ft_s[2 * PS];
#define FT(p, ch, j) ft_s[(p) * PS + (ch) * kApK + (j)]
    __shared__ float rin[2 * kApK][IR + (RELENC ? 0 : 1)];  // +1: rows on distinct banks
    __shared__ int32_t nb_s[2 * kApK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    for (int64_t base = static_cast<int64_t>(blockIdx.x) * 2; base < n; base += static_cast<int64_t>(gridDim.x) * 2) {
        const int np = n - base >= 2 ? 2 : 1;
        // (a) neighbour ids and the MLP input rows (rows of a missing 2nd point: 0)
        if (tid < 2 * kApK) nb_s[tid] = tid < np * kApK ? nbr[base * kApK + tid] : 0;
        __syncthreads();
        if constexpr (RELENC) {
            if (tid < 2 * kApK) {
                const int64_t q = base + (tid >> 4);
                const bool ok = tid < np * kApK;
                const int64_t j = nb_s[tid];
                const float cx = ok ? coords[3 * q] : 0.f, cy = ok ? coords[3 * q + 1] : 0.f,
                            cz = ok ? coords[3 * q + 2] : 0.f;
                const float px = coords[3 * j], py = coords[3 * j + 1], pz = coords[3 * j + 2];
                const float rx = cx - px, ry = cy - py, rz = cz - pz;
                float* r = rin[tid];
                r[0] = sqrtf((rx * rx + ry * ry) + rz * rz);
                r[1] = rx;
                r[2] = ry;
                r[3] = rz;
                r[4] = cx;
                r[5] = cy;
                r[6] = cz;
                r[7] = px;
                r[8] = py;
                r[9] = pz;
            }
        } else {
            for (int e = tid; e < 2 * kApK * IR; e += NT) {
                const int row = e / IR;
                rin[row][e % IR] = row < np * kApK ? rel_in[base * kApK * IR + e] : 0.f;
            }
        }
        // gathered half of F
        for (int e = tid; e < 2 * kApK * H; e += NT) {
            const int row = e / H, cc = e % H;
            FT(row >> 4, cc, row & 15) = x[static_cast<int64_t>(nb_s[row]) * H + cc];
        }
        __syncthreads();
        // (b) relative half of F: leaky(Wr . r + br)
        if constexpr (RELENC) {
            for (int e = tid; e < 2 * kApK * H; e += NT) {
                const int row = e / H, cc = e % H;
                float acc = br[cc];
#pragma unroll
                for (int i = 0; i < IR; ++i) acc = __builtin_fmaf(wrt[i * H + cc], rin[row][i], acc);
                const float v = acc > 0.f ? acc : 0.2f * acc;
                FT(row >> 4, H + cc, row & 15) = v;
                if (rel_out && row < np * kApK) rel_out[(base * kApK + row) * H + cc] = v;
            }
        } else {
            // H / 32 = D / 64 column tiles: one per wave
            const int col = 32 * w + li;
            ap_f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 8
            for (int k = 0; k < IR; k += 2) {
                const float a = rin[li][k + lh];
                const float b = wrt[(k + lh) * H + col];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            }
            const float bb = br[col];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
                const float v0 = acc[r] + bb;
                const float v = v0 > 0.f ? v0 : 0.2f * v0;
                FT(row >> 4, H + col, row & 15) = v;
                if (rel_out && row < np * kApK) rel_out[(base * kApK + row) * H + col] = v;
            }
        }
        __syncthreads();
        // (c) scores: wave w owns output columns [64w, 64w + 64)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int col = 64 * w + 32 * t + li;
            ap_f32x16 acc;
            const float b0 = bs[col];
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = b0;
#pragma unroll 8
            for (int k = 0; k < D; k += 2) {
                const float a = FT(li >> 4, k + lh, li & 15);
                const float b = wst[(k + lh) * D + col];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            }
            // softmax over the 16 neighbours of each point, weighted sum of F
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                float mx = acc[8 * p];
#pragma unroll
                for (int r = 1; r < 8; ++r) mx = fmaxf(mx, acc[8 * p + r]);
                mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
                float den = 0.f, num = 0.f;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const int j = (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float e = __expf(acc[8 * p + r] - mx);
                    den += e;
                    num += e * FT(p, col, j);
                }
                den += __shfl_xor(den, 32, 64);
                num += __shfl_xor(num, 32, 64);
                if (lh == 0 && p < np) out[(base + p) * D + col] = num / den;
            }
        }
        __syncthreads();
    }
}
#undef FT

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

O3DML_API int o3dml_randla_att_pool(const float* coords, const float* x, const int32_t* neighbors, int64_t n, int k,
                                    int d, const float* rel_in, const float* wr_t, const float* br, const float* ws_t,
                                    const float* bs, float* rel_out, float* out, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(k == kApK, "fused attentive pooling needs k == %d, got %d", kApK, k);
    O3DML_REQUIRE(d == 16 || d == 32 || d == 64 || d == 128 || d == 256,
                  "fused attentive pooling: width %d not in {16, 32, 64, 128, 256}", d);
    if (n == 0) return 0;
    hipStream_t st = as_stream(stream);
    static const bool mfma = [] {
        const char* e = std::getenv("O3DML_ATT_MFMA");
        return e ? std::atoi(e) != 0 : true;
    }();
    if (mfma && d >= 64) {
        const unsigned gm = static_cast<unsigned>(std::min<int64_t>(ceil_div(n, 2), 1 << 20));
#define O3DML_APM(D)                                                                                             \
    do {                                                                                                         \
        if (rel_in)                                                                                              \
            att_pool_mfma_kernel<D, false><<<gm, D, 0, st>>>(coords, x, neighbors, n, rel_in, wr_t, br, ws_t, bs,  \
                                                             rel_out, out);                                      \
        else                                                                                                     \
            att_pool_mfma_kernel<D, true><<<gm, D, 0, st>>>(coords, x, neighbors, n, nullptr, wr_t, br, ws_t, bs,  \
                                                            rel_out, out);                                       \
    } while (0)
        if (d == 64) O3DML_APM(64); else if (d == 128) O3DML_APM(128); else O3DML_APM(256);
#undef O3DML_APM
        O3DML_LAUNCH_CHECK();
        return 0;
    }
    const int ppb = d < 64 ? 64 / d : 1, block = d > 64 ? d : 64;
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n, ppb), 1 << 20));
#define O3DML_AP(D)                                                                                              \
    do {                                                                                                         \
        if (rel_in)                                                                                              \
            att_pool_kernel<D, false><<<g, block, 0, st>>>(coords, x, neighbors, n, rel_in, wr_t, br, ws_t, bs,     \
                                                        rel_out, out);                                           \
        else                                                                                                     \
            att_pool_kernel<D, true><<<g, block, 0, st>>>(coords, x, neighbors, n, nullptr, wr_t, br, ws_t, bs,     \
                                                       rel_out, out);                                            \
    } while (0)
    switch (d) {
        case 16: O3DML_AP(16); break;
        case 32: O3DML_AP(32); break;
        case 64: O3DML_AP(64); break;
        case 128: O3DML_AP(128); break;
        default: O3DML_AP(256); break;
    }
#undef O3DML_AP
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
