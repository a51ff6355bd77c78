// nms.hip — rotated bird's-eye-view NMS, replacing open3d.ml.torch.ops.nms as
// bound by ml3d/torch/utils/objdet_helper.py:27 and called from
// multiclass_nms (objdet_helper.py:346) inside PointPillars.get_bboxes_single
// (point_pillars.py:1005).  Boxes are (x_min, y_min, x_max, y_max, yaw) rotated
// about their centre; overlap is the area of the convex intersection polygon
// (edge crossings + contained corners, ordered by angle, shoelace area) and a
// lower-scored box is dropped when IoU > threshold († Open3D IoUImpl /
// NmsImpl, restated in oracle/o3d_oracle.c orc_nms).
//
// Three launches, all on the caller's stream:
//   1. rank kernel: stable descending score order (rank = #{higher score} +
//      #{equal score with lower index}), O(N^2) compares over an LDS-staged
//      score tile — N is a few hundred per class (nms_pre = 100 upstream);
//   2. mask kernel: one 64-lane wavefront per (row, column block) of the upper
//      triangle; lane l tests column block*64+l and the wave ballot is the
//      64-bit suppression word (bit l: box block*64+l overlaps box row);
//   3. sweep kernel: one wavefront walks the sorted boxes in order, keeping
//      the running "removed" bitmap (and, up to 64 KiB, the mask) in LDS and
//      OR-ing in each kept box's row.
#include "common.hpp"

namespace o3dml {

constexpr int kNmsBlock = 64;  // one wavefront == one 64-bit mask word
constexpr float kNmsEps = 1e-8f;

struct P2 {
    float x, y;
};

__device__ __forceinline__ float cross3(P2 p1, P2 p2, P2 p0) {
    return (p1.x - p0.x) * (p2.y - p0.y) - (p2.x - p0.x) * (p1.y - p0.y);
}

__device__ __forceinline__ bool rect_cross(P2 p1, P2 p2, P2 q1, P2 q2) {
    return fminf(p1.x, p2.x) <= fmaxf(q1.x, q2.x) && fminf(q1.x, q2.x) <= fmaxf(p1.x, p2.x) &&
           fminf(p1.y, p2.y) <= fmaxf(q1.y, q2.y) && fminf(q1.y, q2.y) <= fmaxf(p1.y, p2.y);
}

__device__ __forceinline__ bool in_box(const float* b, P2 p) {
    const float margin = 1e-5f;
    const float cx = (b[0] + b[2]) * 0.5f, cy = (b[1] + b[3]) * 0.5f;
    const float c = cosf(-b[4]), s = sinf(-b[4]);
    const float rx = (p.x - cx) * c + (p.y - cy) * s + cx;
    const float ry = -(p.x - cx) * s + (p.y - cy) * c + cy;
    return rx > b[0] - margin && rx < b[2] + margin && ry > b[1] - margin && ry < b[3] + margin;
}

// Segment p0-p1 against q0-q1; writes the crossing point.
__device__ __forceinline__ bool seg_cross(P2 p1, P2 p0, P2 q1, P2 q0, P2& ans) {
    if (!rect_cross(p0, p1, q0, q1)) return false;
    const float s1 = cross3(q0, p1, p0), s2 = cross3(p1, q1, p0);
    const float s3 = cross3(p0, q1, q0), s4 = cross3(q1, p1, q0);
    if (!(s1 * s2 > 0.f && s3 * s4 > 0.f)) return false;
    const float s5 = cross3(q1, p1, p0);
    if (fabsf(s5 - s1) > kNmsEps) {
        ans.x = (s5 * q0.x - s1 * q1.x) / (s5 - s1);
        ans.y = (s5 * q0.y - s1 * q1.y) / (s5 - s1);
    } else {
        const float a0 = p0.y - p1.y, b0 = p1.x - p0.x, c0 = p0.x * p1.y - p1.x * p0.y;
        const float a1 = q0.y - q1.y, b1 = q1.x - q0.x, c1 = q0.x * q1.y - q1.x * q0.y;
        const float d = a0 * b1 - a1 * b0;
        ans.x = (b0 * c1 - b1 * c0) / d;
        ans.y = (a1 * c0 - a0 * c1) / d;
    }
    return true;
}

__device__ __forceinline__ void box_corners(const float* b, P2* c) {
    const float cx = (b[0] + b[2]) * 0.5f, cy = (b[1] + b[3]) * 0.5f;
    const float co = cosf(b[4]), si = sinf(b[4]);
    const float xs[4] = {b[0], b[2], b[2], b[0]}, ys[4] = {b[1], b[1], b[3], b[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c[k].x = (xs[k] - cx) * co + (ys[k] - cy) * si + cx;
        c[k].y = -(xs[k] - cx) * si + (ys[k] - cy) * co + cy;
    }
    c[4] = c[0];
}

__device__ float bev_iou(const float* a, const float* b) {
    P2 ca[5], cb[5], pts[24];  // <= 16 edge crossings + 8 contained corners
    box_corners(a, ca);
    box_corners(b, cb);
    int cnt = 0;
    P2 ctr{0.f, 0.f};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (seg_cross(ca[i + 1], ca[i], cb[j + 1], cb[j], pts[cnt])) {
                ctr.x += pts[cnt].x;
                ctr.y += pts[cnt].y;
                ++cnt;
            }
    for (int k = 0; k < 4; ++k) {
        if (in_box(a, cb[k])) {
            ctr.x += cb[k].x;
            ctr.y += cb[k].y;
            pts[cnt++] = cb[k];
        }
        if (in_box(b, ca[k])) {
            ctr.x += ca[k].x;
            ctr.y += ca[k].y;
            pts[cnt++] = ca[k];
        }
    }
    float area = 0.f;
    if (cnt > 2) {
        ctr.x /= cnt;
        ctr.y /= cnt;
        float ang[16];
        for (int k = 0; k < cnt; ++k) ang[k] = atan2f(pts[k].y - ctr.y, pts[k].x - ctr.x);
        for (int j = 0; j < cnt - 1; ++j)  // bubble sort, ascending angle
            for (int i = 0; i < cnt - j - 1; ++i)
                if (ang[i] > ang[i + 1]) {
                    const P2 tp = pts[i];
                    pts[i] = pts[i + 1];
                    pts[i + 1] = tp;
                    const float ta = ang[i];
                    ang[i] = ang[i + 1];
                    ang[i + 1] = ta;
                }
        for (int k = 0; k < cnt - 1; ++k) {
            const float ux = pts[k].x - pts[0].x, uy = pts[k].y - pts[0].y;
            const float vx = pts[k + 1].x - pts[0].x, vy = pts[k + 1].y - pts[0].y;
            area += ux * vy - uy * vx;
        }
    }
    const float inter = fabsf(area) * 0.5f;
    const float sa = (a[2] - a[0]) * (a[3] - a[1]);
    const float sb = (b[2] - b[0]) * (b[3] - b[1]);
    return inter / fmaxf(sa + sb - inter, kNmsEps);
}

// Total-order sort key of a score: ascending floats map to ascending keys,
// -0 and +0 share a key (they compare equal), every NaN maps to 0, below -inf.
// With the index tie-break the ranks are a permutation for any input, so
// order[] is always fully written.
__device__ __forceinline__ uint32_t score_key(float s) {
    if (s != s) return 0u;
    const uint32_t u = __float_as_uint(s + 0.0f);  // -0 -> +0
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// order[rank(i)] = i, stable descending by score_key.
__global__ void __launch_bounds__(256) nms_rank_kernel(const float* __restrict__ scores, int n,
                                                        int32_t* __restrict__ order) {
    __shared__ uint32_t tile[256];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ki = i < n ? score_key(scores[i]) : 0u;
    int rank = 0;
    for (int base = 0; base < n; base += 256) {
        const int j = base + threadIdx.x;
        tile[threadIdx.x] = j < n ? score_key(scores[j]) : 0u;
        __syncthreads();
        const int lim = min(256, n - base);
        for (int t = 0; t < lim; ++t) {
            const uint32_t kj = tile[t];
            rank += (kj > ki) || (kj == ki && base + t < i);
        }
        __syncthreads();
    }
    if (i < n) order[rank] = i;
}

// mask[i * words + cb] bit l: sorted box (cb*64 + l) > i overlaps sorted box i.
// One wavefront per (row i, column block cb): lane l evaluates column cb*64+l
// and the 64-bit word is the wave ballot, so the n*words words come from
// n*words independent waves (the IoU is ~200 dependent ALU ops with a small
// private polygon array; wave-level parallelism is what hides it).
constexpr int kNmsRowsPerBlock = 4;
__global__ void __launch_bounds__(kNmsBlock* kNmsRowsPerBlock)
        nms_mask_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ order, int n, int words,
                        float thresh, uint64_t* __restrict__ mask) {
    const int lane = threadIdx.x & (kNmsBlock - 1);
    const int i = blockIdx.y * kNmsRowsPerBlock + (threadIdx.x >> 6);
    const int cb = blockIdx.x;
    if (i >= n || cb < (i >> 6)) return;  // wave-uniform
    const int j = cb * kNmsBlock + lane;
    float me[5], other[5];
    const float* src = boxes + static_cast<int64_t>(order[i]) * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) me[k] = src[k];
    bool hit = false;
    if (j > i && j < n) {
        const float* o = boxes + static_cast<int64_t>(order[j]) * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) other[k] = o[k];
        hit = bev_iou(me, other) > thresh;
    }
    const uint64_t bits = __ballot(hit);
    if (lane == 0) mask[static_cast<int64_t>(i) * words + cb] = bits;
}

// One wavefront: greedy sweep in score order.  keep[] gets original indices.
// STAGE: the whole upper-triangular mask is first copied into LDS (coalesced),
// so the sequential loop touches no global memory; otherwise each kept row is
// read from global memory.
template <bool STAGE>
__global__ void __launch_bounds__(kNmsBlock) nms_sweep_kernel(const uint64_t* __restrict__ mask,
                                                              const int32_t* __restrict__ order, int n, int words,
                                                              int64_t* __restrict__ keep,
                                                              int64_t* __restrict__ keep_count) {
    extern __shared__ uint64_t lds[];
    uint64_t* removed = lds;
    uint64_t* rows = lds + words;
    const int t = threadIdx.x;
    for (int w = t; w < words; w += kNmsBlock) removed[w] = 0;
    if (STAGE) {
        const int64_t total = static_cast<int64_t>(n) * words;
        for (int64_t e = t; e < total; e += kNmsBlock) {
            const int r = static_cast<int>(e / words), w = static_cast<int>(e - static_cast<int64_t>(r) * words);
            if (w >= (r >> 6)) rows[e] = mask[e];
        }
    }
    __syncthreads();
    int64_t cnt = 0;
    for (int i = 0; i < n; ++i) {
        const bool gone = (removed[i >> 6] >> (i & 63)) & 1ull;
        __syncthreads();
        if (gone) continue;
        if (t == 0) keep[cnt] = order[i];
        ++cnt;
        const uint64_t* row = (STAGE ? rows : mask) + static_cast<int64_t>(i) * words;
        for (int w = (i >> 6) + t; w < words; w += kNmsBlock) removed[w] |= row[w];
        __syncthreads();
    }
    if (t == 0) *keep_count = cnt;
}

}  // namespace o3dml

using namespace o3dml;

namespace {
constexpr int64_t kNmsMaxBoxes = 1 << 16;  // mask = N^2/8 bytes (512 MiB at the cap)
constexpr size_t kNmsStageBytes = 64 * 1024;  // mask staged in LDS up to ~700 boxes
inline int64_t nms_words(int64_t n) { return ceil_div(n, kNmsBlock); }
}  // namespace

O3DML_API size_t o3dml_nms_workspace_size(int64_t n) {
    if (n <= 0) return 0;
    return ws_bytes<int32_t>(n) + ws_bytes<uint64_t>(n * nms_words(n));
}

// boxes f32 [N,5] (x1,y1,x2,y2,yaw), scores f32 [N] -> keep int64 [<=N]
// (original indices in descending-score order), *keep_count (device int64).
O3DML_API int o3dml_nms(const float* boxes, const float* scores, int64_t n, float nms_overlap_thresh, int64_t* keep,
                        int64_t* keep_count, void* workspace, size_t workspace_bytes, void* stream) {
    O3DML_GUARD_BEGIN
    O3DML_REQUIRE(n >= 0 && n <= kNmsMaxBoxes, "nms: number of boxes %lld outside [0, %lld]", (long long)n,
                  (long long)kNmsMaxBoxes);
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        fill_async(keep_count, 0, sizeof(int64_t), st);
        return 0;
    }
    const int ni = static_cast<int>(n), words = static_cast<int>(nms_words(n));
    Workspace ws(workspace, workspace_bytes);
    int32_t* order = ws.take<int32_t>(n);
    uint64_t* mask = ws.take<uint64_t>(n * words);
    nms_rank_kernel<<<static_cast<unsigned>(ceil_div(n, 256)), 256, 0, st>>>(scores, ni, order);
    O3DML_LAUNCH_CHECK();
    nms_mask_kernel<<<dim3(words, static_cast<unsigned>(ceil_div(n, kNmsRowsPerBlock))), kNmsBlock * kNmsRowsPerBlock,
                      0, st>>>(boxes, order, ni, words, nms_overlap_thresh, mask);
    O3DML_LAUNCH_CHECK();
    const size_t staged = sizeof(uint64_t) * (static_cast<size_t>(words) + static_cast<size_t>(n) * words);
    if (staged <= kNmsStageBytes)
        nms_sweep_kernel<true><<<1, kNmsBlock, staged, st>>>(mask, order, ni, words, keep, keep_count);
    else
        nms_sweep_kernel<false><<<1, kNmsBlock, sizeof(uint64_t) * words, st>>>(mask, order, ni, words, keep,
                                                                                keep_count);
    O3DML_LAUNCH_CHECK();
    O3DML_GUARD_END
}
