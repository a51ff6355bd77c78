/*
 * cpu_frs.c — TEST / BASELINE INFRASTRUCTURE ONLY (bench.py cpu_baseline leg).
 *
 * An optimised multi-threaded CPU fixed-radius self search with exactly the
 * semantics of orc_build_spatial_hash_table + orc_fixed_radius_search
 * (o3d_oracle.c; Open3D ops.build_spatial_hash_table + fixed_radius_search as
 * layers.FixedRadiusSearch calls them, kpconv.py:2016-2034),
 * written the way a tuned CPU library would run it, so the C1 GPU/CPU ratio is
 * not measured against the deliberately plain oracle:
 *   - parallel hash build: per-thread bin histograms over contiguous point
 *     ranges, a (bin, thread) scan, a stable per-thread scatter — ids stay
 *     ascending inside a bin (the canonical order);
 *   - the points copied into bucket order (SoA), so a visited bucket is one
 *     contiguous stream;
 *   - ONE search pass: blocks of queries write their neighbours into
 *     block-local buffers with per-query counts, then a scan and a parallel
 *     concatenation (no count pass + fill pass).
 * L2 only, queries = points (the bench workload).  Output identical to the
 * oracle (tests/test_golden.py::test_cpu_frs_fast_equals_oracle).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_API __attribute__((visibility("default")))

ORC_API int64_t orc_hash_table_splits(int64_t n_batch, const int64_t* points_row_splits, double factor,
                                      int64_t max_size, uint32_t* hash_table_splits);

static inline uint32_t fast_bin(float x, float y, float z, float inv, uint64_t tsize, uint32_t first) {
    const int32_t vx = (int32_t)floorf(x * inv), vy = (int32_t)floorf(y * inv), vz = (int32_t)floorf(z * inv);
    const uint32_t h = ((uint32_t)vx * 73856096u) ^ ((uint32_t)vy * 193649663u) ^ ((uint32_t)vz * 83492791u);
    return first + (uint32_t)((uint64_t)(int64_t)(int32_t)h % tsize);
}

static inline int64_t fast_batch_of(int64_t i, int64_t n_batch, const int64_t* s) {
    int64_t lo = 0, hi = n_batch - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) / 2;
        if (s[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

#define FAST_BLOCK 2048 /* queries per search block */
#define FAST_PAD 8       /* slack after the SoA arrays and the output buffers (8-wide stores) */

/* The candidates [e0, e1) of one bucket against query q: ids of the hits
 * appended at buf[cnt..]; returns the new count.  Scalar, branch-free. */
static size_t scan_scalar(const float* sx, const float* sy, const float* sz, const uint32_t* hti, uint32_t e0,
                          uint32_t e1, float qx, float qy, float qz, float thr, int32_t* buf, size_t cnt) {
    for (uint32_t j = e0; j < e1; ++j) {
        const float dx = sx[j] - qx, dy = sy[j] - qy, dz = sz[j] - qz;
        const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
        buf[cnt] = (int32_t)hti[j];
        cnt += d <= thr;
    }
    return cnt;
}

#if defined(__x86_64__)
#include <immintrin.h>
/* 8 candidates at a time (AVX2 + FMA3, chosen at run time): the fused
 * multiply-adds are exactly fmaf's, so the hits are the scalar ones; the
 * hits' ids are compressed by a permutation table and stored 8-wide. */
static int32_t g_compress[256][8];
static void init_compress(void) {
    for (int m = 0; m < 256; ++m) {
        int k = 0;
        for (int l = 0; l < 8; ++l)
            if (m & (1 << l)) g_compress[m][k++] = l;
        for (; k < 8; ++k) g_compress[m][k] = 0;
    }
}
__attribute__((target("avx2,fma"))) static size_t scan_avx2(const float* sx, const float* sy, const float* sz,
                                                             const uint32_t* hti, uint32_t e0, uint32_t e1, float qx,
                                                             float qy, float qz, float thr, int32_t* buf, size_t cnt) {
    const __m256 vx = _mm256_set1_ps(qx), vy = _mm256_set1_ps(qy), vz = _mm256_set1_ps(qz);
    const __m256 vt = _mm256_set1_ps(thr);
    const __m256i lanes = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    for (uint32_t j = e0; j < e1; j += 8) {
        const __m256 dx = _mm256_sub_ps(_mm256_loadu_ps(sx + j), vx);
        const __m256 dy = _mm256_sub_ps(_mm256_loadu_ps(sy + j), vy);
        const __m256 dz = _mm256_sub_ps(_mm256_loadu_ps(sz + j), vz);
        const __m256 d = _mm256_fmadd_ps(dz, dz, _mm256_fmadd_ps(dy, dy, _mm256_mul_ps(dx, dx)));
        int m = _mm256_movemask_ps(_mm256_cmp_ps(d, vt, _CMP_LE_OQ));
        const uint32_t left = e1 - j;
        if (left < 8) {
            const __m256i live = _mm256_cmpgt_epi32(_mm256_set1_epi32((int)left), lanes);
            m &= _mm256_movemask_ps(_mm256_castsi256_ps(live));
        }
        if (m) {
            const __m256i ids = _mm256_loadu_si256((const __m256i*)(hti + j));
            const __m256i perm = _mm256_loadu_si256((const __m256i*)g_compress[m]);
            _mm256_storeu_si256((__m256i*)(buf + cnt), _mm256_permutevar8x32_epi32(ids, perm));
            cnt += (size_t)__builtin_popcount((unsigned)m);
        }
    }
    return cnt;
}
#endif

typedef size_t (*scan_fn)(const float*, const float*, const float*, const uint32_t*, uint32_t, uint32_t, float,
                          float, float, float, int32_t*, size_t);
static scan_fn pick_scan(int allow_simd) {
#if defined(__x86_64__)
    if (allow_simd && __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) {
        init_compress();
        return scan_avx2;
    }
#endif
    (void)allow_simd;
    return scan_scalar;
}

/* Returns the number of neighbour pairs P; row_splits [n+1] always written,
 * idx [P] only when P <= capacity (else call again with a larger buffer). */
ORC_API int64_t orc_frs_fast(const float* points, int64_t n, float radius, int64_t n_batch, const int64_t* prs,
                             double factor, int64_t max_size, int nthreads, int simd, int64_t* row_splits,
                             int32_t* idx, int64_t capacity) {
    const scan_fn scan = pick_scan(simd);
#ifdef _OPENMP
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    const int nt = 1;
    (void)nthreads;
#endif
    const float inv = 1.0f / (2.0f * radius);
    const float thr = radius * radius;
    uint32_t* hts = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n_batch + 1));
    const int64_t T = orc_hash_table_splits(n_batch, prs, factor, max_size, hts);
    uint32_t* bin = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    uint32_t* hist = (uint32_t*)calloc((size_t)nt * (size_t)T, sizeof(uint32_t));
    uint32_t* cs = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(T + 1));
    uint32_t* hti = (uint32_t*)calloc((size_t)n + FAST_PAD, sizeof(uint32_t));
    float* sx = (float*)calloc((size_t)n + FAST_PAD, sizeof(float));
    float* sy = (float*)calloc((size_t)n + FAST_PAD, sizeof(float));
    float* sz = (float*)calloc((size_t)n + FAST_PAD, sizeof(float));
    const int64_t nblk = (n + FAST_BLOCK - 1) / FAST_BLOCK;
    int32_t** bbuf = (int32_t**)calloc((size_t)(nblk > 0 ? nblk : 1), sizeof(int32_t*));
    int64_t* btot = (int64_t*)calloc((size_t)(nblk + 1), sizeof(int64_t));
    int64_t* rtot = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    int64_t total = 0;
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        /* 1. bins + per-thread histograms over contiguous point ranges */
        const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        uint32_t* h = hist + (size_t)t * (size_t)T;
        int64_t b = lo < hi ? fast_batch_of(lo, n_batch, prs) : 0;
        for (int64_t i = lo; i < hi; ++i) {
            while (i >= prs[b + 1]) ++b;
            const uint32_t k = fast_bin(points[3 * i], points[3 * i + 1], points[3 * i + 2], inv,
                                        hts[b + 1] - hts[b], hts[b]);
            bin[i] = k;
            h[k]++;
        }
#pragma omp barrier
        /* 2. (bin, thread) exclusive scan: each thread scans a bin range, the
         *    range totals are carried by one thread */
        const int64_t b0 = T * t / nt, b1 = T * (t + 1) / nt;
        uint64_t s = 0;
        for (int64_t k = b0; k < b1; ++k)
            for (int u = 0; u < nt; ++u) s += hist[(size_t)u * (size_t)T + (size_t)k];
        rtot[t] = (int64_t)s;
#pragma omp barrier
#pragma omp single
        {
            int64_t run = 0;
            for (int u = 0; u < nt; ++u) {
                const int64_t x = rtot[u];
                rtot[u] = run;
                run += x;
            }
        }
        uint32_t run = (uint32_t)rtot[t];
        for (int64_t k = b0; k < b1; ++k) {
            cs[k] = run;
            for (int u = 0; u < nt; ++u) {
                uint32_t* e = hist + (size_t)u * (size_t)T + (size_t)k;
                const uint32_t c = *e;
                *e = run; /* thread u's first slot in bin k */
                run += c;
            }
        }
        if (t == nt - 1) cs[T] = run;
#pragma omp barrier
        /* 3. stable scatter (ids ascending inside a bin) + SoA copy in bucket order */
        for (int64_t i = lo; i < hi; ++i) {
            const uint32_t pos = h[bin[i]]++;
            hti[pos] = (uint32_t)i;
            sx[pos] = points[3 * i];
            sy[pos] = points[3 * i + 1];
            sz[pos] = points[3 * i + 2];
        }
#pragma omp barrier
        /* 4. one search pass: blocks of queries into block-local buffers */
#pragma omp for schedule(dynamic, 1)
        for (int64_t blk = 0; blk < nblk; ++blk) {
            const int64_t q0 = blk * FAST_BLOCK, q1 = q0 + FAST_BLOCK < n ? q0 + FAST_BLOCK : n;
            size_t cap = (size_t)(q1 - q0) * 48, cnt = 0;
            int32_t* buf = (int32_t*)malloc(sizeof(int32_t) * cap);
            int64_t qb = fast_batch_of(q0, n_batch, prs);
            for (int64_t q = q0; q < q1; ++q) {
                while (q >= prs[qb + 1]) ++qb;
                const float qx = points[3 * q], qy = points[3 * q + 1], qz = points[3 * q + 2];
                const uint64_t tsize = hts[qb + 1] - hts[qb];
                const uint32_t first = hts[qb];
                uint32_t bins[9];
                int nb = 0;
                bins[nb++] = fast_bin(qx, qy, qz, inv, tsize, first);
                for (int dz = -1; dz <= 1; dz += 2)
                    for (int dy = -1; dy <= 1; dy += 2)
                        for (int dx = -1; dx <= 1; dx += 2)
                            bins[nb++] = fast_bin(qx + radius * (float)dx, qy + radius * (float)dy,
                                                  qz + radius * (float)dz, inv, tsize, first);
                for (int i = 1; i < nb; ++i) { /* insertion sort of 9 */
                    const uint32_t v = bins[i];
                    int j = i - 1;
                    while (j >= 0 && bins[j] > v) { bins[j + 1] = bins[j]; --j; }
                    bins[j + 1] = v;
                }
                const size_t c0 = cnt;
                for (int k = 0; k < nb; ++k) {
                    if (k > 0 && bins[k] == bins[k - 1]) continue;
                    const uint32_t e0 = cs[bins[k]], e1 = cs[bins[k] + 1];
                    if (cnt + (e1 - e0) + FAST_PAD > cap) {
                        cap = 2 * cap + (e1 - e0) + FAST_PAD;
                        buf = (int32_t*)realloc(buf, sizeof(int32_t) * cap);
                    }
                    cnt = scan(sx, sy, sz, hti, e0, e1, qx, qy, qz, thr, buf, cnt);
                }
                row_splits[q + 1] = (int64_t)(cnt - c0);
            }
            bbuf[blk] = buf;
            btot[blk + 1] = (int64_t)cnt;
        }
        /* 5. scan of the row counts (blocks in parallel, then block bases) */
#pragma omp single
        {
            row_splits[0] = 0;
            for (int64_t blk = 0; blk < nblk; ++blk) btot[blk + 1] += btot[blk];
            total = btot[nblk];
        }
#pragma omp for schedule(static)
        for (int64_t blk = 0; blk < nblk; ++blk) {
            const int64_t q0 = blk * FAST_BLOCK, q1 = q0 + FAST_BLOCK < n ? q0 + FAST_BLOCK : n;
            int64_t r = btot[blk];
            for (int64_t q = q0; q < q1; ++q) {
                r += row_splits[q + 1];
                row_splits[q + 1] = r;
            }
            if (total <= capacity && idx)
                memcpy(idx + btot[blk], bbuf[blk], sizeof(int32_t) * (size_t)(btot[blk + 1] - btot[blk]));
            free(bbuf[blk]);
        }
    }
    free(rtot);
    free(btot);
    free(bbuf);
    free(sz);
    free(sy);
    free(sx);
    free(hti);
    free(cs);
    free(hist);
    free(bin);
    free(hts);
    return total;
}
