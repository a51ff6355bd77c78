// VALU issue-rate micro-kernel (round-6 verdict item 1): cycles per wave64
// VALU instruction per SIMD at 1, 2, 4 and 8 resident waves per SIMD on every
// CU.  Each lane runs 8 independent chains of one instruction kind (inline asm,
// so the compiler can neither pack them into v_pk_* nor fold them away); a
// 256-thread workgroup puts one wave on each SIMD of its CU, and the grid is
// CUs x W workgroups, so W waves share each SIMD.  Two clocks per wave:
// s_memtime (shader cycles) and the 100-MHz constant counter, giving the
// effective clock; the SIMD cost is  wave cycles / (W x VALU per wave)  while all
// W waves overlap, cross-checked against the HIP-event wall time.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_bin/valu_rate tools/valu_rate.hip
//   tools/_bin/valu_rate [iters=1024]   (16 x 8 VALU per iteration)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kUnroll = 16;  // step8 blocks per loop iteration (loop overhead < 3 %)
enum Kind { FMA = 0, ADD = 1, AND = 2, CMP_CND = 3, CMP_S = 4, MBCNT = 5, BCNT = 6, MBCNT_HI = 7, MIN_U32 = 8,
            LSHL_OR = 9, CNDMASK = 10, DPP_MOV = 11, MIN_F64 = 12, CMP_U64 = 13, FRS_TEST = 14,
            S_ADD = 15, EXEC_MASK = 16 };

template <int KIND>
__device__ __forceinline__ void step8(float (&a)[8], float b, float c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if constexpr (KIND == FMA) {
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b), "v"(c));
        } else if constexpr (KIND == ADD) {
            asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
        } else if constexpr (KIND == AND) {
            asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
        } else if constexpr (KIND == CMP_S) {
            // compare into an SGPR pair (a ballot), 8 independent destinations
            unsigned long long m;
            asm volatile("v_cmp_lt_f32 %0, %1, %2" : "=s"(m) : "v"(b), "v"(a[j]));
        } else if constexpr (KIND == MBCNT) {
            asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(a[j]) : "s"(0x5555u));
        } else if constexpr (KIND == MBCNT_HI) {
            asm volatile("v_mbcnt_hi_u32_b32 %0, %1, %0" : "+v"(a[j]) : "s"(0x5555u));
        } else if constexpr (KIND == BCNT) {
            asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
        } else if constexpr (KIND == MIN_U32) {
            asm volatile("v_min_u32 %0, 63, %0" : "+v"(a[j]));
        } else if constexpr (KIND == LSHL_OR) {
            asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a[j]) : "v"(b));
        } else if constexpr (KIND == CNDMASK) {
            asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "s"(0x5555aaaa5555aaaaull));
        } else if constexpr (KIND == DPP_MOV) {
            asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[j]));
        } else if constexpr (KIND == MIN_F64) {
            // 4 chains of 64-bit values in the 8 floats (2 instructions per j pair)
            if (j & 1) continue;
            double d = __builtin_bit_cast(double, make_float2(a[j], a[j + 1]));
            asm volatile("v_min_f64 %0, %0, %1" : "+v"(d) : "v"(0.75));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(d) : "v"(0.25));
            float2 f = __builtin_bit_cast(float2, d);
            a[j] = f.x;
            a[j + 1] = f.y;
        } else if constexpr (KIND == CMP_U64) {
            if (j & 1) continue;
            unsigned long long m;
            unsigned long long u = __builtin_bit_cast(unsigned long long, make_float2(a[j], a[j + 1]));
            asm volatile("v_cmp_lt_u64 %0, %1, %2" : "=s"(m) : "v"(u), "v"(0x3f80000012345678ull));
            asm volatile("v_cmp_gt_u64 %0, %1, %2" : "=s"(m) : "v"(u), "v"(0x3f80000012345678ull));
        } else if constexpr (KIND == S_ADD) {
            // scalar ALU, 16 instructions on 8 SGPRs in one block (no compiler
            // padding between them): the CU's one scalar unit serves four SIMDs
            if (j != 0) continue;
            asm volatile(
                    "s_add_u32 s20, s20, 1\n\ts_add_u32 s21, s21, 1\n\ts_add_u32 s22, s22, 1\n\ts_add_u32 s23, s23, 1\n\t"
                    "s_add_u32 s24, s24, 1\n\ts_add_u32 s25, s25, 1\n\ts_add_u32 s26, s26, 1\n\ts_add_u32 s27, s27, 1\n\t"
                    "s_add_u32 s20, s20, 1\n\ts_add_u32 s21, s21, 1\n\ts_add_u32 s22, s22, 1\n\ts_add_u32 s23, s23, 1\n\t"
                    "s_add_u32 s24, s24, 1\n\ts_add_u32 s25, s25, 1\n\ts_add_u32 s26, s26, 1\n\ts_add_u32 s27, s27, 1"
                    ::: "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "scc");
        } else if constexpr (KIND == EXEC_MASK) {
            // the exec-mask pattern around each FRS hit store, 4 times: VOPC
            // into VCC, s_and_saveexec, s_or_b64 exec (12 instructions, 4 VALU)
            if (j != 0) continue;
            asm volatile(
                    "v_cmp_lt_f32 vcc, %0, %1\n\ts_and_saveexec_b64 s[20:21], vcc\n\ts_or_b64 exec, exec, s[20:21]\n\t"
                    "v_cmp_lt_f32 vcc, %2, %1\n\ts_and_saveexec_b64 s[20:21], vcc\n\ts_or_b64 exec, exec, s[20:21]\n\t"
                    "v_cmp_lt_f32 vcc, %3, %1\n\ts_and_saveexec_b64 s[20:21], vcc\n\ts_or_b64 exec, exec, s[20:21]\n\t"
                    "v_cmp_lt_f32 vcc, %4, %1\n\ts_and_saveexec_b64 s[20:21], vcc\n\ts_or_b64 exec, exec, s[20:21]"
                    :: "v"(a[0]), "v"(b), "v"(a[1]), "v"(a[2]), "v"(a[3]) : "vcc", "s20", "s21", "exec", "scc");
        } else if constexpr (KIND == FRS_TEST) {
            // one candidate test of nns_frs.hip's search loop as compiled (distance,
            // compare into VCC, group mask, rank of the hit, clamped row address,
            // running count) with the hit branch and the store left out; the
            // row address goes into a sum so it stays live: 17 VALU
            if (j != 0) continue;
            uint32_t t0, t1, t2, h, l, pp;
            asm volatile(
                    "v_sub_f32 %[t0], %[px], %[qx]\n\t"
                    "v_sub_f32 %[t1], %[py], %[qy]\n\t"
                    "v_mul_f32 %[t0], %[t0], %[t0]\n\t"
                    "v_sub_f32 %[t2], %[pz], %[qz]\n\t"
                    "v_fmac_f32 %[t0], %[t1], %[t1]\n\t"
                    "v_fmac_f32 %[t0], %[t2], %[t2]\n\t"
                    "v_cmp_ge_f32 vcc, %[thr], %[t0]\n\t"
                    "s_nop 1\n\t"
                    "v_and_b32 %[h], vcc_hi, %[gh]\n\t"
                    "v_and_b32 %[l], vcc_lo, %[gl]\n\t"
                    "v_mbcnt_lo_u32_b32 %[p], %[l], %[cnt]\n\t"
                    "v_mbcnt_hi_u32_b32 %[p], %[h], %[p]\n\t"
                    "v_min_u32 %[p], 63, %[p]\n\t"
                    "v_lshl_or_b32 %[p], %[p], 1, %[base]\n\t"
                    "v_bcnt_u32_b32 %[l], %[l], %[cnt]\n\t"
                    "v_bcnt_u32_b32 %[cnt], %[h], %[l]\n\t"
                    "v_add_u32 %[acc], %[acc], %[p]"
                    : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [h] "=&v"(h), [l] "=&v"(l), [p] "=&v"(pp),
                      [cnt] "+v"(a[6]), [acc] "+v"(a[7])
                    : [px] "v"(a[0]), [py] "v"(a[1]), [pz] "v"(a[2]), [qx] "v"(a[3]), [qy] "v"(a[4]),
                      [qz] "v"(a[5]), [thr] "s"(c), [gh] "v"(b), [gl] "v"(c), [base] "v"(b)
                    : "vcc");
        } else {
            // compare into VCC + select: the shape of a candidate test's tail
            asm volatile("v_cmp_lt_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc"
                         : "+v"(a[j]) : "v"(b) : "vcc");
        }
    }
}

template <int KIND>
__global__ __launch_bounds__(256) void valu_kernel(int iters, float b, float c,
                                                   float* sink, unsigned long long* stamps) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3f + j;
    __syncthreads();
    unsigned long long c0 = clock64();
    unsigned long long w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) step8<KIND>(a, b, c);
    }
    unsigned long long c1 = clock64();
    unsigned long long w1 = wall_clock64();
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (s == 12345.678f) sink[gw] = s;  // keeps the chains live; never true in practice
    if ((threadIdx.x & 63) == 0) {
        stamps[4 * gw + 0] = c0;
        stamps[4 * gw + 1] = c1;
        stamps[4 * gw + 2] = w0;
        stamps[4 * gw + 3] = w1;
    }
}

static const char* kname(int k) {
    switch (k) {
        case FMA: return "v_fma_f32";
        case ADD: return "v_add_f32";
        case AND: return "v_and_b32";
        case CMP_S: return "v_cmp_lt_f32 (SGPR dst)";
        case MBCNT: return "v_mbcnt_lo_u32_b32";
        case MBCNT_HI: return "v_mbcnt_hi_u32_b32";
        case BCNT: return "v_bcnt_u32_b32";
        case MIN_U32: return "v_min_u32";
        case LSHL_OR: return "v_lshl_or_b32";
        case CNDMASK: return "v_cndmask_b32 (SGPR mask)";
        case DPP_MOV: return "v_mov_b32_dpp";
        case MIN_F64: return "v_min_f64+v_max_f64";
        case CMP_U64: return "v_cmp_lt_u64 (SGPR dst)";
        case FRS_TEST: return "FRS candidate test (17 VALU)";
        case S_ADD: return "s_add_u32 (per SIMD-stream; the scalar unit is per CU)";
        case EXEC_MASK: return "v_cmp vcc + s_and_saveexec + s_or exec (12 per step)";
        default: return "v_cmp_lt_f32+v_cndmask_b32";
    }
}

template <int KIND>
static void run(int cus, int w, int iters, float* sink, unsigned long long* d_st, int wall_mhz) {
    int blocks = cus * w, waves = blocks * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep)  // warm-up then timed
    {
        CHECK(hipEventRecord(e0));
        valu_kernel<KIND><<<blocks, 256>>>(iters, 1.0000001f, 0.5f, sink, d_st);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
    }
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> st(4 * (size_t)waves);
    CHECK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
    double cyc_sum = 0, wall_sum = 0, cyc_max = 0;
    for (int i = 0; i < waves; ++i) {
        double c = double(st[4 * i + 1] - st[4 * i + 0]);
        double t = double(st[4 * i + 3] - st[4 * i + 2]);
        cyc_sum += c;
        wall_sum += t;
        cyc_max = std::max(cyc_max, c);
    }
    double cyc_mean = cyc_sum / waves;
    double clk_ghz = cyc_sum / (wall_sum / (wall_mhz * 1e-3)) ;  // shader cycles per ns
    // VALU-pipe instructions per step8
    const int per_step = KIND == CMP_CND ? 16 : KIND == FRS_TEST ? 17 : KIND == S_ADD ? 16 : KIND == EXEC_MASK ? 12 : 8;
    double valu_per_wave = double(iters) * kUnroll * per_step;
    // per SIMD: w waves overlap, each issuing valu_per_wave
    double cyc_per_valu_simd_wave = cyc_mean / (w * valu_per_wave);
    double cyc_per_valu_simd_event = (ms * 1e6 * clk_ghz) / (w * valu_per_wave);
    printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"waves\": %d, \"valu_per_wave\": %.0f, "
           "\"event_ms\": %.4f, \"clock_ghz\": %.3f, \"wave_cycles_mean\": %.0f, \"wave_cycles_max\": %.0f, "
           "\"cyc_per_valu_per_simd_from_wave\": %.3f, \"cyc_per_valu_per_simd_from_event\": %.3f}\n",
           kname(KIND), w, waves, valu_per_wave, ms, clk_ghz, cyc_mean, cyc_max,
           cyc_per_valu_simd_wave, cyc_per_valu_simd_event);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 1024;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    int wall_mhz = 100;
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, 0) == hipSuccess && v > 0) wall_mhz = v / 1000;
    printf("# %s, %d CUs, wall clock %d MHz, iters %d\n", p.gcnArchName, cus, wall_mhz, iters);
    float* sink;
    unsigned long long* st;
    CHECK(hipMalloc(&sink, sizeof(float) * cus * 8 * 4));
    CHECK(hipMalloc(&st, 8ull * 4 * cus * 8 * 4));
    for (int w : {1, 2, 4, 8}) run<FMA>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 4, 8}) run<ADD>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<AND>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<CMP_S>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<MBCNT>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<CMP_CND>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<BCNT>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<MBCNT_HI>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<MIN_U32>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<LSHL_OR>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<CNDMASK>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<DPP_MOV>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<MIN_F64>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 8}) run<CMP_U64>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 4, 8}) run<FRS_TEST>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<S_ADD>(cus, w, iters, sink, st, wall_mhz);
    for (int w : {1, 2, 8}) run<EXEC_MASK>(cus, w, iters, sink, st, wall_mhz);
    CHECK(hipFree(sink));
    CHECK(hipFree(st));
    return 0;
}
