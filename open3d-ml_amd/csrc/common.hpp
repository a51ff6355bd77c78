// common.hpp — error plumbing, launch helpers and wave-level utilities shared
// by every kernel family of libo3dml_amd.so (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/o3dml_amd.h"

#define O3DML_API extern "C" __attribute__((visibility("default")))

namespace o3dml {

// Thread-local last error, read back through o3dml_last_error().
void set_error(const char* fmt, ...);
const char* last_error();

struct Error {
    int code;
};

#define O3DML_CHECK_HIP(expr)                                                   \
    do {                                                                        \
        hipError_t _e = (expr);                                                 \
        if (_e != hipSuccess) {                                                 \
            ::o3dml::set_error("%s:%d: %s -> %s", __FILE__, __LINE__, #expr,    \
                               hipGetErrorString(_e));                          \
            throw ::o3dml::Error{1};                                            \
        }                                                                       \
    } while (0)

#define O3DML_REQUIRE(cond, ...)                                                \
    do {                                                                        \
        if (!(cond)) {                                                          \
            ::o3dml::set_error(__VA_ARGS__);                                    \
            throw ::o3dml::Error{2};                                            \
        }                                                                       \
    } while (0)

#define O3DML_LAUNCH_CHECK() O3DML_CHECK_HIP(hipGetLastError())

// Wrap a C-ABI entry point body: returns 0 on success, nonzero on error.
#define O3DML_GUARD_BEGIN try {
#define O3DML_GUARD_END                                                         \
    }                                                                           \
    catch (const ::o3dml::Error& e) {                                           \
        return e.code;                                                          \
    }                                                                           \
    catch (...) {                                                               \
        ::o3dml::set_error("unknown C++ exception");                            \
        return 3;                                                               \
    }                                                                           \
    return 0;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Optional per-kernel timing (o3dml_timing_enable): HIP events recorded on the
// launch stream around a region; resolved by o3dml_timing_get.  Off by
// default (zero cost beyond a flag test).
bool timing_enabled();
void timing_record(const char* name, hipEvent_t a, hipEvent_t b);

struct TimedRegion {
    const char* name;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    TimedRegion(const char* n, hipStream_t s) : name(n), st(s) {
        if (timing_enabled() && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
            (void)hipEventRecord(a, st);
        else
            a = b = nullptr;
    }
    void end() {  // close the region early (idempotent)
        if (a) {
            (void)hipEventRecord(b, st);
            timing_record(name, a, b);
            a = nullptr;
        }
    }
    ~TimedRegion() { end(); }
};

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Set `bytes` of device memory at dst to the byte `value` on st with a
// kernel (fill.hip): capture-safe, unlike a hipMemsetAsync node (>= 16 bytes
// re-applied on the first graph replay only).  Throws Error on launch failure.
void fill_async(void* dst, int value, size_t bytes, hipStream_t st);
// Device-to-device copy by a kernel (no memcpy node in captured graphs).
void copy_async(void* dst, const void* src, size_t bytes, hipStream_t st);

// Pinned host scratch for the few int64 sizes a count phase reads back (a
// pageable destination goes through a staging copy): 8 slots per host
// thread, allocated on first use, never freed.
inline int64_t* pinned_scratch() {
    thread_local int64_t* p = nullptr;
    if (!p) O3DML_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), 8 * sizeof(int64_t), 0));
    return p;
}

// Grid size for grid-stride streaming kernels: enough workgroups to fill the
// 256 CUs several times over, capped (cdna_hip_programming.md Guideline 11).
inline unsigned stream_grid(int64_t n, int block, int64_t cap = 256 * 8) {
    int64_t g = ceil_div(n, block);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<unsigned>(g);
}

// Bump allocator over a caller-provided device workspace (no hipMalloc in
// any launch function: everything stays capturable into a hipGraph).
struct Workspace {
    char* base;
    size_t size;
    size_t used = 0;
    Workspace(void* b, size_t s) : base(static_cast<char*>(b)), size(s) {}
    template <class T>
    T* take(int64_t count) {
        size_t bytes = (static_cast<size_t>(count < 0 ? 0 : count) * sizeof(T) + 255) & ~size_t(255);
        O3DML_REQUIRE(base != nullptr || bytes == 0, "workspace is null");
        O3DML_REQUIRE(used + bytes <= size, "workspace too small: need %zu more bytes (have %zu of %zu)",
                      bytes, size - used, size);
        T* p = reinterpret_cast<T*>(base + used);
        used += bytes;
        return p;
    }
};

// Bytes a Workspace::take<T>(count) will consume (used by *_workspace_size).
template <class T>
inline size_t ws_bytes(int64_t count) {
    return (static_cast<size_t>(count < 0 ? 0 : count) * sizeof(T) + 255) & ~size_t(255);
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
// sum over split-K slabs of element e, in slab order (0.f + p0 + p1 + ...),
// the loads issued 16 at a time so a deep split is not one L2 round trip per
// slab; the same bits as the plain loop
__device__ __forceinline__ float sum_slabs(const float* __restrict__ part, int nsplit, int64_t total, int64_t e) {
    float v = 0.f;
    int s = 0;
    for (; s + 16 <= nsplit; s += 16) {
        float t[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) t[j] = part[(s + j) * total + e];
#pragma unroll
        for (int j = 0; j < 16; ++j) v += t[j];
    }
    for (; s < nsplit; ++s) v += part[s * total + e];
    return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

template <class T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T t = __shfl_up(v, d, 64);
        if (lane_id() >= d) v += t;
    }
    return v;
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const T o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Squared L2 distance with the contraction pattern shared with the oracle:
// fma(dz,dz, fma(dy,dy, dx*dx)), dx = p - q.
__device__ __forceinline__ float dist_l2(float px, float py, float pz, float qx, float qy, float qz) {
    const float dx = px - qx, dy = py - qy, dz = pz - qz;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

enum Metric { kL1 = 0, kL2 = 1, kLinf = 2 };

template <int METRIC>
__device__ __forceinline__ float dist_metric(float px, float py, float pz, float qx, float qy, float qz) {
    if constexpr (METRIC == kL2) {
        return dist_l2(px, py, pz, qx, qy, qz);
    } else {
        const float ax = fabsf(px - qx), ay = fabsf(py - qy), az = fabsf(pz - qz);
        if constexpr (METRIC == kL1) {
            return (ax + ay) + az;
        } else {
            const float m = ax > ay ? ax : ay;
            return m > az ? m : az;
        }
    }
}

// Index of the batch item containing element i (row_splits sorted, size B+1).
__device__ __forceinline__ int batch_of(int64_t i, const int64_t* __restrict__ splits, int n_batch) {
    int lo = 0, hi = n_batch - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (splits[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// v_writelane: set lane LANE of v to the uniform value x (one instruction;
// the lane select is an inline constant, the value an SGPR).
template <int LANE>
__device__ __forceinline__ int write_lane(int v, int x) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(LANE));
    return v;
}

// Fourth word of a raw buffer resource on gfx950 (32-bit data format, no
// swizzle/stride): used with __builtin_amdgcn_make_buffer_rsrc.
constexpr int kBufferFlags = 0x00020000;

// Row splits staged in LDS for the batch lookups of a streaming kernel (the
// binary search then costs LDS latency, not a chain of global loads); splits
// that do not fit are searched in global memory.  Call from every thread.
constexpr int kLdsSplits = 1024;
__device__ __forceinline__ const int64_t* stage_splits(int64_t* lds, const int64_t* __restrict__ splits,
                                                       int n_batch) {
    if (n_batch + 1 > kLdsSplits) return splits;
    for (int i = threadIdx.x; i <= n_batch; i += blockDim.x) lds[i] = splits[i];
    __syncthreads();
    return lds;
}

// XCD-contiguous block order for streaming kernels whose blocks each take one
// contiguous range: workgroups are dealt round-robin to the 8 XCDs, so with a
// grid that is a multiple of 8, XCD x runs blocks x, x+8, ... — remapped here
// to ranges x*G/8 ... (x+1)*G/8-1, i.e. one contiguous slice of the array per
// XCD (its L2 then holds the data that slice touches).
__device__ __forceinline__ int64_t xcd_block() {
    const int64_t g = gridDim.x, b = blockIdx.x;
    return (g & 7) ? b : (b & 7) * (g >> 3) + (b >> 3);
}

// Grid for xcd_block() kernels: a multiple of 8, ~4 block-strides of work per
// block, at most 2048 blocks.
inline unsigned xcd_grid(int64_t n, int block) {
    int64_t g = ceil_div(n, 4 * static_cast<int64_t>(block));
    g = ((g + 7) / 8) * 8;
    if (g < 8) g = 8;
    if (g > 2048) g = 2048;
    return static_cast<unsigned>(g);
}

}  // namespace o3dml
