// fill.hip — the library's one way to set device memory to a byte value:
// a kernel, never hipMemsetAsync.  On this runtime (ROCm 7.2 HIP, torch
// 2.10+rocm7.0) a memset node of >= 16 bytes captured into a graph takes
// effect on the graph's FIRST replay only; every later replay leaves the range
// untouched (tools/graph_memset_probe.py, profiles/r05/graph_memset_probe.txt:
// 4-, 8- and 12-byte nodes are re-applied, 16 bytes and up are not).  Every
// launch function of libo3dml_amd is meant to be capturable, so counters,
// histograms and map fills that must start from zero on each replay go
// through fill_async, and device-to-device copies through copy_async (no
// memcpy node either).
#include "common.hpp"

namespace o3dml {

namespace {

__global__ void fill_u32_kernel(uint32_t* __restrict__ p, uint32_t v, int64_t n) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        p[i] = v;
}

__global__ void fill_u128_kernel(uint4* __restrict__ p, uint32_t v, int64_t n) {
    const uint4 w = make_uint4(v, v, v, v);
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        p[i] = w;
}

__global__ void fill_u8_kernel(uint8_t* __restrict__ p, uint8_t v, int64_t n) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        p[i] = v;
}

__global__ void copy_u32_kernel(uint32_t* __restrict__ d, const uint32_t* __restrict__ s, int64_t n) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        d[i] = s[i];
}

__global__ void copy_u8_kernel(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, int64_t n) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        d[i] = s[i];
}

}  // namespace

void copy_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes == 0) return;
    if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes) & 3) == 0) {
        const int64_t n = static_cast<int64_t>(bytes >> 2);
        copy_u32_kernel<<<stream_grid(n, 256), 256, 0, st>>>(static_cast<uint32_t*>(dst),
                                                             static_cast<const uint32_t*>(src), n);
    } else {
        copy_u8_kernel<<<stream_grid(static_cast<int64_t>(bytes), 256), 256, 0, st>>>(
                static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), static_cast<int64_t>(bytes));
    }
    O3DML_LAUNCH_CHECK();
}

void fill_async(void* dst, int value, size_t bytes, hipStream_t st) {
    if (bytes == 0) return;
    const uint8_t b = static_cast<uint8_t>(value);
    const uint32_t w = 0x01010101u * b;
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    if ((a & 15) == 0 && (bytes & 15) == 0 && bytes >= 4096) {
        const int64_t n = static_cast<int64_t>(bytes >> 4);
        fill_u128_kernel<<<stream_grid(n, 256), 256, 0, st>>>(static_cast<uint4*>(dst), w, n);
    } else if ((a & 3) == 0 && (bytes & 3) == 0) {
        const int64_t n = static_cast<int64_t>(bytes >> 2);
        fill_u32_kernel<<<stream_grid(n, 256), 256, 0, st>>>(static_cast<uint32_t*>(dst), w, n);
    } else {
        fill_u8_kernel<<<stream_grid(static_cast<int64_t>(bytes), 256), 256, 0, st>>>(static_cast<uint8_t*>(dst), b,
                                                                                      static_cast<int64_t>(bytes));
    }
    O3DML_LAUNCH_CHECK();
}

}  // namespace o3dml
