// counters.hpp — tile arrival counters for split-K reductions finished by
// the last-arriving block / wave of each output tile (dense.hip,
// sparse_conv.hip): one slab per device (zeroed once, outside any stream
// capture), one slot of kTileCounterSlot counters per stream that ever asks —
// a stream keeps its slot for the process lifetime, so a captured graph
// replays against the same counters.  Every launch leaves its counters at 0
// (the finishing block resets them) and launches on one stream are ordered,
// so kernels of different kinds can share a stream's slot.  nullptr (the
// caller falls back to a separate reduce launch) when the slab cannot be had:
// first use inside a capture, all slots taken, or more tiles than a slot holds.
#pragma once

#include <mutex>
#include <unordered_map>

#include "common.hpp"

namespace o3dml {

constexpr int64_t kTileCounterSlot = 1 << 16;
constexpr int kTileCounterSlots = 64;

inline uint32_t* tile_counters(hipStream_t st, int64_t need) {
    if (need > kTileCounterSlot) return nullptr;
    struct Slab {
        uint32_t* base = nullptr;
        int used = 0;
        std::unordered_map<hipStream_t, int> slot;
    };
    static std::mutex mu;
    static std::unordered_map<int, Slab> slabs;
    int dev = 0;
    if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    Slab& sl = slabs[dev];
    if (!sl.base) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(dev) != hipSuccess) return nullptr;
        uint32_t* p = nullptr;
        const size_t bytes = sizeof(uint32_t) * kTileCounterSlot * kTileCounterSlots;
        const bool ok = hipMalloc(&p, bytes) == hipSuccess && hipMemset(p, 0, bytes) == hipSuccess;
        (void)hipSetDevice(cur);
        if (!ok) return nullptr;
        sl.base = p;
    }
    auto it = sl.slot.find(st);
    if (it == sl.slot.end()) {
        if (sl.used >= kTileCounterSlots) return nullptr;
        it = sl.slot.emplace(st, sl.used++).first;
    }
    return sl.base + static_cast<int64_t>(it->second) * kTileCounterSlot;
}

}  // namespace o3dml
