// capi.cpp — library-wide C-ABI entry points: error reporting and version.
#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"

namespace o3dml {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const char* last_error() { return g_err; }

namespace {
struct TimingState {
    std::mutex mu;
    bool on = false;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::map<std::string, std::pair<double, int64_t>> totals;
};
TimingState& timing() {
    static TimingState t;
    return t;
}
void resolve_locked(TimingState& t) {
    for (auto& e : t.pending) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second.second) == hipSuccess &&
            hipEventElapsedTime(&ms, e.second.first, e.second.second) == hipSuccess) {
            auto& tot = t.totals[e.first];
            tot.first += ms;
            tot.second += 1;
        }
        (void)hipEventDestroy(e.second.first);
        (void)hipEventDestroy(e.second.second);
    }
    t.pending.clear();
}
}  // namespace

bool timing_enabled() { return timing().on; }

void timing_record(const char* name, hipEvent_t a, hipEvent_t b) {
    TimingState& t = timing();
    std::lock_guard<std::mutex> g(t.mu);
    t.pending.push_back({name, {a, b}});
}

}  // namespace o3dml

O3DML_API const char* o3dml_last_error() { return o3dml::last_error(); }

O3DML_API int o3dml_version() { return 1; }

// Device properties the host layer needs (CU count for grid sizing).
O3DML_API int o3dml_device_info(int device, int* cu_count, int* arch_major, int* arch_minor) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) {
        o3dml::set_error("hipGetDeviceProperties(%d) failed", device);
        return 1;
    }
    if (cu_count) *cu_count = p.multiProcessorCount;
    if (arch_major) *arch_major = p.major;
    if (arch_minor) *arch_minor = p.minor;
    return 0;
}

O3DML_API void o3dml_timing_enable(int on) {
    auto& t = o3dml::timing();
    std::lock_guard<std::mutex> g(t.mu);
    t.on = on != 0;
}

O3DML_API void o3dml_timing_reset() {
    auto& t = o3dml::timing();
    std::lock_guard<std::mutex> g(t.mu);
    o3dml::resolve_locked(t);
    t.totals.clear();
}

// Total milliseconds and launch count recorded under `name` since the last reset.
O3DML_API int o3dml_timing_get(const char* name, double* total_ms, int64_t* count) {
    auto& t = o3dml::timing();
    std::lock_guard<std::mutex> g(t.mu);
    o3dml::resolve_locked(t);
    auto it = t.totals.find(name);
    *total_ms = it == t.totals.end() ? 0.0 : it->second.first;
    *count = it == t.totals.end() ? 0 : it->second.second;
    return 0;
}
