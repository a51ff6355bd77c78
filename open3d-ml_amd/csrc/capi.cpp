// capi.cpp — library-wide C-ABI entry points: error reporting and version.
#include <cstdarg>
#include <cstdio>

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
