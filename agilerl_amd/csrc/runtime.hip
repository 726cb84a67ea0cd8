// Library-level entry points: error reporting, version, device info.
#include <cstring>

#include "agx_common.h"

namespace agx {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace agx

extern "C" const char *agx_last_error(void) { return agx::g_err; }

extern "C" int agx_version(void) { return 100; /* 0.1.0 */ }

extern "C" int agx_device_info(int *out3) {
    if (!out3) {
        agx::set_error("agx_device_info: null output");
        return AGX_EINVAL;
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        agx::set_error("agx_device_info: %s", hipGetErrorString(e));
        return AGX_EHIP;
    }
    out3[0] = prop.multiProcessorCount;
    int arch = 0;  // "gfx950:sramecc+:xnack-" -> 950
    for (const char *c = prop.gcnArchName + 3; *c >= '0' && *c <= '9'; ++c) arch = arch * 10 + (*c - '0');
    out3[1] = arch;
    out3[2] = prop.warpSize;
    return AGX_OK;
}
