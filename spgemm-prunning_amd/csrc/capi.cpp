// Library-level C ABI: version, per-thread error message, device probe.
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace maxk {
namespace {
thread_local char g_err[512] = {0};
}

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

}  // namespace maxk

extern "C" int maxk_version(void) { return 100; }

#ifndef MAXK_SRC_DIGEST
#define MAXK_SRC_DIGEST "unknown"
#endif
extern "C" const char *maxk_source_digest(void) { return MAXK_SRC_DIGEST; }

// EXTRA_HIPFLAGS the library was built with ("" for the product build): every MAXK_* tuning
// or ablation macro set away from its default in common.h shows here.
#ifndef MAXK_BUILD_FLAGS
#define MAXK_BUILD_FLAGS "unknown"
#endif
extern "C" const char *maxk_build_config(void) { return MAXK_BUILD_FLAGS; }

extern "C" const char *maxk_last_error(void) { return maxk::g_err; }

extern "C" int maxk_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}
