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

__global__ void zero_words_kernel(uint32_t *__restrict__ p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0u;
}

int zero_words(void *p, int64_t n, hipStream_t s) {
    if (n <= 0) return MAXK_OK;
    const int64_t blocks = ceil_div(n, kBlock);
    hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)),
                       dim3(kBlock), 0, s, reinterpret_cast<uint32_t *>(p), n);
    MAXK_LAUNCHED("zero_words_kernel");
    return MAXK_OK;
}

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
