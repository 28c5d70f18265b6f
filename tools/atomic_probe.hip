// Float-atomic rate and exactness by memory scope and footprint (probe, not product).
// Each wave issues, per step, 4 atomic segments of 16 lanes x 4 B (the backward's shape:
// one 64-B contribution row per edge) at hashed rows of a buffer of `rows` x 16 floats.
// Scopes: agent (atomicAdd), workgroup, wavefront.  The buffer is zeroed, every add is
// 1.0f, so the exact total is known: a wrong sum means the scope did not make the add
// atomic across CUs.  Footprints: 1.86 MB (one XCD's slice of Reddit's k=16 gradient) and
// 1 GiB.  Also: 8 XCD-private buffers (workgroup b writes only buffer b % 8).
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int SCOPE, bool XCD_PRIVATE>
__global__ void adds(float *buf, uint32_t rows, int steps) {
    const int lane = threadIdx.x % 64, g = lane / 16, q = lane % 16;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    float *b = buf;
    if (XCD_PRIVATE) b = buf + (size_t)(blockIdx.x % 8) * rows * 16;
    for (int s = 0; s < steps; ++s) {
        const uint32_t row = hash32(wave * 4096u + s * 4u + g) % rows;
        float *p = b + (size_t)row * 16 + q;
        if (SCOPE == 0) atomicAdd(p, 1.0f);
        if (SCOPE == 1) __hip_atomic_fetch_add(p, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (SCOPE == 2) __hip_atomic_fetch_add(p, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
}

template <int SCOPE, bool XCD_PRIVATE>
void run(const char *name, float *buf, uint32_t rows, size_t nbuf_floats) {
    const int blocks = 8192, steps = 64;
    CK(hipMemset(buf, 0, nbuf_floats * 4));
    adds<SCOPE, XCD_PRIVATE><<<blocks, 256>>>(buf, rows, steps);  // warm
    CK(hipDeviceSynchronize());
    CK(hipMemset(buf, 0, nbuf_floats * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    adds<SCOPE, XCD_PRIVATE><<<blocks, 256>>>(buf, rows, steps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<float> h(nbuf_floats);
    CK(hipMemcpy(h.data(), buf, nbuf_floats * 4, hipMemcpyDeviceToHost));
    double tot = 0;
    for (float v : h) tot += v;
    const double expect = (double)blocks * 256 * steps;  // one add per lane per step
    const double reqs = (double)blocks * 4 * 4 * steps;  // 64-B segments
    printf("%-34s rows=%8u %8.3f ms  %7.1f G seg/s  %7.0f GB/s added  sum %s (%.0f / %.0f)\n",
           name, rows, ms, reqs / ms / 1e6, expect * 4 / ms / 1e6,
           tot == expect ? "EXACT" : "WRONG", tot, expect);
}

int main() {
    const size_t big = (1ull << 30) / 4;  // 1 GiB of floats
    float *buf;
    CK(hipMalloc(&buf, big * 4));
    const uint32_t small_rows = 29121;  // 232965/8 vertices x 16 floats = 1.86 MB
    const uint32_t big_rows = (uint32_t)(big / 16);
    run<0, false>("agent scope, 1.86 MB", buf, small_rows, (size_t)small_rows * 16);
    run<1, false>("workgroup scope, 1.86 MB", buf, small_rows, (size_t)small_rows * 16);
    run<2, false>("wavefront scope, 1.86 MB", buf, small_rows, (size_t)small_rows * 16);
    run<0, false>("agent scope, 1 GiB", buf, big_rows, big);
    run<1, false>("workgroup scope, 1 GiB", buf, big_rows, big);
    run<0, true>("agent, 8 XCD-private 1.86 MB", buf, small_rows, (size_t)small_rows * 16 * 8);
    run<1, true>("workgroup, 8 XCD-private 1.86 MB", buf, small_rows, (size_t)small_rows * 16 * 8);
    return 0;
}
