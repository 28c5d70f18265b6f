// Random-row gather rate vs buffer size (does an Infinity-Cache-resident buffer gather
// faster than HBM?), and whether freshly WRITTEN lines are resident.  Probe, not product.
//   for S in 4 MB .. 7 GB:  gather NG random 64-B (or 128-B) rows of an S-byte buffer
//   (a) after a streaming read of the buffer, (b) right after a streaming write of it.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

__global__ void wr(float4 *p, size_t n4, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(v, 1.f, 2.f, (float)i);
}
__global__ void rd(const float4 *p, size_t n4, float *out) {
    float a = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x)
        a += p[i].x;
    if (a == 1234.5f) out[0] = a;
}
// S-byte random rows, LR = S/16 lanes per row, U rows per lane-group in flight
template <int S, int U>
__global__ void gather(const float4 *p, uint32_t n_rows, size_t n_gathers, uint32_t salt,
                       float *out) {
    constexpr int LR = S / 16, RI = 64 / LR;
    const int lane = threadIdx.x % 64, g = lane / LR, q = lane % LR;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const size_t nw = (size_t)gridDim.x * blockDim.x / 64;
    float a = 0.f;
    for (size_t base = wave * RI * U; base < n_gathers; base += nw * RI * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t row = hash32((uint32_t)(base + u * RI + g) ^ salt) % n_rows;
            v[u] = p[(size_t)row * LR + q];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) a += v[u].x + v[u].w;
    }
    if (a == 1234.5f) out[0] = a;
}

int main() {
    const size_t max_bytes = 7ull << 30;
    float4 *buf;
    float *out;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, max_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t NG = 114600000;  // Reddit E
    const size_t sizes_mb[] = {4, 16, 32, 64, 128, 192, 256, 512, 1024, 7168};
    auto time_gather = [&](auto kern, size_t bytes, int S, uint32_t salt) {
        const uint32_t rows = (uint32_t)(bytes / S);
        CK(hipEventRecord(a));
        kern<<<8192, 256>>>(buf, rows, NG, salt, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    auto time_k = [&](auto f) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    printf("%9s %10s %10s %10s %10s %10s\n", "buf_MB", "g64_ms", "g64_GB/s", "g128_ms",
           "wr+g64_ms", "wr_ms");
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20;
        const size_t n4 = bytes / 16;
        // warm: stream-read the buffer, then gather twice (second is timed)
        rd<<<4096, 256>>>(buf, n4, out);
        time_gather(gather<64, 8>, bytes, 64, 1u);
        const float g64 = time_gather(gather<64, 8>, bytes, 64, 2u);
        rd<<<4096, 256>>>(buf, n4, out);
        time_gather(gather<128, 8>, bytes, 128, 3u);
        const float g128 = time_gather(gather<128, 8>, bytes, 128, 4u);
        // write the buffer, then gather: are freshly stored lines served on-die?
        const float w = time_k([&] { wr<<<4096, 256>>>(buf, n4, 1.f); });
        const float wg = time_gather(gather<64, 8>, bytes, 64, 5u);
        printf("%9zu %10.3f %10.0f %10.3f %10.3f %10.3f\n", mb, g64, NG * 64.0 / g64 / 1e6, g128,
               wg, w);
    }
    return 0;
}
