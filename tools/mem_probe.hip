// HBM access-shape probe for the two-phase backward (not product code).
// Measures on a buffer far larger than the Infinity Cache:
//   W1 streaming stores, grid-stride, 16 B/lane (1 KiB per wave-instruction)
//   W2 per-wave contiguous regions (128 KiB each), 4 B/lane stores (256 B/instr)
//   W3 = W2 with 16 B/lane stores
//   R1 streaming reads 16 B/lane
//   Rg random row gathers of S bytes (S = 64, 128, 256), 16 B/lane
// Build: hipcc --offload-arch=gfx950 -O3 tools/mem_probe.hip -o tools/mem_probe
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

__global__ void w1(float4 *p, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
// each wave owns region [w*R, (w+1)*R) floats, writes it front to back
template <int VEC>
__global__ void w2(float *p, size_t region_floats, int n_waves) {
    const int w = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (w >= n_waves) return;
    float *r = p + (size_t)w * region_floats;
    if (VEC) {
        for (size_t i = lane * 4; i < region_floats; i += 256)
            *reinterpret_cast<float4 *>(r + i) = make_float4(1.f, 2.f, 3.f, (float)i);
    } else {
        for (size_t i = lane; i < region_floats; i += 64) r[i] = (float)i;
    }
}
__global__ void r1(const float4 *p, size_t n4, float *out) {
    float4 a = make_float4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x) {
        float4 v = p[i];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (a.x == 12345.f) out[0] = a.y + a.z + a.w;
}
// random rows of S bytes: LR = S/16 lanes per row, 64/LR rows per instruction
template <int S, int U>
__global__ void rg(const float4 *p, size_t n_rows, size_t n_gathers, float *out) {
    constexpr int LR = S / 16, RI = 64 / LR;
    const int lane = threadIdx.x % 64, g = lane / LR, q = lane % LR;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const size_t nw = (size_t)gridDim.x * blockDim.x / 64;
    float4 a = make_float4(0, 0, 0, 0);
    for (size_t base = wave * RI * U; base < n_gathers; base += nw * RI * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t row = hash32((uint32_t)(base + u * RI + g)) % n_rows;
            v[u] = p[row * LR + q];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { a.x += v[u].x; a.y += v[u].y; }
    }
    if (a.x == 12345.f) out[0] = a.y;
}

template <typename F>
float timeit(F f, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t bytes = 7ull << 30;  // 7 GiB >> 256 MiB Infinity Cache
    float *p, *out;
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&out, 64));
    const size_t n4 = bytes / 16;
    auto gbs = [&](double b, float ms) { return b / ms / 1e6; };
    float ms;
    ms = timeit([&] { w1<<<8192, 256>>>((float4 *)p, n4); });
    printf("W1 stream store 16B/lane            %7.3f ms %7.0f GB/s\n", ms, gbs(bytes, ms));
    const size_t region = 32768;  // floats = 128 KiB per wave
    const int nw = (int)(bytes / 4 / region);
    ms = timeit([&] { w2<0><<<(nw + 3) / 4, 256>>>(p, region, nw); });
    printf("W2 per-wave regions, 4B/lane        %7.3f ms %7.0f GB/s\n", ms, gbs(bytes, ms));
    ms = timeit([&] { w2<1><<<(nw + 3) / 4, 256>>>(p, region, nw); });
    printf("W3 per-wave regions, 16B/lane       %7.3f ms %7.0f GB/s\n", ms, gbs(bytes, ms));
    ms = timeit([&] { r1<<<8192, 256>>>((const float4 *)p, n4, out); });
    printf("R1 stream read 16B/lane             %7.3f ms %7.0f GB/s\n", ms, gbs(bytes, ms));
    const size_t ng = 114000000;  // Reddit E gathers
    ms = timeit([&] { rg<64, 4><<<8192, 256>>>((const float4 *)p, bytes / 64, ng, out); });
    printf("Rg 64-B random rows  U=4            %7.3f ms %7.0f GB/s\n", ms, gbs(ng * 64.0, ms));
    ms = timeit([&] { rg<64, 8><<<8192, 256>>>((const float4 *)p, bytes / 64, ng, out); });
    printf("Rg 64-B random rows  U=8            %7.3f ms %7.0f GB/s\n", ms, gbs(ng * 64.0, ms));
    ms = timeit([&] { rg<128, 4><<<8192, 256>>>((const float4 *)p, bytes / 128, ng / 2, out); });
    printf("Rg 128-B random rows U=4            %7.3f ms %7.0f GB/s\n", ms, gbs(ng * 64.0, ms));
    ms = timeit([&] { rg<256, 4><<<8192, 256>>>((const float4 *)p, bytes / 256, ng / 4, out); });
    printf("Rg 256-B random rows U=4            %7.3f ms %7.0f GB/s\n", ms, gbs(ng * 64.0, ms));
    ms = timeit([&] { rg<1024, 4><<<8192, 256>>>((const float4 *)p, bytes / 1024, ng / 16, out); });
    printf("Rg 1KiB random rows  U=4            %7.3f ms %7.0f GB/s\n", ms, gbs(ng * 64.0, ms));
    return 0;
}
