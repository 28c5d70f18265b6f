// Probe, not product.  Streaming-write rate of HBM on MI355X for the backward's T stream
// (7.3 GB at Reddit k=16): 16-B stores per lane with default / nt / sc1 policy, grid sizes,
// and a mixed stream (1 B read per 2 B written, like phase 1).
// Build: hipcc --offload-arch=gfx950 -O3 tools/write_probe.hip -o tools/write_probe
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

template <int AUX, int UNR>
__global__ void wr(float *p, size_t n4, uint32_t v) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
    (void)rs;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 *q = reinterpret_cast<u32x4 *>(p);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride * UNR) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const size_t j = i + u * stride;
            if (j < n4) {
                u32x4 x = {v, (uint32_t)j, 1u, 2u};
                if (AUX == 2)
                    __builtin_nontemporal_store(x, q + j);
                else
                    q[j] = x;
            }
        }
    }
}
// each wave writes its own contiguous chunk of CH bytes, 1 KB per store instruction
// (phase 1's pattern: one work item = one contiguous run of contribution rows)
__global__ void wr_chunk(float *p, size_t n4, size_t ch4, uint32_t v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 *q = reinterpret_cast<u32x4 *>(p);
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x % 64;
    const size_t b = wave * ch4, e = b + ch4 < n4 ? b + ch4 : n4;
    for (size_t i = b + lane; i < e; i += 64) {
        u32x4 x = {v, (uint32_t)i, 1u, 2u};
        __builtin_nontemporal_store(x, q + i);
    }
}
// read 1 float4 per 2 float4 written (phase 1: ~3.4 GB read for 7.4 GB written)
__global__ void mix(const float4 *src, float *p, size_t n4, uint32_t v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 *q = reinterpret_cast<u32x4 *>(p);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
        if ((i & 1) == 0) a += __float_as_uint(src[i >> 1].x);
        u32x4 x = {v ^ a, (uint32_t)i, 1u, 2u};
        __builtin_nontemporal_store(x, q + i);
    }
}

int main() {
    const size_t bytes = 7ull << 30, n4 = bytes / 16;
    float *buf;
    float4 *src;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&src, bytes / 2));
    CK(hipMemset(src, 0, bytes / 2));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto t = [&](const char *name, auto f) {
        f();
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; ++r) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 3;
        printf("%-32s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    for (int grid : {2048, 8192, 32768}) {
        char n[64];
        snprintf(n, sizeof n, "plain   grid %5d", grid);
        t(n, [&] { wr<0, 1><<<grid, 256>>>(buf, n4, 1u); });
        snprintf(n, sizeof n, "nt      grid %5d", grid);
        t(n, [&] { wr<2, 1><<<grid, 256>>>(buf, n4, 1u); });
        snprintf(n, sizeof n, "nt x4   grid %5d", grid);
        t(n, [&] { wr<2, 4><<<grid, 256>>>(buf, n4, 1u); });
    }
    for (size_t ch : {4096, 16384, 57344, 262144}) {
        char n[64];
        const size_t ch4 = ch / 16, waves = (n4 + ch4 - 1) / ch4;
        snprintf(n, sizeof n, "chunk/wave %6zu B", ch);
        t(n, [&] { wr_chunk<<<(unsigned)((waves + 3) / 4), 256>>>(buf, n4, ch4, 1u); });
    }
    t("mixed 1 read : 2 write (nt)", [&] { mix<<<8192, 256>>>(src, buf, n4, 1u); });
    return 0;
}
