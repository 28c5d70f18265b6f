// Probe, not product.  Does the Infinity Cache (MALL) absorb a write -> read round trip
// through a REUSED buffer?  The backward writes 7.3 GB of contribution rows T and reads them
// back once; if T were produced and consumed in chunks through one buffer of S bytes, would
// the chunk stay on die between its write and its read (and never reach HBM)?
//   for S in 16 MB .. 1 GB, total 7 GB moved:  n = 7 GB / S rounds of
//     W: stream-write the S-byte buffer (16 B per lane, plain or nt stores)
//     R: stream-read it back (sequential) or gather its 64-B rows in random order
//   reported: ms for all rounds, and the equivalent GB/s of write+read traffic.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mall_reuse_probe.hip -o tools/mall_reuse_probe
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <bool NT>
__global__ void wr(u32x4 *p, size_t n4, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x) {
        u32x4 x = {v, (uint32_t)i, 2u, 3u};
        if (NT)
            __builtin_nontemporal_store(x, p + i);
        else
            p[i] = x;
    }
}
__global__ void rd(const u32x4 *p, size_t n4, uint32_t *out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
         i += (size_t)gridDim.x * blockDim.x)
        a += p[i].x ^ p[i].w;
    if (a == 0x12345u) out[0] = a;
}
// random 64-B rows, 4 lanes per row
__global__ void gather(const u32x4 *p, uint32_t rows, uint32_t salt, uint32_t *out) {
    const int q = threadIdx.x % 4;
    uint32_t a = 0;
    const size_t n = (size_t)rows * 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t r = hash32((uint32_t)(i / 4) ^ salt) % rows;
        a += p[(size_t)r * 4 + q].x;
    }
    if (a == 0x12345u) out[0] = a;
}

int main() {
    const size_t total = 7ull << 30;
    u32x4 *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, 1ull << 30));
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t sizes_mb[] = {16, 32, 64, 128, 192, 256, 512, 1024};
    printf("%8s %6s %12s %12s %12s %12s\n", "S_MB", "rounds", "wr+rd ms", "wr_nt+rd ms",
           "wr+gath ms", "wr_nt+gath");
    for (size_t mb : sizes_mb) {
        const size_t S = mb << 20, n4 = S / 16;
        const int rounds = (int)(total / S);
        float ms[4];
        for (int v = 0; v < 4; ++v) {
            auto body = [&](int r) {
                if (v == 0 || v == 2)
                    wr<false><<<4096, 256>>>(buf, n4, (uint32_t)r);
                else
                    wr<true><<<4096, 256>>>(buf, n4, (uint32_t)r);
                if (v < 2)
                    rd<<<4096, 256>>>(buf, n4, out);
                else
                    gather<<<4096, 256>>>(buf, (uint32_t)(S / 64), (uint32_t)r, out);
            };
            body(0);
            CK(hipEventRecord(a));
            for (int r = 0; r < rounds; ++r) body(r);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms[v], a, b));
        }
        printf("%8zu %6d %12.3f %12.3f %12.3f %12.3f\n", mb, rounds, ms[0], ms[1], ms[2], ms[3]);
    }
    return 0;
}
