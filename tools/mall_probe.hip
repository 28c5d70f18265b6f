// Does a write-then-gather round trip stay in the Infinity Cache when the
// buffer is ~100 MB and reused?  (probe for a source-blocked backward; not product)
//   A: one 7.3 GB buffer: per-wave region stores, then random 64-B row gathers
//   B: NB blocks of 7.3GB/NB over ONE reused buffer, write + gather per block
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

// 4 B/lane stores, each wave a contiguous region
__global__ void wr(float *p, size_t region_floats, int n_waves, float v) {
    const int w = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (w >= n_waves) return;
    float *r = p + (size_t)w * region_floats;
    for (size_t i = lane; i < region_floats; i += 64) r[i] = v + (float)i;
}
// random 64-B rows, 4 lanes per row, 16 rows per instruction
__global__ void gather64(const float4 *p, size_t n_rows, size_t n_gathers, uint32_t salt,
                         float *out) {
    const int lane = threadIdx.x % 64, g = lane / 4, q = lane % 4;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const size_t nw = (size_t)gridDim.x * blockDim.x / 64;
    float4 a = make_float4(0, 0, 0, 0);
    for (size_t base = wave * 64; base < n_gathers; base += nw * 64) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            size_t row = hash32((uint32_t)(base + u * 16 + g) ^ salt) % n_rows;
            v[u] = p[row * 4 + q];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) { a.x += v[u].x; a.y += v[u].y; }
    }
    if (a.x == 12345.f) out[0] = a.y;
}

int main() {
    const size_t total = 7300ull << 20;  // ~ Reddit k=16 contributions
    float *big, *out;
    CK(hipMalloc(&big, total));
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](size_t blk_bytes, int nb, const char *name) {
        const size_t region = 32768;  // floats per wave
        const int nw = (int)(blk_bytes / 4 / region);
        const size_t rows = blk_bytes / 64;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int i = 0; i < nb; ++i) {
                wr<<<(nw + 3) / 4, 256>>>(big, region, nw, (float)i);
                gather64<<<4096, 256>>>((const float4 *)big, rows, rows, i * 7919u, out);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep == 1)
                printf("%-34s nb=%4d block=%7.1f MB  %8.3f ms  (%.0f GB/s write+read)\n", name, nb,
                       blk_bytes / 1048576.0, ms, 2.0 * blk_bytes * nb / ms / 1e6);
        }
    };
    run(total, 1, "A one 7.3 GB buffer");
    run(total / 32, 32, "B 32 blocks reuse");
    run(total / 64, 64, "B 64 blocks reuse");
    run(total / 128, 128, "B 128 blocks reuse");
    run(total / 256, 256, "B 256 blocks reuse");
    return 0;
}
