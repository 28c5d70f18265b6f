// Calibrates rocprofv3's FETCH_SIZE on gfx950 for sub-line gathers: the
// guide documents FETCH_SIZE = 1/2 of the bytes only for wide coalesced streaming reads
// (128-B fabric requests tallied at 64 B).  The forward's record gathers are 80 B (k = 16) or
// 160 B (k = 32) at random offsets, so the doubling tools/pmc_summary.py applies there is
// unvalidated.  This probe gathers known records -- R bytes at stride R, R/4 lanes x 4 B each --
// from a random record of a table, and a 16-B-per-lane streaming read of the table (the
// documented case), at two table sizes (Infinity-Cache resident and far past it).  Read with
// tools/fetch_probe_summary.py against rocprofv3 --pmc passes of FETCH_SIZE and of
// TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_32B_sum / TCC_EA0_RDREQ_128B_sum (the request-size split
// FETCH_SIZE is derived from).  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe tools/fetch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
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
    x ^= x >> 16;
    x *= 0x7feb352d;
    x ^= x >> 15;
    x *= 0x846ca68b;
    x ^= x >> 16;
    return x;
}

// R-byte records at stride R (record i at byte i * R, 16-B aligned for R % 16 == 0): a group of
// G lanes (G = pow2 >= R / 4) loads one record, lane q < R / 4 its dword q; 64 / G records per
// wave instruction, 4 instructions in flight.  TBL only tells the table sizes apart in the
// profiler's kernel names.
template <int R, int TBL>
__global__ __launch_bounds__(256) void gather_rec(const uint8_t *__restrict__ table, uint32_t n_rec,
                                                  uint32_t n_gathers, uint32_t salt,
                                                  float *__restrict__ out) {
    constexpr int W = R / 4;
    constexpr int G = W <= 16 ? 16 : (W <= 32 ? 32 : 64);
    constexpr int PER = 64 / G;
    const int lane = threadIdx.x % 64, g = lane / G, q = lane % G;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint32_t nw = gridDim.x * blockDim.x / 64;
    float a = 0.f;
    for (uint32_t base = wave * PER * 4; base < n_gathers; base += nw * PER * 4) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t rec = hash32((base + u * PER + g) ^ salt) % n_rec;
            v[u] = q < W ? *reinterpret_cast<const float *>(table + (uint64_t)rec * R + q * 4) : 0.f;
        }
        a += (v[0] + v[1]) + (v[2] + v[3]);
    }
    if (a == 12345.f) out[0] = a;
}

// 16 B per lane, the whole table once (the guide's documented FETCH_SIZE = bytes / 2 case)
template <int TBL>
__global__ __launch_bounds__(256) void stream_read(const float4 *__restrict__ p, uint64_t n16,
                                                   float *__restrict__ out) {
    float a = 0.f;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        a += (v.x + v.y) + (v.z + v.w);
    }
    if (a == 12345.f) out[0] = a;
}

template <int R, int TBL>
float run_gather(const uint8_t *t, uint64_t bytes, uint32_t n, float *out, hipEvent_t e0,
                 hipEvent_t e1) {
    const uint32_t n_rec = (uint32_t)(bytes / R);
    const dim3 grid(256 * 8), block(256);
    hipLaunchKernelGGL((gather_rec<R, TBL>), grid, block, 0, 0, t, n_rec, n, 1u, out);  // warm
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((gather_rec<R, TBL>), grid, block, 0, 0, t, n_rec, n, 7u, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("gather_rec<%d,%d> table %.0f MiB records %u gathers %u bytes_requested %llu "
           "ms %.4f GBs %.1f\n",
           R, TBL, bytes / 1048576.0, n_rec, n, (unsigned long long)n * R, ms,
           (double)n * R / ms / 1e6);
    return ms;
}

template <int TBL>
void run_table(const uint8_t *t, uint64_t bytes, uint32_t n, float *out, hipEvent_t e0,
               hipEvent_t e1) {
    hipLaunchKernelGGL(stream_read<TBL>, dim3(256 * 8), dim3(256), 0, 0,
                       reinterpret_cast<const float4 *>(t), bytes / 16, out);  // warm
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(stream_read<TBL>, dim3(256 * 8), dim3(256), 0, 0,
                       reinterpret_cast<const float4 *>(t), bytes / 16, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream_read<%d> table %.0f MiB bytes_requested %llu ms %.4f GBs %.1f\n", TBL,
           bytes / 1048576.0, (unsigned long long)bytes, ms, bytes / ms / 1e6);
    run_gather<64, TBL>(t, bytes, n, out, e0, e1);
    run_gather<80, TBL>(t, bytes, n, out, e0, e1);
    run_gather<128, TBL>(t, bytes, n, out, e0, e1);
    run_gather<160, TBL>(t, bytes, n, out, e0, e1);
    run_gather<256, TBL>(t, bytes, n, out, e0, e1);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (8u << 20);  // gathers per launch
    const uint64_t small = 24ull << 20, big = 2048ull << 20;  // IC-resident / past the IC
    uint8_t *t;
    float *out;
    CK(hipMalloc(&t, big));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(t, 0x3c, big));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    run_table<0>(t, small, n, out, e0, e1);
    run_table<1>(t, big, n, out, e0, e1);
    CK(hipDeviceSynchronize());
    CK(hipFree(t));
    CK(hipFree(out));
    return 0;
}
