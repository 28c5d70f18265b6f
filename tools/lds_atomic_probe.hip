// Probe, not product.  LDS accumulate throughput on gfx950, all CUs busy (1024 workgroups
// x 256 threads, 4096 ops per lane): cycles per wave instruction for
//   ds_add_f32 / ds_add_u32 / ds_add_u64 / ds_add_f64 and plain ds_write_b32,
// with (a) conflict-free addresses (lane-consecutive words) and (b) random words of a
// 16K-word table.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_probe.hip -o tools/lds_atomic_probe
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

constexpr int N_OPS = 4096, WORDS = 16384;

template <typename T, int OP, bool RAND>
__global__ __launch_bounds__(256) void k(T *out, unsigned salt) {
    __shared__ T tab[WORDS];
    for (int i = threadIdx.x; i < WORDS; i += 256) tab[i] = (T)0;
    __syncthreads();
    unsigned x = threadIdx.x * 2654435761u ^ salt ^ blockIdx.x;
    const int base = (threadIdx.x / 64) * 4096 + (threadIdx.x % 64);
    T v = (T)1;
#pragma unroll 8
    for (int i = 0; i < N_OPS; ++i) {
        int a;
        if (RAND) {
            x = x * 1664525u + 1013904223u;
            a = (x >> 8) & (WORDS - 1);
        } else {
            a = base + ((i * 64) & 4095);
        }
        if (OP == 0)
            atomicAdd(&tab[a], v);
        else
            tab[a] = v + (T)i;
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = tab[salt & (WORDS - 1)];
}

int main() {
    double *out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const int grid = 1024;
    auto run = [&](const char *name, auto f) {
        f();
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        // wave instructions per CU: grid * 4 waves * N_OPS / 256 CUs
        const double wi = (double)grid * 4 * N_OPS / 256;
        printf("%-28s %8.3f ms  %6.1f cycles/wave-instr per CU (at %.0f MHz)\n", name, ms,
               ms * 1e-3 * clk_khz * 1e3 / wi, clk_khz / 1e3);
    };
    run("ds_add_f32 seq", [&] { k<float, 0, false><<<grid, 256>>>((float *)out, 1); });
    run("ds_add_f32 rand", [&] { k<float, 0, true><<<grid, 256>>>((float *)out, 1); });
    run("ds_add_u32 seq", [&] { k<unsigned, 0, false><<<grid, 256>>>((unsigned *)out, 1); });
    run("ds_add_u32 rand", [&] { k<unsigned, 0, true><<<grid, 256>>>((unsigned *)out, 1); });
    run("ds_add_u64 seq", [&] { k<unsigned long long, 0, false><<<grid, 256>>>((unsigned long long *)out, 1); });
    run("ds_add_u64 rand", [&] { k<unsigned long long, 0, true><<<grid, 256>>>((unsigned long long *)out, 1); });
    run("ds_add_f64 seq", [&] { k<double, 0, false><<<grid, 256>>>(out, 1); });
    run("ds_write_b32 seq", [&] { k<float, 1, false><<<grid, 256>>>((float *)out, 1); });
    run("ds_write_b32 rand", [&] { k<float, 1, true><<<grid, 256>>>((float *)out, 1); });
    CK(hipDeviceSynchronize());
    return 0;
}
