// Probe, not product.  Rate of scattered small-row stores on MI355X, for a two-phase
// backward whose phase 1 writes each edge's k-float contribution row at its CSC position
// (so phase 2 reads them in order) instead of in CSR order: rows of R = 16..128 bytes
// written (a) in order, (b) each at a scattered row (an odd-multiplier bijection of the row
// index), with default / nt store policy; and the read side, rows read in order vs gathered
// at scattered rows.  N rows of R bytes per pass (~4-16 GB).
// Build: hipcc --offload-arch=gfx950 -O3 tools/scatter_store_probe.hip -o tools/scatter_store_probe
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

// LPR = lanes per row (R / 16); row i -> destination row (SCAT ? i * A mod N : i)
template <int LPR, bool SCAT, bool NT>
__global__ __launch_bounds__(256) void store_rows(u32x4 *p, uint32_t n_rows_log2, uint32_t v) {
    const uint64_t n = 1ull << n_rows_log2;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x / LPR;
    const int sub = threadIdx.x % LPR;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR; i < n; i += stride) {
        const uint64_t d = SCAT ? (i * 0x9E3779B1ull) & (n - 1) : i;
        u32x4 x = {v, (uint32_t)i, (uint32_t)sub, 7u};
        if (NT)
            __builtin_nontemporal_store(x, p + d * LPR + sub);
        else
            p[d * LPR + sub] = x;
    }
}

template <int LPR, bool SCAT>
__global__ __launch_bounds__(256) void load_rows(const u32x4 *p, uint32_t n_rows_log2, uint32_t *sink) {
    const uint64_t n = 1ull << n_rows_log2;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x / LPR;
    const int sub = threadIdx.x % LPR;
    uint32_t a = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR; i < n; i += stride * 4) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t j = i + u * stride;
            const uint64_t d = SCAT ? (j * 0x9E3779B1ull) & (n - 1) : j;
            x[u] = j < n ? p[d * LPR + sub] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) a += x[u].x ^ x[u].w;
    }
    if (a == 0x12345678u) sink[0] = a;
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int LPR>
void run(void *buf, uint32_t *sink, uint64_t bytes) {
    const int R = 16 * LPR;
    uint32_t lg = 0;
    while ((1ull << (lg + 1)) * R <= bytes) ++lg;
    const double gb = (double)(1ull << lg) * R / 1e9;
    const dim3 grid(256 * 16), blk(256);
    u32x4 *p = reinterpret_cast<u32x4 *>(buf);
    auto rep = [&](const char *what, float ms) {
        printf("R=%3d B  %-28s %8.3f ms  %6.2f TB/s  (%.2f GB)\n", R, what, ms, gb / ms, gb);
    };
    rep("store in order (plain)", time_ms([&] { store_rows<LPR, false, false><<<grid, blk>>>(p, lg, 1); }, 5));
    rep("store in order (nt)", time_ms([&] { store_rows<LPR, false, true><<<grid, blk>>>(p, lg, 1); }, 5));
    rep("store scattered (plain)", time_ms([&] { store_rows<LPR, true, false><<<grid, blk>>>(p, lg, 1); }, 5));
    rep("store scattered (nt)", time_ms([&] { store_rows<LPR, true, true><<<grid, blk>>>(p, lg, 1); }, 5));
    rep("load in order", time_ms([&] { load_rows<LPR, false><<<grid, blk>>>(p, lg, sink); }, 5));
    rep("load scattered", time_ms([&] { load_rows<LPR, true><<<grid, blk>>>(p, lg, sink); }, 5));
}

int main() {
    const uint64_t bytes = 4ull << 30;  // 4 GiB per pass (products k=8 T is 3.96 GB)
    void *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, bytes));
    run<1>(buf, sink, bytes);
    run<2>(buf, sink, bytes);
    run<4>(buf, sink, bytes);
    run<8>(buf, sink, bytes);
    CK(hipFree(buf));
    return 0;
}
