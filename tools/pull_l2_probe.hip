// Probe, not product.  Could the backward skip the contribution rows T?  A "tiled pull"
// would process the adjacency in (row block, destination bucket) tiles: per edge, gather the
// k values G'[r, sel[c, l]] straight from an L2-resident row block of G' and add them into an
// fp64 LDS accumulator of the bucket (as bucket_sum_kernel does with T rows).  This probe
// measures that inner loop alone at Reddit scale: 114.6M edges, k = 16, rows in CSR order
// (runs of ~2 edges per row and bucket), each XCD's workgroups sharing one G' row block.
//   mode 0: the full loop (selector load, 4 gathers per lane, 4 ds_add_f64)
//   mode 1: gathers only (no LDS adds)
//   mode 2: LDS adds only (G' value replaced by the selector byte)
// Build: hipcc --offload-arch=gfx950 -O3 tools/pull_l2_probe.hip -o tools/pull_l2_probe
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

constexpr int K = 16, NB = 1024, ACC = NB * (K + 1);

template <int MODE>
__global__ __launch_bounds__(1024) void pull(const float *__restrict__ G, int block_rows,
                                             const uint32_t *__restrict__ sel, int64_t per_wg,
                                             float run, float *out) {
    __shared__ double acc[ACC];
    for (int i = threadIdx.x; i < ACC; i += 1024) acc[i] = 0.0;
    __syncthreads();
    const int xcd = blockIdx.x % 8;
    const float *Gb = G + (size_t)xcd * block_rows * 256;
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const int grp = lane / 4, q = lane % 4;
    float dummy = 0.f;
    // entries [0, per_wg): wave w takes steps w, w+16, ... of 16 entries each
    for (int64_t base = (int64_t)wave * 16; base < per_wg; base += 16 * 16) {
        const int64_t e = base + grp;
        const uint32_t ge = (uint32_t)(e + blockIdx.x * per_wg);
        const int r = (int)((float)e / run) % block_rows;  // CSR order: runs of ~`run` entries
        const int d = (int)(hash32(ge) % NB);
        const uint32_t s = sel[d * 4 + q];
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = (s >> (8 * i)) & 255;
            v[i] = MODE == 2 ? (float)col : Gb[(size_t)r * 256 + col];
        }
        if (MODE == 1) {
            dummy += v[0] + v[1] + v[2] + v[3];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&acc[d * (K + 1) + q * 4 + i], (double)v[i]);
        }
    }
    __syncthreads();
    if (MODE == 1) {
        if (dummy == 1234.5f) out[0] = dummy;
        return;
    }
    for (int i = threadIdx.x; i < NB * K; i += 1024)
        out[(size_t)blockIdx.x * NB * K + i] = (float)acc[i + i / K];
}

int main() {
    const int64_t E = 114615891;
    const int wgs = 256;
    const int64_t per_wg = (E + wgs - 1) / wgs;
    float *G, *out;
    uint32_t *sel;
    const int block_rows_list[] = {1024, 2048, 4096, 16384};
    CK(hipMalloc(&G, (size_t)8 * 16384 * 256 * 4));
    CK(hipMalloc(&out, (size_t)wgs * NB * K * 4));
    CK(hipMalloc(&sel, NB * 16));
    CK(hipMemset(G, 0, (size_t)8 * 16384 * 256 * 4));
    {
        uint32_t h[NB * 4];
        for (int i = 0; i < NB * 4; ++i) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) x |= (uint32_t)((i * 37 + b * 61 + (i >> 2) * 11) & 255) << (8 * b);
            h[i] = x;
        }
        CK(hipMemcpy(sel, h, sizeof h, hipMemcpyHostToDevice));
    }
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
        printf("%-44s %8.3f ms\n", name, ms / 3);
    };
    for (int br : block_rows_list) {
        for (float run : {1.0f, 2.15f, 8.0f}) {
            char n[96];
            snprintf(n, sizeof n, "full   rows/block %5d run %.2f", br, run);
            t(n, [&] { pull<0><<<wgs, 1024>>>(G, br, sel, per_wg, run, out); });
            snprintf(n, sizeof n, "gather rows/block %5d run %.2f", br, run);
            t(n, [&] { pull<1><<<wgs, 1024>>>(G, br, sel, per_wg, run, out); });
        }
    }
    t("lds-add only", [&] { pull<2><<<wgs, 1024>>>(G, 1024, sel, per_wg, 2.15f, out); });
    return 0;
}
