// Probe, not product.  Cost of writing a contiguous byte stream on MI355X when each wave
// instruction covers 64 consecutive bytes (the forward's edge-selector emission: a wave step's
// G edges x k bytes): every lane storing a byte, a quarter of the lanes a dword (bytes combined
// in quads by DPP), or four lanes 16 B; against 64 lanes x 16 B (a full-width stream), and each
// with some loads in between (a read stream of the same length), as in the forward.
// Build: hipcc --offload-arch=gfx950 -O3 tools/store_width_probe.hip -o tools/store_width_probe
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

__device__ __forceinline__ uint32_t quad_word(uint32_t b) {
    const uint32_t b1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x55, 0xf, 0xf, false);
    const uint32_t b2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0xaa, 0xf, 0xf, false);
    const uint32_t b3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0xff, 0xf, 0xf, false);
    return (b & 0xffu) | ((b1 & 0xffu) << 8) | ((b2 & 0xffu) << 16) | (b3 << 24);
}

// MODE 0: 64 x b8; 1: quad leaders b32; 2: 4 lanes b128 (row leaders, DPP row combine);
// 3: full-width 64 x 16 B (1 KB per instruction).  LD: one 4-B load per lane per step from a
// read buffer (a dependent value: the stored byte is the loaded word's low byte).
template <int MODE, bool LD>
__global__ __launch_bounds__(256) void stream_kernel(uint8_t *out, const uint32_t *in,
                                                     uint64_t n_steps_total) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint64_t n_waves = (uint64_t)gridDim.x * blockDim.x / 64;
    const uint32_t bytes_per_step = MODE == 3 ? 1024u : 64u;
    for (uint64_t st = wave; st < n_steps_total; st += n_waves) {
        uint32_t v = (uint32_t)(st * 64 + lane);
        if (LD) v = in[(st * 64 + lane) & ((1u << 26) - 1)];
        uint8_t *p = out + st * bytes_per_step;
        if (MODE == 0) {
            p[lane] = (uint8_t)v;
        } else if (MODE == 1) {
            const uint32_t w = quad_word(v & 0xffu);
            if ((lane & 3) == 0) *reinterpret_cast<uint32_t *>(p + lane) = w;
        } else if (MODE == 2) {
            const uint32_t w = quad_word(v & 0xffu);  // valid in lanes 4m
            // row_shl:s (0x100 + s) gives lane i the value of lane i + s in its row: the row
            // leader 16r collects the quad words of lanes 16r + 4, + 8, + 12
            const uint32_t w1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x104, 0xf, 0xf, false);
            const uint32_t w2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x108, 0xf, 0xf, false);
            const uint32_t w3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x10c, 0xf, 0xf, false);
            if ((lane & 15) == 0)
                *reinterpret_cast<u32x4 *>(p + lane) = u32x4{w, w1, w2, w3};
        } else {
            reinterpret_cast<u32x4 *>(p)[lane] = u32x4{v, v, v, v};
        }
    }
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

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t *out;
    uint32_t *in;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&in, 4u << 26));
    CK(hipMemset(in, 1, 4u << 26));
    const dim3 grid(256 * 32), blk(256);
    auto rep = [&](const char *what, float ms) {
        printf("%-36s %8.3f ms  %6.2f TB/s of stream\n", what, ms, bytes / 1e9 / ms);
    };
    const uint64_t s64 = bytes / 64, s1k = bytes / 1024;
    rep("64 lanes x b8 (64 B / instr)", time_ms([&] { stream_kernel<0, false><<<grid, blk>>>(out, in, s64); }, 5));
    rep("16 quad leaders x b32", time_ms([&] { stream_kernel<1, false><<<grid, blk>>>(out, in, s64); }, 5));
    rep("4 row leaders x b128", time_ms([&] { stream_kernel<2, false><<<grid, blk>>>(out, in, s64); }, 5));
    rep("64 lanes x b128 (1 KB / instr)", time_ms([&] { stream_kernel<3, false><<<grid, blk>>>(out, in, s1k); }, 5));
    rep("+load: 64 lanes x b8", time_ms([&] { stream_kernel<0, true><<<grid, blk>>>(out, in, s64); }, 5));
    rep("+load: 16 quad leaders x b32", time_ms([&] { stream_kernel<1, true><<<grid, blk>>>(out, in, s64); }, 5));
    rep("+load: 4 row leaders x b128", time_ms([&] { stream_kernel<2, true><<<grid, blk>>>(out, in, s64); }, 5));
    CK(hipFree(out));
    CK(hipFree(in));
    return 0;
}
