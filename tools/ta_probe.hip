// Probe, not product.  What does one vector-memory wave instruction cost the texture path
// (TA/TCP) when its data sits in L2?  The pull backward is bound there (TA busy ~75 %), so
// the cost model decides how its gathers should be shaped.  Every XCD's workgroups read
// their own 2 MiB table (L2-resident, L1-missing), 8 independent loads in flight per wave,
// 32 waves per CU.  Printed: ns per launch, and cycles per wave instruction per CU at
// 2.4 GHz (every CU issuing).
//   gather N : 64 lanes x 4 B, the lanes spread over N random 128-B lines
//   gatherb N: the same through a wave-uniform buffer descriptor (32-bit offsets)
//   x2 N     : 64 lanes x 8 B over N random lines;  x4 N: 64 lanes x 16 B over N lines
//   row1k    : one random 1 KiB row, 16 B per lane (8 lines, coalesced)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ta_probe.hip -o tools/ta_probe
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

constexpr int kTableBytes = 2 << 20;               // per XCD
constexpr int kLines = kTableBytes / 128;          // 16384 lines of 128 B
constexpr int U = 8;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

__constant__ uint16_t c_pat[64];  // MODE 5: lane -> (line id << 8 | dword offset)

// MODE 0: global dword gather; 1: buffer dword gather; 2: dwordx2; 3: dwordx4; 4: row1k;
// 5: dword gather by the lane pattern c_pat (line ids made random per instruction)
template <int MODE>
__global__ __launch_bounds__(256) void probe(const float *__restrict__ T, int iters, int N,
                                             float *out, uint32_t lmask, int shared) {
    const int lane = threadIdx.x % 64;
    const uint32_t wave = (blockIdx.x * 4 + threadIdx.x / 64);
    const float *Tb = T + (shared ? 0 : (size_t)(blockIdx.x % 8) * (lmask + 1) * 32);
    const auto rs = make_rsrc(Tb, (lmask + 1) * 128);
    float acc = 0.f;
    const int grp = MODE >= 6 ? lane / (64 / N) : lane % N;  // lane's line in the instruction
    const int pos = MODE >= 6 ? lane % (64 / N) : lane / N;  // lane's slot within its line
    const uint32_t gmul = (uint32_t)(MODE == 5 ? (c_pat[lane] >> 8) : grp) * 2654435761u;
    const uint32_t poff = c_pat[lane] & 255u;
    for (int it = 0; it < iters; ++it) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t seed = hash32(wave * 7919u + (uint32_t)(it * U + u) * 104729u);
            const uint32_t line = ((seed + gmul) >> 7) & lmask;
            if (MODE == 6) {  // x4, consecutive lanes per line (a record read whole)
                const f32x4 x = *reinterpret_cast<const f32x4 *>(Tb + line * 32 + (pos * 4) % 32);
                v[u] = x.x + x.y + x.z + x.w;
            } else if (MODE == 7) {  // dword, consecutive lanes per line
                v[u] = Tb[line * 32 + pos % 32];
            } else if (MODE == 5) {
                v[u] = Tb[line * 32 + poff];
            } else if (MODE == 0) {
                v[u] = Tb[line * 32 + (pos * 4) % 32];
            } else if (MODE == 1) {
                v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rs, (int)((line * 32 + (pos * 4) % 32) * 4), 0, 0));
            } else if (MODE == 2) {
                const f32x2 x = *reinterpret_cast<const f32x2 *>(Tb + line * 32 + (pos * 2) % 32);
                v[u] = x.x + x.y;
            } else if (MODE == 3) {
                const f32x4 x = *reinterpret_cast<const f32x4 *>(Tb + line * 32 + (pos * 4) % 32);
                v[u] = x.x + x.y + x.z + x.w;
            } else {
                const uint32_t row = seed & (lmask >> 3);
                const f32x4 x = *reinterpret_cast<const f32x4 *>(Tb + row * 256 + lane * 4);
                v[u] = x.x + x.y + x.z + x.w;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main(int argc, char **argv) {
    const uint32_t lmask = (argc > 1 ? (uint32_t)atoi(argv[1]) : (uint32_t)kLines) - 1;  // table lines
    const int shared = argc > 2 ? atoi(argv[2]) : 0;  // 1: one table for all XCDs
    printf("table %u lines of 128 B %s\n", lmask + 1, shared ? "shared by all XCDs" : "per XCD");
    float *T, *out;
    CK(hipMalloc(&T, (size_t)8 * (lmask + 1) * 128));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(T, 0, (size_t)8 * (lmask + 1) * 128));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int wgs = 2048, iters = 256;
    const double instrs = (double)wgs * 4 * iters * U;
    auto t = [&](const char *name, int n, auto f) {
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 5; ++r) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 5;
        const double cyc = ms * 1e-3 * 2.4e9 * 256 / instrs;
        printf("%-8s N=%2d  %8.3f ms  %6.1f cyc/instr/CU  %6.2f cyc/line\n", name, n, ms, cyc,
               cyc / n);
    };
    for (int n : {1, 2, 4, 8, 16, 32, 64}) {
        t("gather", n, [&] { probe<0><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
        t("gatherb", n, [&] { probe<1><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
        t("x2", n, [&] { probe<2><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
        t("x4", n, [&] { probe<3><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
    }
    t("row1k", 8, [&] { probe<4><<<wgs, 256>>>(T, iters, 8, out, lmask, shared); });
    for (int n : {4, 8, 16}) {  // records: 64 / n consecutive lanes per random line
        t("rec_x4", n, [&] { probe<6><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
        t("rec_dw", n, [&] { probe<7><<<wgs, 256>>>(T, iters, n, out, lmask, shared); });
    }
    // quarter patterns (16 lanes each; j = lane % 16, q = lane / 16):
    //  P2: 4 lines x both 64-B halves per quarter   P3: 8 lines, first half only
    //  P4: 2 lines x both halves                    P5: 8 lines x both halves (16 segments)
    //  P6: 1 line, 16 dwords over both halves       P7: 4 lines, first half only
    //  P8: 4 lines, random lane->line, random offsets   P9: 4 lines (j % 4), random offsets
    //  P10: 4 lines, random lane->line, offsets j       P11: 1 line, random offsets
    //  P12: 4 lines, lane->line j / 4, random offsets   P13: 2 lines (j / 8), random offsets
    srand(7);
    for (int pid = 2; pid <= 13; ++pid) {
        uint16_t pat[64];
        for (int l = 0; l < 64; ++l) {
            const int q = l / 16, j = l % 16;
            int line = 0, off = 0;
            if (pid == 2) { line = q * 4 + j % 4; off = (j / 4 % 2) * 16 + j / 8; }
            if (pid == 3) { line = q * 8 + j % 8; off = j / 8; }
            if (pid == 4) { line = q * 2 + j % 2; off = (j / 2 % 2) * 16 + j / 4; }
            if (pid == 5) { line = q * 8 + j % 8; off = (j / 8) * 16; }
            if (pid == 6) { line = q; off = 2 * j; }
            if (pid == 7) { line = q * 4 + j % 4; off = j / 4; }
            const int rl = rand() % 4, ro = rand() % 32;
            if (pid == 8) { line = q * 4 + rl; off = ro; }
            if (pid == 9) { line = q * 4 + j % 4; off = ro; }
            if (pid == 10) { line = q * 4 + rl; off = j; }
            if (pid == 11) { line = q; off = ro; }
            if (pid == 12) { line = q * 4 + j / 4; off = ro; }
            if (pid == 13) { line = q * 2 + j / 8; off = ro; }
            pat[l] = (uint16_t)(line << 8 | off);
        }
        CK(hipMemcpyToSymbol(HIP_SYMBOL(c_pat), pat, sizeof pat));
        char nm[16];
        snprintf(nm, sizeof nm, "P%d", pid);
        t(nm, pid, [&] { probe<5><<<wgs, 256>>>(T, iters, 1, out, lmask, shared); });
    }
    return 0;
}
