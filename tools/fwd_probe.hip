// Ablation probe for the forward SpGEMM on gfx950 (not product code).
// Reddit-sized random graph (uniform degree), k=16, D=256.  Times variants:
//   A  full kernel (gather data+sel, ds_add into per-wave LDS row)
//   B  no LDS atomics (register sum)         -> cost of gathers alone
//   C  no sel gather (synthetic selector)     -> cost of data gather + atomics
//   D  no gathers at all (col/val stream + atomics)
//   P  packed 128-B CBSR records (data+sel in one line), dwordx4 per lane
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/fwd_probe.hip -o tools/fwd_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int K = 16, D = 256, KG = 16, G = 64 / KG;

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

__global__ void init_graph(int *col, float *val, int64_t E, int V) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        col[e] = hash32((uint32_t)e * 2654435761u + 17u) % V;
        val[e] = (hash32((uint32_t)e + 99u) & 0xffff) / 65536.f;
    }
}
__global__ void init_cbsr(float *cv, uint8_t *ci, int V) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V * K; i += gridDim.x * blockDim.x) {
        cv[i] = (hash32(i + 5u) & 0xffff) / 65536.f;
        const uint32_t h = hash32(i / K + 7u);
        ci[i] = (uint8_t)(((h & 255) + (i % K) * ((h >> 8) | 1)) & 255);  // distinct within a row
    }
}
// packed record per vertex: 64 B data + 16 B sel + 48 B pad = 128 B
__global__ void pack_cbsr(const float *cv, const uint8_t *ci, uint4 *rec, int V) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const uint4 *d = reinterpret_cast<const uint4 *>(cv + (int64_t)v * K);
    const uint4 *s = reinterpret_cast<const uint4 *>(ci + (int64_t)v * K);
    for (int j = 0; j < 4; ++j) rec[(int64_t)v * 8 + j] = d[j];
    rec[(int64_t)v * 8 + 4] = s[0];
}

template <int MODE, int U>
__global__ __launch_bounds__(256) void fwd(const int *row_ptr, const int *col, const float *val,
                                           const float *cv, const uint8_t *ci, float *out, int V) {
    __shared__ __attribute__((aligned(16))) float lds[4][256];
    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = blockIdx.x * 4 + wid;
    if (r >= V) return;
    float *acc = lds[wid];
    *reinterpret_cast<float4 *>(&acc[lane * 4]) = make_float4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    const int grp = lane / KG, l = lane % KG;
    const int sb = row_ptr[r], se = row_ptr[r + 1];
    float regsum = 0.f;
    for (int base = sb; base < se; base += G * U) {
        int c[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int e = base + u * G + grp;
            int ec = e < se ? e : se - 1;
            c[u] = col[ec];
            float wv = val[ec];
            w[u] = e < se ? wv : 0.f;
        }
        float v[U];
        int s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int q = c[u] * K + l;
            if (MODE == 3) {
                v[u] = 1.f;
                s[u] = (c[u] * 7 + l * 16) & 255;
            } else {
                v[u] = cv[q];
                s[u] = MODE == 2 ? ((c[u] * 7 + l * 16) & 255) : ci[q];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE == 1)
                regsum += w[u] * v[u] * (float)(s[u] + 1);
            else
                atomicAdd(&acc[s[u]], w[u] * v[u]);
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float4 a = *reinterpret_cast<float4 *>(&acc[lane * 4]);
    a.x += regsum;
    *reinterpret_cast<float4 *>(&out[(int64_t)r * D + lane * 4]) = a;
}

// packed: 5 lanes per edge (4 data dwordx4 + 1 sel dwordx4), 12 edges per wave step
template <int U>
__global__ __launch_bounds__(256) void fwd_packed(const int *row_ptr, const int *col,
                                                  const float *val, const uint4 *rec, float *out,
                                                  int V) {
    __shared__ __attribute__((aligned(16))) float lds[4][256];
    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = blockIdx.x * 4 + wid;
    if (r >= V) return;
    float *acc = lds[wid];
    *reinterpret_cast<float4 *>(&acc[lane * 4]) = make_float4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    const int grp = lane / 5, sub = lane % 5;  // grp 0..12 (12 = idle lanes 60..63)
    const int sb = row_ptr[r], se = row_ptr[r + 1];
    const int selsrc = (lane - sub + 4) * 4;  // byte address of this group's sel lane for bpermute
    for (int base = sb; base < se; base += 12 * U) {
        int c[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int e = base + u * 12 + grp;
            bool ok = grp < 12 && e < se;
            int ec = ok ? e : se - 1;
            c[u] = col[ec];
            float wv = val[ec];
            w[u] = ok ? wv : 0.f;
        }
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = rec[(int64_t)c[u] * 8 + sub];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // fetch this group's sel dword #sub from lane (group base + 4)
            const int sx = __builtin_amdgcn_ds_bpermute(selsrc, (int)q[u].x);
            const int sy = __builtin_amdgcn_ds_bpermute(selsrc, (int)q[u].y);
            const int sz = __builtin_amdgcn_ds_bpermute(selsrc, (int)q[u].z);
            const int sw = __builtin_amdgcn_ds_bpermute(selsrc, (int)q[u].w);
            const int sel4 = sub == 0 ? sx : sub == 1 ? sy : sub == 2 ? sz : sw;
            if (sub < 4) {
                atomicAdd(&acc[sel4 & 255], w[u] * __uint_as_float(q[u].x));
                atomicAdd(&acc[(sel4 >> 8) & 255], w[u] * __uint_as_float(q[u].y));
                atomicAdd(&acc[(sel4 >> 16) & 255], w[u] * __uint_as_float(q[u].z));
                atomicAdd(&acc[(sel4 >> 24) & 255], w[u] * __uint_as_float(q[u].w));
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    *reinterpret_cast<float4 *>(&out[(int64_t)r * D + lane * 4]) =
        *reinterpret_cast<float4 *>(&acc[lane * 4]);
}

// RMW: one LDS accumulator copy per edge group (selectors distinct within an edge ->
// no address conflicts inside one instruction); plain ds_read + ds_write.
// CO=1: coalesced col/val loads (lane i loads edge base+i) + bpermute distribution.
template <int U, int CO>
__global__ __launch_bounds__(256) void fwd_rmw(const int *row_ptr, const int *col, const float *val,
                                               const float *cv, const uint8_t *ci, float *out,
                                               int V) {
    __shared__ __attribute__((aligned(16))) float lds[4][G][256];
    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = blockIdx.x * 4 + wid;
    if (r >= V) return;
    const int grp = lane / KG, l = lane % KG;
    float *acc = lds[wid][grp];
    for (int g = 0; g < G; ++g)
        *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]) = make_float4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    const int sb = row_ptr[r], se = row_ptr[r + 1];
    for (int base = sb; base < se; base += G * U) {
        int c[U];
        float w[U];
        if (CO) {
            static_assert(G * U <= 64, "one coalesced load per step");
            const int e = base + lane;
            const int ec = e < se ? e : se - 1;
            const int cl = col[ec];
            const float wl = e < se ? val[ec] : 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int src = (u * G + grp) * 4;
                c[u] = __builtin_amdgcn_ds_bpermute(src, cl);
                w[u] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(wl)));
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int e = base + u * G + grp;
                int ec = e < se ? e : se - 1;
                c[u] = col[ec];
                float wv = val[ec];
                w[u] = e < se ? wv : 0.f;
            }
        }
        float v[U];
        int s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int q = c[u] * K + l;
            v[u] = cv[q];
            s[u] = ci[q];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[s[u]] += w[u] * v[u];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float4 a = make_float4(0, 0, 0, 0);
    for (int g = 0; g < G; ++g) {
        float4 b = *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4 *>(&out[(int64_t)r * D + lane * 4]) = a;
}

// dwordx4 data gather: 4 lanes per edge, 4 consecutive l per lane, 16 edges/step, 16 copies
template <int U>
__global__ __launch_bounds__(256) void fwd_x4(const int *row_ptr, const int *col, const float *val,
                                              const float *cv, const uint8_t *ci, float *out, int V) {
    constexpr int GE = 16;  // edges per step
    __shared__ __attribute__((aligned(16))) float lds[4][GE][256];
    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = blockIdx.x * 4 + wid;
    if (r >= V) return;
    const int grp = lane / 4, q4 = lane % 4;
    float *acc = lds[wid][grp];
    for (int g = 0; g < GE; ++g)
        *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]) = make_float4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    const int sb = row_ptr[r], se = row_ptr[r + 1];
    for (int base = sb; base < se; base += GE * U) {
        int c[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int e = base + u * GE + grp;
            int ec = e < se ? e : se - 1;
            c[u] = col[ec];
            float wv = val[ec];
            w[u] = e < se ? wv : 0.f;
        }
        float4 v[U];
        uint32_t s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = reinterpret_cast<const float4 *>(cv)[c[u] * 4 + q4];
            s[u] = reinterpret_cast<const uint32_t *>(ci)[c[u] * 4 + q4];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc[s[u] & 255] += w[u] * v[u].x;
            acc[(s[u] >> 8) & 255] += w[u] * v[u].y;
            acc[(s[u] >> 16) & 255] += w[u] * v[u].z;
            acc[s[u] >> 24] += w[u] * v[u].w;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float4 a = make_float4(0, 0, 0, 0);
    for (int g = 0; g < GE; ++g) {
        float4 b = *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4 *>(&out[(int64_t)r * D + lane * 4]) = a;
}

// packed record stride RS bytes: [k f32 | k u8 | pad]; same lane mapping as fwd_rmw
__global__ void pack_rs(const float *cv, const uint8_t *ci, uint8_t *rec, int V, int RS) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;  // one thread per (v, l)
    if (i >= V * K) return;
    int v = i / K, l = i % K;
    reinterpret_cast<float *>(rec + (int64_t)v * RS)[l] = cv[i];
    rec[(int64_t)v * RS + 4 * K + l] = ci[i];
}
template <int U>
__global__ __launch_bounds__(256) void fwd_q(const int *row_ptr, const int *col, const float *val,
                                             const uint8_t *rec, int RS, float *out, int V) {
    __shared__ __attribute__((aligned(16))) float lds[4][G][256];
    const int wid = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = blockIdx.x * 4 + wid;
    if (r >= V) return;
    const int grp = lane / KG, l = lane % KG;
    float *acc = lds[wid][grp];
    for (int g = 0; g < G; ++g)
        *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]) = make_float4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    const int sb = row_ptr[r], se = row_ptr[r + 1];
    for (int base = sb; base < se; base += G * U) {
        int c[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int e = base + u * G + grp;
            int ec = e < se ? e : se - 1;
            c[u] = col[ec];
            float wv = val[ec];
            w[u] = e < se ? wv : 0.f;
        }
        float v[U];
        int s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint8_t *p = rec + (int64_t)c[u] * RS;
            v[u] = reinterpret_cast<const float *>(p)[l];
            s[u] = p[4 * K + l];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[s[u]] += w[u] * v[u];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float4 a = make_float4(0, 0, 0, 0);
    for (int g = 0; g < G; ++g) {
        float4 b = *reinterpret_cast<float4 *>(&lds[wid][g][lane * 4]);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4 *>(&out[(int64_t)r * D + lane * 4]) = a;
}

template <typename F>
float timeit(F f, int reps = 10) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
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

int main(int argc, char **argv) {
    const int V = 232965;
    const int deg = argc > 1 ? atoi(argv[1]) : 492;
    const int64_t E = (int64_t)V * deg;
    std::vector<int> hrp(V + 1);
    for (int i = 0; i <= V; ++i) hrp[i] = (int)((int64_t)i * deg);
    int *rp, *col;
    float *val, *cv, *out;
    uint8_t *ci;
    uint4 *rec;
    CK(hipMalloc(&rp, (V + 1) * 4));
    CK(hipMalloc(&col, E * 4));
    CK(hipMalloc(&val, E * 4));
    CK(hipMalloc(&cv, (size_t)V * K * 4));
    CK(hipMalloc(&ci, (size_t)V * K));
    CK(hipMalloc(&rec, (size_t)V * 128));
    CK(hipMalloc(&out, (size_t)V * D * 4));
    CK(hipMemcpy(rp, hrp.data(), (V + 1) * 4, hipMemcpyHostToDevice));
    init_graph<<<4096, 256>>>(col, val, E, V);
    init_cbsr<<<1024, 256>>>(cv, ci, V);
    pack_cbsr<<<(V + 255) / 256, 256>>>(cv, ci, rec, V);
    CK(hipDeviceSynchronize());
    const dim3 grid((V + 3) / 4), blk(256);
    const double alg = 4.0 * (V + 1) + 8.0 * E + 5.0 * K * E + 4.0 * V * D;
    auto rep = [&](const char *name, float ms) {
        printf("%-40s %8.3f ms  %7.2f GTEPS  %7.1f GB/s alg\n", name, ms, E / ms / 1e6, alg / ms / 1e6);
    };
    printf("V=%d deg=%d E=%lld\n", V, deg, (long long)E);
    rep("A full U=8", timeit([&] { fwd<0, 8><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("A full U=4", timeit([&] { fwd<0, 4><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("A full U=16", timeit([&] { fwd<0, 16><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("B no LDS atomics", timeit([&] { fwd<1, 8><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("C no sel gather", timeit([&] { fwd<2, 8><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("D no gathers (atomics only)",
        timeit([&] { fwd<3, 8><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("P packed 128B records U=4",
        timeit([&] { fwd_packed<4><<<grid, blk>>>(rp, col, val, rec, out, V); }));
    rep("P packed 128B records U=8",
        timeit([&] { fwd_packed<8><<<grid, blk>>>(rp, col, val, rec, out, V); }));
    rep("R rmw U=4", timeit([&] { fwd_rmw<4, 0><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("R rmw U=8", timeit([&] { fwd_rmw<8, 0><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("R rmw U=16", timeit([&] { fwd_rmw<16, 0><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("R rmw coalesced col U=8", timeit([&] { fwd_rmw<8, 1><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("R rmw coalesced col U=16", timeit([&] { fwd_rmw<16, 1><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("X dwordx4 gather U=2", timeit([&] { fwd_x4<2><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    rep("X dwordx4 gather U=4", timeit([&] { fwd_x4<4><<<grid, blk>>>(rp, col, val, cv, ci, out, V); }));
    uint8_t *rec2;
    CK(hipMalloc(&rec2, (size_t)V * 128));
    for (int RS : {80, 96, 128}) {
        pack_rs<<<(V * K + 255) / 256, 256>>>(cv, ci, rec2, V, RS);
        CK(hipDeviceSynchronize());
        char nm[64];
        snprintf(nm, sizeof nm, "Q packed RS=%d U=8", RS);
        rep(nm, timeit([&] { fwd_q<8><<<grid, blk>>>(rp, col, val, rec2, RS, out, V); }));
        snprintf(nm, sizeof nm, "Q packed RS=%d U=16", RS);
        rep(nm, timeit([&] { fwd_q<16><<<grid, blk>>>(rp, col, val, rec2, RS, out, V); }));
    }
    rep("pack_rs kernel", timeit([&] { pack_rs<<<(V * K + 255) / 256, 256>>>(cv, ci, rec2, V, 128); }));
    rep("pack kernel", timeit([&] { pack_cbsr<<<(V + 255) / 256, 256>>>(cv, ci, rec, V); }));
    return 0;
}
