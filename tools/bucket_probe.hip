// Probe, not product.  Phase-2 read pattern of the two-phase backward: does reading the
// contribution rows T (CSR edge order, 64 B each at k=16) bucket by bucket in source order
// beat the per-destination CSC gather, and what does LDS accumulation cost?
//   graph: V=232,965, 492 stratified-random sorted columns per row (E=114.6M, Reddit-sized)
//   K1 csc      : 16 rows per wave instruction, CSC order (today's phase-2 pattern), register sum
//   K2 bucket   : same loop over the bucket list (edges whose column lies in one 2^B-column
//                 bucket, CSR order) -- neighbouring entries of one source row share lines
//   K3 wg+ds_add: one workgroup per bucket, LDS accumulator [2^B][16], ds_add_f32
//   K4 wg+rmw   : same, non-atomic ds_read_b128 / add / ds_write_b128 (racy: timing only)
//   K5 wg+reg   : same workgroup structure, register sum (no LDS)
//   K6 wg+f64   : LDS accumulator in fp64, ds_add_f64 (fast on gfx950, unlike ds_add_f32)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bucket_probe.hip -o tools/bucket_probe
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

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

constexpr int V = 232965, DEG = 492;
constexpr long long E = (long long)V * DEG;

__global__ void gen_cols(int *col, int *eid) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int r = (int)(e / DEG), i = (int)(e % DEG);
    const float u = (hash32((uint32_t)e * 2654435761u ^ 0x9e3779b9u) & 0xffffff) / 16777216.f;
    int c = (int)(((double)i + u) * V / DEG);
    col[e] = c < V ? c : V - 1;
    eid[e] = (int)e;
    (void)r;
}
__global__ void shift_keys(const int *col, int *key, int shift) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E) key[e] = col[e] >> shift;
}
__global__ void fill_t(float4 *T, long long n4) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x)
        T[i] = make_float4(1.f, 2.f, 3.f, (float)(i & 7));
}
__global__ void local_dest(const int *list, const int *col, unsigned short *ld, int mask) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < E) ld[i] = (unsigned short)(col[list[i]] & mask);
}
__global__ void bucket_ptr_k(const int *skey, int *bptr, int nb) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > E) return;
    int cur = t < E ? skey[t] : nb;
    int prev = t == 0 ? -1 : skey[t - 1];
    for (int b = prev + 1; b <= cur; ++b) bptr[b] = (int)t;
}

// K1/K2: waves walk contiguous chunks of `list`, 16 T rows (4 lanes x 16 B) per instruction.
template <int U>
__global__ __launch_bounds__(256) void list_gather(const float4 *T, const int *list, float *out,
                                                   long long chunk) {
    const int lane = threadIdx.x % 64, g = lane / 4, q = lane % 4;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const long long b0 = wave * chunk, b1 = b0 + chunk < E ? b0 + chunk : E;
    float4 a = make_float4(0, 0, 0, 0);
    for (long long base = b0; base < b1; base += 16 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long t = base + u * 16 + g;
            const int e = list[t < b1 ? t : b1 - 1];
            v[u] = T[(long long)e * 4 + q];
            if (t >= b1) v[u] = make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
        }
    }
    if (a.x == 1234.5f) out[0] = a.y + a.z + a.w;
}

// K3-K5: one workgroup (1024 threads) per bucket; wave w takes every 16th 16-entry step.
template <int MODE, int U, int NB>
__global__ __launch_bounds__(1024) void bucket_wg(const float4 *T, const int *list,
                                                  const unsigned short *ld, const int *bptr,
                                                  float *out) {
    using AT = typename std::conditional<MODE == 3, double, float>::type;
    __shared__ __attribute__((aligned(16))) AT acc[MODE == 2 ? 16 : NB * 16];
    const int lane = threadIdx.x % 64, g = lane / 4, q = lane % 4, w = threadIdx.x / 64;
    const int b = blockIdx.x;
    if (MODE != 2)
        for (int i = threadIdx.x; i < NB * 16; i += 1024) acc[i] = 0.f;
    __syncthreads();
    const long long s0 = bptr[b], s1 = bptr[b + 1];
    float4 a = make_float4(0, 0, 0, 0);
    for (long long base = s0 + (long long)w * 16 * U; base < s1; base += 16LL * 16 * U) {
        float4 v[U];
        int d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long t = base + u * 16 + g;
            const long long tc = t < s1 ? t : s1 - 1;
            const int e = list[tc];
            d[u] = ld[tc];
            v[u] = T[(long long)e * 4 + q];
            if (t >= s1) v[u] = make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (MODE == 0) {
                float *p = &acc[d[u] * 16 + q * 4];
                atomicAdd(p + 0, v[u].x);
                atomicAdd(p + 1, v[u].y);
                atomicAdd(p + 2, v[u].z);
                atomicAdd(p + 3, v[u].w);
            } else if constexpr (MODE == 3) {
                double *p = &acc[d[u] * 16 + q * 4];
                atomicAdd(p + 0, (double)v[u].x);
                atomicAdd(p + 1, (double)v[u].y);
                atomicAdd(p + 2, (double)v[u].z);
                atomicAdd(p + 3, (double)v[u].w);
            } else if constexpr (MODE == 1) {
                float4 *p = reinterpret_cast<float4 *>(&acc[d[u] * 16 + q * 4]);
                float4 o = *p;
                o.x += v[u].x; o.y += v[u].y; o.z += v[u].z; o.w += v[u].w;
                *p = o;
            } else {
                a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
            }
        }
    }
    __syncthreads();
    if (MODE != 2) {
        for (int i = threadIdx.x; i < NB * 16; i += 1024) a.x += (float)acc[i];
    }
    if (a.x == 1234.5f) out[0] = a.y + a.z + a.w;
}

int main() {
    int *col, *eid, *key, *skey, *csc, *blist, *bptr;
    unsigned short *ld;
    float4 *T;
    float *out;
    CK(hipMalloc(&col, E * 4));
    CK(hipMalloc(&eid, E * 4));
    CK(hipMalloc(&key, E * 4));
    CK(hipMalloc(&skey, E * 4));
    CK(hipMalloc(&csc, E * 4));
    CK(hipMalloc(&blist, E * 4));
    CK(hipMalloc(&ld, E * 2));
    CK(hipMalloc(&bptr, (V + 2) * 4));
    CK(hipMalloc(&T, E * 64));
    CK(hipMalloc(&out, 64));
    const int gb = (int)((E + 255) / 256);
    gen_cols<<<gb, 256>>>(col, eid);
    fill_t<<<8192, 256>>>(T, E * 4);
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, col, skey, eid, csc, (int)E, 0, 18));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, col, skey, eid, csc, (int)E, 0, 18));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto f) {
        f();
        CK(hipEventRecord(a));
        for (int i = 0; i < 5; ++i) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 5;
    };
    const long long chunk = 2048;
    const int waves = (int)((E + chunk - 1) / chunk);
    const int grid = (waves + 3) / 4;
    printf("K1 csc gather                 %.3f ms\n",
           timeit([&] { list_gather<8><<<grid, 256>>>(T, csc, out, chunk); }));
    for (int shift : {9, 10, 11}) {
        shift_keys<<<gb, 256>>>(col, key, shift);
        CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, skey, eid, blist, (int)E, 0, 9));
        const int nb = (V >> shift) + 1;
        bucket_ptr_k<<<(int)((E + 256) / 256), 256>>>(skey, bptr, nb);
        local_dest<<<gb, 256>>>(blist, col, ld, (1 << shift) - 1);
        printf("B=%d (%d buckets)\n", 1 << shift, nb);
        printf("  K2 bucket-list gather        %.3f ms\n",
               timeit([&] { list_gather<8><<<grid, 256>>>(T, blist, out, chunk); }));
        if (shift == 9) {
            printf("  K3 wg + ds_add_f32           %.3f ms\n",
                   timeit([&] { bucket_wg<0, 4, 512><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K4 wg + rmw (racy)           %.3f ms\n",
                   timeit([&] { bucket_wg<1, 4, 512><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K5 wg + reg                  %.3f ms\n",
                   timeit([&] { bucket_wg<2, 4, 512><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K6 wg + ds_add_f64           %.3f ms\n",
                   timeit([&] { bucket_wg<3, 4, 512><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K6 wg + ds_add_f64 U8        %.3f ms\n",
                   timeit([&] { bucket_wg<3, 8, 512><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
        } else if (shift == 10) {
            printf("  K3 wg + ds_add_f32           %.3f ms\n",
                   timeit([&] { bucket_wg<0, 4, 1024><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K4 wg + rmw (racy)           %.3f ms\n",
                   timeit([&] { bucket_wg<1, 4, 1024><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K5 wg + reg                  %.3f ms\n",
                   timeit([&] { bucket_wg<2, 4, 1024><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K6 wg + ds_add_f64           %.3f ms\n",
                   timeit([&] { bucket_wg<3, 4, 1024><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
            printf("  K6 wg + ds_add_f64 U8        %.3f ms\n",
                   timeit([&] { bucket_wg<3, 8, 1024><<<nb, 1024>>>(T, blist, ld, bptr, out); }));
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
