// Shared host/device helpers for libmaxk_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>

#include "maxk_hip.h"

namespace maxk {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kBlock = 256;        // threads per workgroup (4 waves; 512 / 1024 measured slower)
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kMaxDim = 256;       // uint8 selector range: per-wave LDS rows are 256 floats
// Bucketed backward, phase 2: fp64 LDS accumulator of one destination bucket (144 KiB);
// a bucket holds 2^shift destinations with 2^shift * (k + 1) <= kBucketAccDoubles (rows
// padded to k + 1 doubles so the rows of one wave instruction's random destinations spread
// over the LDS banks instead of all starting on the same few).
constexpr int kBucketAccDoubles = 18432;

// Tuning knobs (compile-time; tools/tune.sh builds variants).  *_U = edge
// batches in flight per wave, *_WAVES = __launch_bounds__ min waves per SIMD.
#ifndef MAXK_FWD_U
#define MAXK_FWD_U 8
#endif
#ifndef MAXK_BWD_U
#define MAXK_BWD_U 8
#endif
#ifndef MAXK_FWD_SHORT  // forward: rows of at most this many edges go in batches of 64/KG
#define MAXK_FWD_SHORT 16  // (one row per lane group); 0 = off
#endif
#ifndef MAXK_FWD_STREAM  // forward, sparse graphs: lane groups stream rows of at most this many
#define MAXK_FWD_STREAM 64  // edges each (stream_rows); 0 = off (the short-row batches)
#endif
#ifndef MAXK_FWD_RECORDS  // streaming forward, k in [24, 32]: 5k-byte transport records instead
#define MAXK_FWD_RECORDS 1  // of the packed ones (maxk_records_ok); 0 = the packed records
#endif
#ifndef MAXK_FWD_RECORDS_DEEP  // ... and in the dense graphs' deep-batch walk (Reddit k = 32
                               // forward 3.296 -> 3.274 ms, profiles/r05/tune/transport_records/)
#define MAXK_FWD_RECORDS_DEEP 1
#endif
#ifndef MAXK_FWD_WAVES
#define MAXK_FWD_WAVES 1
#endif
#ifndef MAXK_FWD_EMIT_WAVES  // the forward emitting edge selectors: __launch_bounds__ minimum
#define MAXK_FWD_EMIT_WAVES 1   // (workgroups per CU) -- a VGPR cap for its occupancy
#endif
#ifndef MAXK_BWD_WAVES
#define MAXK_BWD_WAVES 1
#endif
#ifndef MAXK_XCD_SUM  // XCD-contiguous work order in the backward's phase 2
#define MAXK_XCD_SUM 1
#endif
#ifndef MAXK_XCD_SUM_RUN  // csc phase 2: blocks per XCD run (0: one contiguous eighth each)
#define MAXK_XCD_SUM_RUN 64
#endif
#ifndef MAXK_BWD_X4  // 4-l-per-lane phase 1 of the two-phase backward (k % 4 == 0)
#define MAXK_BWD_X4 1
#endif
#ifndef MAXK_X4_U  // phase-1 depth; 0 = chosen per launch from the average degree
#define MAXK_X4_U 0
#endif
#ifndef MAXK_PULL_SHIFT_DELTA  // pull buckets of 2^(maxk_bucket_shift(k) - delta) columns
#define MAXK_PULL_SHIFT_DELTA 0
#endif
constexpr size_t kPullLdsBytes = 160 * 1024;  // LDS of one workgroup on gfx950
// pull_q_kernel accumulator row stride in doubles: kp + 1 (the pad spreads a wave's
// destinations over the LDS banks) when the padded bucket fits, else kp
__host__ __device__ inline int pull_ks(int kp, int shift) {
    return ((((size_t)(kp + 1) * 8 + kp) << shift) <= kPullLdsBytes) ? kp + 1 : kp;
}
#ifndef MAXK_PULL_SHFL  // pull: the step's entries by one load + lane shuffles
#define MAXK_PULL_SHFL 1
#endif
#ifndef MAXK_PULL_F4_FLUSH  // pull: tile partials stored 16 B per lane
#define MAXK_PULL_F4_FLUSH 1
#endif
#ifndef MAXK_PULL_U  // pull_tile_kernel: wave instructions of entries per step
#define MAXK_PULL_U 4
#endif
#ifndef MAXK_PULL_QU  // pull_q_kernel: wave instructions of entries per step (U=2 vs 4: Reddit
#define MAXK_PULL_QU 2   // k=8 1.53 vs 1.62 ms, k=32 3.60 vs 3.80, k=16 equal)
#endif
#ifndef MAXK_PULL_Q  // pull, k % 4 == 0: quantile-slot selectors + pipelined pull_q_kernel
#define MAXK_PULL_Q 1
#endif
#ifndef MAXK_PULL_H  // pull_q_kernel: most parts per tile (destination slots split by rank)
#define MAXK_PULL_H 16
#endif
#ifndef MAXK_PULL_MIN_KP  // pull_q_kernel: fewest slots per destination a part keeps, k < 32
#define MAXK_PULL_MIN_KP 8
#endif
#ifndef MAXK_PULL_MIN_KP_WIDE  // ... and for k >= 32
#define MAXK_PULL_MIN_KP_WIDE 16
#endif
#ifndef MAXK_PULL_TRANSPOSE  // pull_q_kernel: a quarter's entries interleaved across its quads
#define MAXK_PULL_TRANSPOSE 1
#endif
// pull_q_kernel: values per lane for 8-slot parts (2, 4 or 8; 0: 8 when k = 8, else 4).
// Reddit (profiles/r02/tune/pull_vpl.txt): k = 16 VPL 2 / 4 / 8 = 2.54 / 2.39 / 2.41 ms
// (2.23 / 2.25 at S = 33); k = 8 VPL 4 / 8 = 1.54 / 1.50 ms
#ifndef MAXK_PULL_VPL8
#define MAXK_PULL_VPL8 0
#endif
#ifndef MAXK_PACK4  // forward record pack: four l per thread (k % 4 == 0, aligned CBSR)
#define MAXK_PACK4 1
#endif
#ifndef MAXK_TOPK_BISECT  // four-row top-k: bisection over [lower bound, max] of the keys
#define MAXK_TOPK_BISECT 1
#endif
#ifndef MAXK_TOPK_LB  // four-row top-k: bit search from a lower bound of the k-th key
#define MAXK_TOPK_LB 1
#endif
#ifndef MAXK_PULL_SEL4  // pull_sel4_kernel: four selectors per thread (aligned selectors)
#define MAXK_PULL_SEL4 1
#endif
#ifndef MAXK_PULL_XCD  // pull_q_kernel: XCD x runs the x-th eighth of the tile sequence
#define MAXK_PULL_XCD 1
#endif
#ifndef MAXK_FWD_XCD  // forward items in XCD-contiguous order
#define MAXK_FWD_XCD 1  // Reddit / products neutral, ordered products_comm 4.71 -> 3.65 ms
#endif
#ifndef MAXK_P1_XCD  // backward phase 1 items in XCD-contiguous order
#define MAXK_P1_XCD 1  // products_comm ordered 8.47 -> 8.39 ms, random graphs neutral
#endif
#ifndef MAXK_CSC_STAGE  // csc phase 2: an item's csc_eid slots staged in LDS first
#define MAXK_CSC_STAGE 1
#endif
#ifndef MAXK_T_AUX  // cache policy of the contribution stores: 0 plain, 2 nt, 16 sc1
#define MAXK_T_AUX 2
#endif
#ifndef MAXK_SCATTER_ROWS4  // dense scatter: four rows per wave
#define MAXK_SCATTER_ROWS4 1
#endif
#ifndef MAXK_TOPK_BLOCKS  // grid cap of the grid-stride top-k (rows per wave grow past it)
#define MAXK_TOPK_BLOCKS 16384
#endif
#ifndef MAXK_P1_ITEMS  // backward auto item size: items per resident wave slot (phase 1 / 2)
#define MAXK_P1_ITEMS 16
#endif
#ifndef MAXK_P2_ITEMS
#define MAXK_P2_ITEMS 16
#endif
#ifndef MAXK_PACK_GRID  // grid cap of the grid-stride record pack
#define MAXK_PACK_GRID 4096
#endif
#ifndef MAXK_BUCKET_U  // bucketed phase-2 depth (wave steps of loads in flight)
#define MAXK_BUCKET_U 8
#endif
#ifndef MAXK_BUCKET_PARTS  // bucketed phase 2: parts (workgroups) per CU
#define MAXK_BUCKET_PARTS 4
#endif
#ifndef MAXK_TOPK_ROWS4  // top-k: 4 rows per wave on 16-lane DPP rows (0: one row per wave)
#define MAXK_TOPK_ROWS4 1
#endif
#ifndef MAXK_TOPK_ROWS4_KMAX  // ... for k up to this (at most 64; k=64 ties one row per wave)
#define MAXK_TOPK_ROWS4_KMAX 48
#endif
#ifndef MAXK_TOPK_FENCE_WAIT  // tools only: s_waitcnt lgkmcnt(0) in the four-row top-k's fences
#define MAXK_TOPK_FENCE_WAIT 0
#endif
#ifndef MAXK_FWD_OUT_NT  // forward: non-temporal output row stores (0 never, 1 always, 2 when
#define MAXK_FWD_OUT_NT 2   // the output exceeds the Infinity Cache)
#endif
constexpr size_t kInfinityCacheBytes = 256ull << 20;  // MI355X MALL (MI355X_MICROARCH.md)
#ifndef MAXK_BSORT_U  // window-sorted phase 1: wave instructions of edges per batch
#define MAXK_BSORT_U 2
#endif
#ifndef MAXK_DENSE_ROUTE  // k >= D / 2: aggregate dense rows (dense_route.hip); 0 = off
#define MAXK_DENSE_ROUTE 1
#endif
#ifndef MAXK_DENSE_DMAX  // the dense route's largest D
#define MAXK_DENSE_DMAX 128
#endif
#ifndef MAXK_DENSE_U  // dense_rows_kernel: edges per lane-group step (Flickr-sized D = 64,
#define MAXK_DENSE_U 4  // k = 64: 0.094 ms at 8, 0.070 at 4)
#endif
#ifndef MAXK_DENSE_PICK  // the dense backward below k = D / 2: selected columns per lane
#define MAXK_DENSE_PICK 1   // (pick_rows_kernel); 0 = dense rows and a selecting store
#endif
#ifndef MAXK_DENSE_PICK_DMAX  // the automatic mode takes the pick form on small graphs of D at
#define MAXK_DENSE_PICK_DMAX 64  // most this, k >= D / 4 (0 = never)
#endif
#ifndef MAXK_DENSE_WAVES  // dense_rows_kernel: resident waves per CU its item size assumes
#define MAXK_DENSE_WAVES 24
#endif
#ifndef MAXK_CSC_GROUP_DEG  // csc phase 2: lane groups per destination (csc_groups) below this
#define MAXK_CSC_GROUP_DEG 16  // average in-degree (slots per destination); 0 = off
#endif
#ifndef MAXK_CSC_GROUP_U  // csc_groups: slots per lane-group step
#define MAXK_CSC_GROUP_U 4
#endif
#ifndef MAXK_T_LOAD_NT  // csc phase 2: non-temporal reads of whole-line T rows (k % 32 == 0)
#define MAXK_T_LOAD_NT 1
#endif
#ifndef MAXK_SUM_U  // phase-2 depth; 0 = chosen per launch from the average in-degree
#define MAXK_SUM_U 0
#endif

// ---- error reporting (host) ----
void set_error(const char *fmt, ...);
void clear_error();

#define MAXK_REQUIRE(cond, ...)                  \
    do {                                         \
        if (!(cond)) {                           \
            ::maxk::set_error(__VA_ARGS__);      \
            return MAXK_ERR_INVALID;             \
        }                                        \
    } while (0)

#define MAXK_HIP(call)                                                              \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) {                                                     \
            ::maxk::set_error("%s failed: %s", #call, hipGetErrorString(e_));       \
            return MAXK_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

// After a launch: report a launch error (never synchronises).
#define MAXK_LAUNCHED(name)                                                         \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) {                                                     \
            ::maxk::set_error("%s launch failed: %s", name, hipGetErrorString(e_)); \
            return MAXK_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// CUs of the current device (hipDeviceAttributeMultiprocessorCount), cached per device ordinal:
// the grid and work-item sizing of every launch scales with it.  256 (MI355X) when no device
// answers (the CPU-only build check, the workspace-size queries of the C-ABI tests).
inline int64_t device_cus() {
    constexpr int kMaxDevices = 64;
    static std::atomic<int> cache[kMaxDevices] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        (void)hipGetLastError();
        return 256;
    }
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0) {
            (void)hipGetLastError();
            n = 256;
        }
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

// The current device's ordinal (0 without one): the key of per-device launch-size caches.
inline int device_ordinal() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) {
        (void)hipGetLastError();
        return 0;
    }
    return dev;
}

// Lanes per edge group: next power of two >= k, capped at a wave.
inline int lanes_per_edge(int k) {
    int g = 1;
    while (g < k && g < kWave) g <<= 1;
    return g;
}

// ---- device helpers ----
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Zero n 4-byte words on the stream with a kernel.  Launch paths use this instead of
// hipMemsetAsync: a memset captured into a hipGraph (ROCm 7.2) zeroed its buffer on the first
// replay only, so the hybrid backward (tests/test_parity_gpu.py hipgraph capture) summed onto
// stale values from the second replay on (tools/capture_probe*.py).
__global__ void zero_words_kernel(uint32_t *__restrict__ p, int64_t n);
int zero_words(void *p, int64_t n, hipStream_t s);

// Dense route (dense_route.hip): whether (D, k) takes it, and the forward through it
bool dense_route(int D, int k);
bool dense_pick(int D, int k);  // the dense backward's selected-column form below k = D / 2
size_t dense_forward_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e, int D,
                                    int chunk);
int dense_forward(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                  const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div,
                  float *out, int64_t num_rows, int64_t num_cols, int64_t num_e, int D, int k,
                  int chunk, void *workspace, size_t workspace_bytes, hipStream_t s,
                  int accumulate);

// The hardware hands workgroup b to XCD b % 8 (each XCD has its own L2).  With
// grid = 8 * per, logical block (b % 8) * per + b / 8 makes XCD x run the contiguous
// logical range [x * per, (x + 1) * per) in launch order, so work items that are
// neighbours (and touch neighbouring lines) share one L2 instead of eight.
constexpr int kXcds = 8;
inline int64_t xcd_grid(int64_t blocks) { return (blocks + kXcds - 1) / kXcds * kXcds; }
__device__ __forceinline__ int xcd_contiguous_block(int b, int grid) {
    const int per = grid / kXcds;
    return (b % kXcds) * per + b / kXcds;
}
// The same inside windows of kXcds * run blocks (grid a multiple of kXcds): each XCD walks
// runs of `run` consecutive blocks, one run per window, so work whose cost varies along the
// block sequence (a community-ordered shard: dense destination ranges beside nearly empty
// ones) still reaches every XCD evenly, which one contiguous eighth per XCD does not.
__device__ __forceinline__ int xcd_window_block(int b, int grid, int run) {
    const int w = kXcds * run;
    const int base = b / w * w;
    const int ws = grid - base < w ? grid - base : w;
    return base + xcd_contiguous_block(b - base, ws);
}

// Raw buffer descriptor over [p, p + bytes), built from wave-uniform values (SGPRs).
// The range check covers voffset + the instruction offset (not soffset): a load past
// the end returns 0 and a store past it is dropped, so clamps and predicates on the
// tail of a segment are unnecessary.  Offsets are 32-bit: no 64-bit address math.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_buffer(const void *p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo),
                                             0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                             0x00020000);
}

// Orders this wave's LDS traffic at a phase change (all lanes of ONE wave):
// LDS executes a wave's instructions in order; this only stops the compiler
// from moving LDS accesses across the boundary.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Token-stream work partition shared by the SpGEMM/SSpMM kernels: row r's token
// sits at r + row_ptr[r], edge e of row q at e + q + 1; a work item owns a
// contiguous token range.  Returns the first r in [0, n] whose token is >= d
// (row_ptr[n] + n >= d required).  64-ary search by the whole wave; the result
// is wave-uniform.
__device__ __forceinline__ int wave_first_row_token(const int32_t *__restrict__ row_ptr, int n,
                                                    int64_t d) {
    const int lane = lane_id();
    int lo = 0, hi = n;  // answer in [lo, hi]
    while (hi - lo > 63) {
        const int step = (hi - lo + 62) / 63;  // lo + 63*step >= hi
        int p = lo + lane * step;
        p = p > hi ? hi : p;
        const uint64_t m = __ballot((int64_t)row_ptr[p] + p >= d);  // lane 63 probes hi: true
        const int f = __builtin_ctzll(m);
        if (f == 0) {
            hi = lo;
        } else {
            const int pf = lo + f * step;
            lo = lo + (f - 1) * step + 1;
            hi = pf > hi ? hi : pf;
        }
    }
    const int p = lo + lane;
    const int pc = p > hi ? hi : p;
    const uint64_t m = __ballot(p <= hi && (int64_t)row_ptr[pc] + pc >= d) | (1ull << 63);
    const int r = lo + __builtin_ctzll(m);
    return r > hi ? hi : r;
}


// ---- split-row fixup shared by the forward (TAG 0) and the backward's phase 2 (TAG 1) ----
// out[row, 0:width] += slab[i, 0:width] for every run of consecutive items i whose
// slab_row[i] == row (a row split over items), added in item order: deterministic.  16
// lanes per item (4 items per wave): one wave per item made the launch bound by workgroup
// dispatch (65k items -> 16k workgroups), while most items do carry a slab, so every head
// must still run in parallel.  TAG only separates the two ops in profiles.
namespace {
template <int TAG>
__global__ __launch_bounds__(kBlock) void slab_fixup_kernel(const float *__restrict__ slab,
                                                            const int32_t *__restrict__ slab_row,
                                                            float *__restrict__ out, int width,
                                                            int n_items) {
    const int item = (int)((blockIdx.x * (int64_t)kBlock + threadIdx.x) / 16);
    const int g = threadIdx.x % 16;
    const int grp = (threadIdx.x % kWave) / 16;  // this item's lane group in the wave
    if (item >= n_items) return;
    const int row = slab_row[item];
    if (row < 0 || (item > 0 && slab_row[item - 1] == row)) return;
    // n = this row's slabs (consecutive items), found 16 items per step by the group's lanes:
    // a hub row cut into many items (a vertex-range shard's small chunks: Reddit's max-degree
    // row spans ~80 items of 256 tokens) would otherwise cost one dependent load per slab.
    int n = 1;
    for (int base = item + 1;; base += 16) {
        const int i = base + g;
        const bool same = i < n_items && slab_row[i] == row;
        const uint32_t mine = (uint32_t)(__ballot(same) >> (16 * grp)) & 0xffffu;
        const int run = __builtin_ctz(~mine | 0x10000u);
        n += run;
        if (run < 16) break;
    }
    float *o = out + (int64_t)row * width;
    const float *sl = slab + (int64_t)item * width;
    if ((width & 3) == 0 && width <= 256) {
        // up to 4 float4 columns per lane; slabs added in item order, 4 x 4 loads in flight
        constexpr int SU = 4;
        float4 a[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = g * 4 + 64 * c;
            a[c] = j < width ? *reinterpret_cast<const float4 *>(o + j) : make_float4(0, 0, 0, 0);
        }
        for (int i0 = 0; i0 < n; i0 += SU) {
            float4 b[SU][4];
#pragma unroll
            for (int u = 0; u < SU; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int j = g * 4 + 64 * c;
                    const int i = i0 + u < n ? i0 + u : n - 1;  // clamped: loaded, not added
                    b[u][c] = j < width ? *reinterpret_cast<const float4 *>(sl + (int64_t)i * width + j)
                                        : make_float4(0, 0, 0, 0);
                }
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                if (i0 + u >= n) break;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a[c].x += b[u][c].x;
                    a[c].y += b[u][c].y;
                    a[c].z += b[u][c].z;
                    a[c].w += b[u][c].w;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = g * 4 + 64 * c;
            if (j < width) *reinterpret_cast<float4 *>(o + j) = a[c];
        }
    } else {
        for (int j = g; j < width; j += 16) {
            float a = o[j];
            for (int i = 0; i < n; ++i) a += sl[(int64_t)i * width + j];
            o[j] = a;
        }
    }
}
}  // namespace

template <int TAG>
inline int launch_slab_fixup(const float *slab, const int32_t *slab_row, float *out, int width,
                             int n_items, hipStream_t s) {
    if (n_items <= 0) return MAXK_OK;
    hipLaunchKernelGGL(slab_fixup_kernel<TAG>, dim3((unsigned)ceil_div(n_items, kBlock / 16)),
                       dim3(kBlock), 0, s, slab, slab_row, out, width, n_items);
    MAXK_LAUNCHED("slab_fixup_kernel");
    return MAXK_OK;
}

}  // namespace maxk
