// Forward row-wise-product SpGEMM for gfx950:  out = diag(1/row_div) . A . scatter(CBSR)
//
// Semantics: kernels/spmm_maxk.cu:17-106 (spmm_kernel_opt2_sparse_v3) and the
// /in_degrees of maxk_spgemm_function.py:85-86.  Design (not a translation):
//
//  1. cbsr_pack_kernel: the CBSR of every source vertex is copied into ONE
//     record [k f32 | k u16 | pad] of RS bytes (RS = 128 for k = 16), so an edge
//     gathers one cache line instead of two (values and selectors live in
//     separate arrays at the boundary).  The pack also folds duplicate selectors
//     of a row into their first occurrence (later ones point at a never-read
//     trash column), which makes step 2's non-atomic accumulation exact for any
//     input.  Measured on MI355X (tools/fwd_probe.hip): 1 line/edge instead of 2
//     takes the Reddit-sized forward from 2.8 ms to 1.9 ms.
//  2. spgemm_fwd_kernel, one wavefront per work item:
//     * work partition: the CSR is read as a token stream of V row tokens and E
//       edge tokens (common.h); item i = tokens [i*C, (i+1)*C) -> every wave gets
//       <= C edges and <= C rows whatever the degree skew;
//     * KG = pow2ceil(k) (>= 8) lanes per edge, G = 64/KG edges per wave step,
//       U steps in flight, all loads unconditional (clamped addresses);
//     * accumulation: G LDS copies of the output row, one per edge group, with
//       plain ds_read/ds_write.  Within a step the lanes of one group hit
//       distinct columns (deduplicated selectors) and different groups hit
//       different copies, so no atomics are needed.  (ds_add_f32 LDS atomics cost
//       ~3 cycles per lane on gfx950: 9.4 ms vs 2.8 ms for the same gathers.)
//     * write-back: a row whose tokens all lie in this item is stored once
//       (copies summed in fixed order, divided by row_div, 16-B stores): no
//       zero-init of `out`, no global atomics.  A hub row continued from the
//       previous item goes to a per-item slab.
//  3. slab_fixup_kernel<0> (common.h) adds the slabs of each split row in item order
//     (deterministic) onto the owner's partial.
#include "common.h"

namespace maxk {
namespace {

// Record stride: one power-of-two slot per vertex while the record
// [k f32 | k u16 selectors] fits a 128-B line, else whole lines.
// Past one line: whole 64-B sectors while the table stays well inside the 256 MiB
// Infinity Cache (a smaller cache-resident table: Reddit k=32 3.60 -> 3.49 ms), whole
// 128-B lines once it does not (every gather is then a random HBM request per line and
// line-aligned records measured better: products k=32 6.53 -> 6.40 ms).
inline int record_stride(int k, int64_t num_cols) {
    const int b = 6 * k;
    if (b <= 128) {
        int s = 16;
        while (s < b) s <<= 1;
        return s;
    }
    const int s64 = (b + 63) / 64 * 64;
    if ((int64_t)s64 * num_cols <= (128LL << 20)) return s64;
    return (b + 127) / 128 * 128;
}

// Lanes per edge in the main kernel: pow2ceil(k), at least 8 (bounds the LDS copies per wave
// to 8, one per edge group).  On a sparse graph (average degree below kFwdSparseDegree) at
// least 16: a wave then walks many short rows, one dependent round of loads and an LDS flush
// each, and its 8 LDS copies at 8 lanes per edge (8.3 KB per wave at D = 256) cap a CU at 16
// waves; 16 lanes per edge (half of them idle at k <= 8) halve the copies and lift the cap to
// the VGPR limit (28 waves).  ogbn-products-sized, k = 8, forward with the edge-selector
// stream: 3.44 -> 3.16 ms, and 3.37 -> 3.15 ms on another box; Reddit-sized (average degree
// 492), where rows are long and the doubled gather instructions cost more than the occupancy
// buys: 1.395 -> 1.44 ms, so it keeps 8 (profiles/r04/tune/fwd_occupancy_ab*.txt).
constexpr int64_t kFwdSparseDegree = 128;
inline int fwd_lanes_per_edge(int k, int64_t num_rows, int64_t num_e) {
    const int g = lanes_per_edge(k);
    const int gmin = num_e < kFwdSparseDegree * num_rows ? 16 : 8;
    return g < gmin ? gmin : g;
}

// Packs the records of groups of whole vertices (vpw = min(32, 512 / k) per
// workgroup, one thread per (vertex, l)), grid-stride: a launch of one small
// workgroup per 256 (vertex, l) pairs is bound by workgroup dispatch (products
// k=32: 306k workgroups, 1.65 ms).  Duplicate selectors of a vertex: the first
// occurrence (lowest l, found with an LDS atomicMin per (vertex, selector))
// carries the sum of their values in l order, the others point at the trash
// column with value 0.  Selectors >= D also go to trash.  A record's u16 selector is the
// selector itself when it is kept, else 0x100 | selector: the walkers take min(selector,
// trash) as the LDS column (every index in [D, DS) is a never-flushed pad column of the copy),
// and the low byte stays the caller's selector, which the edge-selector stream of
// maxk_spgemm_forward_sel needs.
constexpr int kPackMaxV = 32;     // vertices per group (LDS: 32 x 256 first-occurrence slots)
constexpr int kPackBlock = 512;   // threads per pack workgroup (products: 0.34 -> 0.21 ms vs 256)

__global__ __launch_bounds__(kPackBlock) void cbsr_pack_kernel(const float *__restrict__ cbsr_val,
                                                           const uint8_t *__restrict__ cbsr_idx,
                                                           uint8_t *__restrict__ rec, int num_cols,
                                                           int k, int RS, int D, int trash) {
    __shared__ uint32_t s_first[kPackMaxV][256];
    __shared__ uint8_t s_sel[kPackBlock];
    __shared__ float s_val[kPackBlock];
    __shared__ int s_dup[kPackMaxV];
    const int vpw = k >= kPackBlock / kPackMaxV ? kPackBlock / k : kPackMaxV;
    const int t = threadIdx.x;
    const int vl = t / k, l = t - vl * k;
    for (int64_t g0 = (int64_t)blockIdx.x * vpw; g0 < num_cols; g0 += (int64_t)gridDim.x * vpw) {
        const int64_t v = g0 + vl;
        const bool act = vl < vpw && v < num_cols;
        int s = 0;
        float val = 0.f;
        if (act) {
            s = cbsr_idx[v * k + l];
            val = cbsr_val[v * k + l];
            s_sel[t] = (uint8_t)s;
            s_val[t] = val;
            s_first[vl][s] = 0xffffffffu;
        }
        if (t < vpw) s_dup[t] = 0;
        __syncthreads();
        if (act) atomicMin(&s_first[vl][s], (uint32_t)l);
        __syncthreads();
        const bool first = act && s_first[vl][s] == (uint32_t)l;
        if (act && !first) s_dup[vl] = 1;
        __syncthreads();
        if (act) {
            float outv = val;
            if (first && s_dup[vl]) {  // rare: fold the later duplicates, in l order
                for (int j = l + 1; j < k; ++j)
                    if (s_sel[vl * k + j] == s) outv += s_val[vl * k + j];
            }
            const bool keep = first && s < D;
            uint8_t *p = rec + v * RS;
            reinterpret_cast<float *>(p)[l] = keep ? outv : 0.f;
            reinterpret_cast<uint16_t *>(p + 4 * k)[l] = (uint16_t)(keep ? s : (0x100 | s));
        }
        __syncthreads();  // LDS is reused by the next group
    }
}

// cbsr_pack_kernel with four l per thread (k % 4 == 0, 16-B aligned values, 4-B aligned
// selectors): one u32 selector load, one float4 value load, one 16-B and one 8-B store per
// thread.  Duplicates are detected with a 256-bit column set per vertex (atomicOr returns
// the bit already set); a vertex with any takes the byte loop of cbsr_pack_kernel's rule
// (the lowest l of a selector carries the sum of its duplicates in l order).
__global__ __launch_bounds__(kPackBlock) void cbsr_pack4_kernel(const float *__restrict__ cbsr_val,
                                                            const uint8_t *__restrict__ cbsr_idx,
                                                            uint8_t *__restrict__ rec,
                                                            int num_cols, int k, int RS, int D,
                                                            int trash) {
    __shared__ uint32_t s_bits[kPackBlock * 8];  // up to kPackBlock vertices (k = 4)
    __shared__ int s_dup[kPackBlock];
    const int tpv = k >> 2;          // threads per vertex
    const int vpw = kPackBlock / tpv;  // vertices per group
    const int t = threadIdx.x;
    const int vl = t / tpv, l0 = (t - vl * tpv) * 4;
    for (int64_t g0 = (int64_t)blockIdx.x * vpw; g0 < num_cols; g0 += (int64_t)gridDim.x * vpw) {
        const int64_t v = g0 + vl;
        const bool act = vl < vpw && v < num_cols;
        for (int i = t; i < vpw * 8; i += kPackBlock) s_bits[i] = 0u;
        if (t < vpw) s_dup[t] = 0;
        __syncthreads();
        uint32_t w = 0u;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (act) {
            w = *reinterpret_cast<const uint32_t *>(cbsr_idx + v * k + l0);
            x = *reinterpret_cast<const float4 *>(cbsr_val + v * k + l0);
            uint32_t dup = 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sj = (w >> (8 * j)) & 255u;
                const uint32_t old = atomicOr(&s_bits[vl * 8 + (sj >> 5)], 1u << (sj & 31));
                dup |= (old >> (sj & 31)) & 1u;
            }
            if (dup) s_dup[vl] = 1;
        }
        __syncthreads();
        if (act) {
            float o[4] = {x.x, x.y, x.z, x.w};
            uint32_t sel[4];
            const bool any_dup = s_dup[vl] != 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sj = (w >> (8 * j)) & 255u;
                bool first = true;
                if (any_dup) {  // rare
                    const int l = l0 + j;
                    const uint8_t *ci = cbsr_idx + v * k;
                    const float *cv = cbsr_val + v * k;
                    for (int m = 0; m < l; ++m) first = first && ci[m] != sj;
                    if (first)
                        for (int m = l + 1; m < k; ++m)
                            if (ci[m] == sj) o[j] += cv[m];
                }
                const bool keep = first && (int)sj < D;
                o[j] = keep ? o[j] : 0.f;
                sel[j] = keep ? sj : (0x100u | sj);
            }
            uint8_t *p = rec + v * RS;
            *reinterpret_cast<float4 *>(p + 4 * l0) = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<uint2 *>(p + 4 * k + 2 * l0) =
                make_uint2(sel[0] | (sel[1] << 16), sel[2] | (sel[3] << 16));
        }
        __syncthreads();  // LDS is reused by the next group
    }
}

// Transport records (r05, maxk_cbsr_records / maxk_spgemm_forward_records): [k f32 | k u8] per
// vertex at a stride of 5k bytes -- the bytes a sharded forward all-gathers anyway -- so owners
// build them for their own rows before the exchange and receivers walk the gathered buffer with
// no pack over every gathered vertex.  The selectors stay the caller's bytes (the backward reads
// them); a repeated selector's first occurrence carries the sum of its values in l order and
// the later ones, and any selector >= D, carry kRecSkip (a NaN payload the walkers send to the
// trash column); a NaN value the caller kept is stored as the canonical quiet NaN, so kRecSkip
// never stands for a kept value.  One thread per (vertex, four l), k % 4 == 0.
constexpr uint32_t kRecSkip = 0x7fbadbadu;
__global__ __launch_bounds__(kPackBlock) void cbsr_records_kernel(const float *__restrict__ cbsr_val,
                                                                  const uint8_t *__restrict__ cbsr_idx,
                                                                  uint8_t *__restrict__ rec,
                                                                  int num_rows, int k, int D) {
    __shared__ uint32_t s_bits[kPackBlock * 8];
    __shared__ int s_dup[kPackBlock];
    const int tpv = k >> 2;
    const int vpw = kPackBlock / tpv;
    const int t = threadIdx.x;
    const int vl = t / tpv, l0 = (t - vl * tpv) * 4;
    const int RS = 5 * k;
    for (int64_t g0 = (int64_t)blockIdx.x * vpw; g0 < num_rows; g0 += (int64_t)gridDim.x * vpw) {
        const int64_t v = g0 + vl;
        const bool act = vl < vpw && v < num_rows;
        for (int i = t; i < vpw * 8; i += kPackBlock) s_bits[i] = 0u;
        if (t < vpw) s_dup[t] = 0;
        __syncthreads();
        uint32_t w = 0u;
        float o[4] = {0.f, 0.f, 0.f, 0.f};
        if (act) {
            const uint8_t *ci = cbsr_idx + v * k;
            const float *cv = cbsr_val + v * k;
            w = (uint32_t)ci[l0] | ((uint32_t)ci[l0 + 1] << 8) | ((uint32_t)ci[l0 + 2] << 16) |
                ((uint32_t)ci[l0 + 3] << 24);
            uint32_t bad = 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[j] = cv[l0 + j];
                const uint32_t sj = (w >> (8 * j)) & 255u;
                const uint32_t old = atomicOr(&s_bits[vl * 8 + (sj >> 5)], 1u << (sj & 31));
                bad |= ((old >> (sj & 31)) & 1u) | (sj >= (uint32_t)D ? 1u : 0u);
            }
            if (bad) s_dup[vl] = 1;
        }
        __syncthreads();
        if (act) {
            const bool any = s_dup[vl] != 0;
            uint8_t *p = rec + v * RS;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sj = (w >> (8 * j)) & 255u;
                float x = o[j];
                bool keep = sj < (uint32_t)D;
                if (any) {  // rare: the pack's rule (the first occurrence sums, in l order)
                    const int l = l0 + j;
                    const uint8_t *ci = cbsr_idx + v * k;
                    const float *cv = cbsr_val + v * k;
                    for (int m = 0; m < l; ++m) keep = keep && ci[m] != sj;
                    if (keep)
                        for (int m = l + 1; m < k; ++m)
                            if (ci[m] == sj) x += cv[m];
                }
                const uint32_t xb = __float_as_uint(x);
                const uint32_t ob = !keep ? kRecSkip : (x != x ? 0x7fc00000u : xb);
                reinterpret_cast<uint32_t *>(p)[l0 + j] = ob;
            }
            *reinterpret_cast<uint32_t *>(p + 4 * k + l0) = w;
        }
        __syncthreads();
    }
}

// EMIT (maxk_spgemm_forward_sel, k <= KG so one pass over l): every lane stores its edge's
// selector byte to esel[e * k + l] -- a wave step's G edges x k bytes are one contiguous run.
// The stores go one batch late, right after the next batch's column loads and before that
// batch's waits: on gfx950 stores count in vmcnt with the loads, so a store issued right after
// its own batch would make the next wait for loads wait for the store too, and one held past
// the next record loads keeps its bytes live through the batch's peak register use.  They are
// non-temporal (the stream must not push the record lines out of L2), and the pending bytes sit
// four to a register with the batch position kept wave-uniform.
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KG, int U, bool WIDE, bool EMIT = false>
struct EdgeWalker {
    static constexpr int G = kWave / KG;  // edges per wave step

    struct Pending {
        uint32_t b[(U + 3) / 4];
        int pos = -1;  // the pending batch's first edge offset (-1: none yet)
        __device__ __forceinline__ void keep(int u, int sel) {
            const uint32_t x = ((uint32_t)sel & 0xffu) << (8 * (u % 4));
            b[u / 4] = u % 4 == 0 ? x : (b[u / 4] | x);
        }
        // step u of the pending batch is edge offset pos + u * ustride + lane_off (in the
        // segment), stored when it is below lim and the lane's l below k
        __device__ __forceinline__ void flush(__amdgpu_buffer_rsrc_t ers, int ustride, int lane_off,
                                              int lim, int k, int l) const {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = pos + u * ustride + lane_off;
                const int off = pos >= 0 && e < lim && l < k ? e * k + l : (int)0x80000000;
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(b[u / 4] >> (8 * (u % 4))), ers,
                                                     off, 0, MAXK_T_AUX);
            }
        }
    };

    // Short-row batch: group g (KG lanes) walks row g's edges [sb_g, se_g) alone, U at a
    // time, into its own copy acc_g; the rows are consecutive, so their edges are one
    // contiguous range [e0, e_end) and one descriptor covers every group.  Edges past a
    // group's row (the next row's, or past e_end: 0) go to the trash column with weight 0.
    // esel (EMIT): each edge's selector bytes are stored to esel[e * k + l] on the way.
    __device__ __forceinline__ static void run_rows(float *acc_g, const int32_t *__restrict__ col_idx,
                                                    const float *__restrict__ edge_val,
                                                    const uint8_t *__restrict__ rec, int RS,
                                                    int e0, int e_end, int sb_g, int len_g,
                                                    int n_it, int k, int trash, int lane,
                                                    uint8_t *__restrict__ esel) {
        const int l0 = lane % KG;
        const int n = e_end - e0;  // wave-uniform
        const auto crs = wave_buffer(col_idx + e0, (uint32_t)n * 4u);
        const auto vrs = wave_buffer(edge_val + e0, (uint32_t)n * 4u);
        const auto rrs = wave_buffer(rec, 0xffffffffu);
        const int lo = (sb_g - e0) * 4;
        const auto ers = wave_buffer(EMIT ? esel + (size_t)(uint32_t)e0 * k : nullptr,
                                     EMIT ? (uint32_t)n * (uint32_t)k : 0u);
        // EMIT: group g's edge j (its row's j-th) sits at offset sb_g - e0 + j of the range;
        // stored right away (a short-row batch is one or two iterations: nothing to lag)
        const int g_off = sb_g - e0;
        for (int it = 0; it < n_it; ++it) {
            int c[U];
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                c[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, lo + (it * U + u) * 4, 0, 0);
                w[u] = __uint_as_float(
                    __builtin_amdgcn_raw_buffer_load_b32(vrs, lo + (it * U + u) * 4, 0, 0));
            }
            for (int lb = 0; lb < k; lb += KG) {
                const int l = lb + l0;
                const bool lok = l < k;
                const uint32_t lc = (uint32_t)(lok ? l : k - 1);
                const uint32_t vo = 4u * lc, so = 4u * (uint32_t)k + 2u * lc;
                float v[U];
                int s[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t ro = __umul24((uint32_t)c[u], (uint32_t)RS);
                    v[u] = __uint_as_float(
                        __builtin_amdgcn_raw_buffer_load_b32(rrs, (int)(ro + vo), 0, 0));
                    s[u] = __builtin_amdgcn_raw_buffer_load_b16(rrs, (int)(ro + so), 0, 0);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool live = lok && it * U + u < len_g;
                    float *a = &acc_g[live ? min(s[u], trash) : trash];
                    *a = __builtin_fmaf(w[u], v[u], *a);  // one rounding, in every variant
                    if constexpr (EMIT)
                        __builtin_amdgcn_raw_buffer_store_b8(
                            (uint8_t)s[u], ers, live ? (g_off + it * U + u) * k + l : (int)0x80000000,
                            0, MAXK_T_AUX);
                }
            }
        }
    }

    // acc_g[sel] += val[e] * value over e in [sb, se), sb < se.  acc_g is this
    // lane's group copy.  Padding lanes (l >= k) and edges past se write to the trash
    // column: two lanes of one group must never hit the same live address in one
    // ds_write, and an idle lane's product (weight 0 times any value) must not reach a
    // live column.
    // Default: every load goes through a wave-uniform buffer descriptor with 32-bit
    // offsets (wave_buffer, common.h): col_idx / edge_val over [sb, se) (past se they
    // return 0: column 0, weight 0, so nothing is clamped), the record table at
    // c*RS + 4l (values) and c*RS + 4k + 2l (selectors), one 24-bit multiply-add each.
    // WIDE (tables past 2^24 columns or 4 GiB): 64-bit addresses, clamped loads.
    __device__ __forceinline__ static void run(float *acc_g, const int32_t *__restrict__ col_idx,
                                               const float *__restrict__ edge_val,
                                               const uint8_t *__restrict__ rec, int RS, int sb,
                                               int se, int k, int trash, int lane,
                                               uint8_t *__restrict__ esel) {
        const int grp = lane / KG;
        const int l0 = lane % KG;
        if constexpr (!WIDE) {
            const int n = se - sb;  // wave-uniform, <= chunk
            const auto crs = wave_buffer(col_idx + sb, (uint32_t)n * 4u);
            const auto vrs = wave_buffer(edge_val + sb, (uint32_t)n * 4u);
            const auto rrs = wave_buffer(rec, 0xffffffffu);  // offsets < num_cols * RS < 2^32
            // EMIT: the segment's edge-selector rows
            const auto ers = wave_buffer(EMIT ? esel + (size_t)(uint32_t)sb * k : nullptr,
                                         EMIT ? (uint32_t)n * (uint32_t)k : 0u);
            Pending pend;
            for (int base = 0; base < n; base += G * U) {
                int c[U];
                float w[U];
                const int lo = (base + grp) * 4;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    c[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, lo + u * G * 4, 0, 0);
                    w[u] = __uint_as_float(
                        __builtin_amdgcn_raw_buffer_load_b32(vrs, lo + u * G * 4, 0, 0));
                }
                if constexpr (EMIT) {
                    pend.flush(ers, G, grp, n, k, l0);
                    __builtin_amdgcn_sched_barrier(0);  // the stores stay ahead of the record loads
                }
                for (int lb = 0; lb < k; lb += KG) {  // one pass unless k > 64
                    const int l = lb + l0;
                    const bool lok = l < k;
                    const uint32_t lc = (uint32_t)(lok ? l : k - 1);
                    const uint32_t vo = 4u * lc, so = 4u * (uint32_t)k + 2u * lc;
                    float v[U];
                    int s[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t ro = __umul24((uint32_t)c[u], (uint32_t)RS);
                        v[u] = __uint_as_float(
                            __builtin_amdgcn_raw_buffer_load_b32(rrs, (int)(ro + vo), 0, 0));
                        s[u] = __builtin_amdgcn_raw_buffer_load_b16(rrs, (int)(ro + so), 0, 0);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const bool live = lok && base + u * G + grp < n;
                        float *a = &acc_g[live ? min(s[u], trash) : trash];
                        *a = __builtin_fmaf(w[u], v[u], *a);  // one rounding, in every variant
                        if constexpr (EMIT) pend.keep(u, s[u]);
                    }
                    if constexpr (EMIT) pend.pos = base;
                }
            }
            if constexpr (EMIT) pend.flush(ers, G, grp, n, k, l0);
        } else {
            const int last = se - 1;
            for (int base = sb; base < se; base += G * U) {
                int c[U];
                float w[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = base + u * G + grp;
                    const int ec = e < se ? e : last;
                    c[u] = col_idx[ec];
                    const float wv = edge_val[ec];
                    w[u] = e < se ? wv : 0.f;
                }
                for (int lb = 0; lb < k; lb += KG) {
                    const int l = lb + l0;
                    const bool lok = l < k;
                    const int lc = lok ? l : k - 1;
                    float v[U];
                    int s[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint8_t *p = rec + (size_t)(uint32_t)c[u] * RS;
                        v[u] = reinterpret_cast<const float *>(p)[lc];
                        s[u] = reinterpret_cast<const uint16_t *>(p + 4 * k)[lc];
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        float *a = &acc_g[lok ? min(s[u], trash) : trash];
                        *a = __builtin_fmaf(w[u], v[u], *a);
                    }
                }
            }
        }
    }
};

// dst[0:D] = (sum_g acc[g][0:D]) / div ; acc = 0.  One wave; copies of stride DS.
// add (maxk_spgemm_forward_accumulate): dst[0:D] += instead.
template <int NC>
__device__ __forceinline__ void flush_row(float *acc, int DS, float *__restrict__ dst, int D,
                                          float div, bool scale, int lane, bool add = false,
                                          bool nt = false) {
    wave_lds_fence();
    if ((D & 3) == 0) {
        for (int j = lane * 4; j < D; j += kWave * 4) {
            float4 a = *reinterpret_cast<float4 *>(&acc[j]);
            *reinterpret_cast<float4 *>(&acc[j]) = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int g = 1; g < NC; ++g) {
                float4 *pg = reinterpret_cast<float4 *>(&acc[g * DS + j]);
                const float4 b = *pg;
                a.x += b.x;
                a.y += b.y;
                a.z += b.z;
                a.w += b.w;
                *pg = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            if (scale) {
                a.x = a.x / div;
                a.y = a.y / div;
                a.z = a.z / div;
                a.w = a.w / div;
            }
            if (add) {
                const float4 o = *reinterpret_cast<const float4 *>(&dst[j]);
                a.x += o.x;
                a.y += o.y;
                a.z += o.z;
                a.w += o.w;
            }
            if (nt)  // output rows streamed past the caches (the record lines stay)
                __builtin_nontemporal_store(
                    __builtin_bit_cast(f32x4, a), reinterpret_cast<f32x4 *>(&dst[j]));
            else
                *reinterpret_cast<float4 *>(&dst[j]) = a;
        }
    } else {
        for (int j = lane; j < D; j += kWave) {
            float a = 0.f;
#pragma unroll
            for (int g = 0; g < NC; ++g) {
                a += acc[g * DS + j];
                acc[g * DS + j] = 0.f;
            }
            dst[j] = (scale ? a / div : a) + (add ? dst[j] : 0.f);
        }
    }
    wave_lds_fence();
}

// Records of the streaming walker: cbsr_pack*_kernel's, value at c*RS + 4l, u16 selector at
// c*RS + 4k + 2l (a folded duplicate or a selector >= D is stored as 0x100 | s, so
// min(s, trash) is the LDS column).
struct PackedSrc {
    __amdgpu_buffer_rsrc_t rrs;
    uint32_t vo, so, RS;
    __device__ __forceinline__ void load(int c, float &v, int &s) const {
        const uint32_t ro = __umul24((uint32_t)c, RS);
        v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, (int)(ro + vo), 0, 0));
        s = __builtin_amdgcn_raw_buffer_load_b16(rrs, (int)(ro + so), 0, 0);
    }
    __device__ __forceinline__ int col(int s, int D, int trash) const {
        (void)D;
        return min(s, trash);
    }
};
// Transport records (cbsr_records_kernel): value at c*5k + 4l, selector byte at c*5k + 4k + l;
// kRecSkip values and selectors >= D go to the trash column.
struct RecordSrc {
    __amdgpu_buffer_rsrc_t rrs;
    uint32_t vo, so, RS;
    __device__ __forceinline__ void load(int c, float &v, int &s) const {
        const uint32_t ro = __umul24((uint32_t)c, RS);
        const uint32_t vb = __builtin_amdgcn_raw_buffer_load_b32(rrs, (int)(ro + vo), 0, 0);
        const int sb = __builtin_amdgcn_raw_buffer_load_b8(rrs, (int)(ro + so), 0, 0);
        v = __uint_as_float(vb);
        s = vb == kRecSkip ? 0x100 : sb;  // 0x100 >= any D: the trash column
    }
    __device__ __forceinline__ int col(int s, int D, int trash) const {
        return s < D ? s : trash;
    }
};

// EdgeWalker::run's single-pass buffer path (KG >= k, no selector stream) over a source: the
// transport-record walks of hub-row pieces and of rows longer than the streaming groups take.
template <int KG, int U, class Src>
__device__ __forceinline__ void walk_src(float *acc_g, const int32_t *__restrict__ col_idx,
                                         const float *__restrict__ edge_val, const Src &src,
                                         int sb, int se, int D, int trash, bool lok, int lane) {
    constexpr int G = kWave / KG;
    const int grp = lane / KG;
    const int n = se - sb;  // wave-uniform
    const auto crs = wave_buffer(col_idx + sb, (uint32_t)n * 4u);
    const auto vrs = wave_buffer(edge_val + sb, (uint32_t)n * 4u);
    for (int base = 0; base < n; base += G * U) {
        int c[U];
        float w[U];
        const int lo = (base + grp) * 4;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, lo + u * G * 4, 0, 0);
            w[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vrs, lo + u * G * 4, 0, 0));
        }
        float v[U];
        int s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) src.load(c[u], v[u], s[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool live = lok && base + u * G + grp < n;
            float *a = &acc_g[live ? src.col(s[u], D, trash) : trash];
            *a = __builtin_fmaf(w[u], v[u], *a);  // one rounding, in every variant
        }
    }
}
// four consecutive copy columns, zeroed as they are read
__device__ __forceinline__ float4 acc_take4(float *a) {
    const float4 x = *reinterpret_cast<float4 *>(a);
    *reinterpret_cast<float4 *>(a) = make_float4(0.f, 0.f, 0.f, 0.f);
    return x;
}
// dst[j..j+4) = x / div (+ dst), 16-B store (nt: past the caches)
__device__ __forceinline__ void store_out4(float *dst, float4 a, bool scale, float div, bool add,
                                           bool nt) {
    if (scale) {
        a.x = a.x / div;
        a.y = a.y / div;
        a.z = a.z / div;
        a.w = a.w / div;
    }
    if (add) {
        const float4 o = *reinterpret_cast<const float4 *>(dst);
        a.x += o.x;
        a.y += o.y;
        a.z += o.z;
        a.w += o.w;
    }
    if (nt)
        __builtin_nontemporal_store(__builtin_bit_cast(f32x4, a), reinterpret_cast<f32x4 *>(dst));
    else
        *reinterpret_cast<float4 *>(dst) = a;
}

// Streaming rows (r05; sparse graphs: KG >= 16, so a lane group covers a D = 64 row with one
// 16-B access per lane).  Each lane group walks whole rows on its own, U edges per step, and
// takes the item's next row the step its current one ends, so the wave keeps NC rows in flight
// with no batch boundary; the next step's columns and weights (and a new row's divisor) are
// loaded while this step's records are in flight.  A row then costs about one dependent round
// of loads per U edges, against two in the batched path (columns, then records), which on a
// small sparse graph -- one round of waves, each a chain of such rounds -- is the whole time.
// A group flushes its finished row from its own LDS copy (16-B stores).  Rows are taken in
// order while the next one is owned by the item (token < d1) and has at most lmax edges (the
// callers pass at most `chunk`: a longer row is split over items, and its pieces past d1 belong
// to the items holding them);
// returns the first row not taken (the caller walks a longer one with the whole wave).  Copies
// are zero on entry and on return.  D % 4 == 0.
template <int KG, int U, class Src>
__device__ __forceinline__ int stream_rows(float *acc, int DS, int r,
                                           const int32_t *__restrict__ row_ptr, int num_rows,
                                           int64_t d1, const int32_t *__restrict__ col_idx,
                                           const float *__restrict__ edge_val, const Src &src,
                                           const float *__restrict__ row_div,
                                           float *__restrict__ out, int D, int k, int trash,
                                           int lane, int flags, int lmax, int64_t num_e) {
    constexpr int NC = kWave / KG;
    const int g = lane / KG, l0 = lane % KG;
    float *acc_g = acc + g * DS;
    const bool lok = l0 < k;
    const bool add = flags & 1, nt = flags & 2;
    // row_ptr window: rows [wb, wb + 64), one per lane
    int wb = r;
    int rpw = row_ptr[wb + lane <= num_rows ? wb + lane : num_rows];
    const int ebase = __builtin_amdgcn_readfirstlane(rpw);  // = row_ptr[r]
    const int64_t span = (num_e - ebase) * 4;
    const auto crs = wave_buffer(col_idx + ebase, (uint32_t)(span < 0xffffffffLL ? span : 0xffffffffLL));
    const auto vrs = wave_buffer(edge_val + ebase, (uint32_t)(span < 0xffffffffLL ? span : 0xffffffffLL));
    int next = r;       // the next row to hand out (wave-uniform)
    bool stop = false;  // the next row is not the item's or is too long (wave-uniform)
    int row = -1, e = 0, ee = 0;  // this group's row and its edge range [e, ee)
    float div = 1.f;
    auto assign = [&]() {
        const uint64_t idle = __ballot(row < 0);
#pragma unroll
        for (int gi = 0; gi < NC; ++gi) {
            if (stop || !((idle >> (gi * KG)) & 1ull)) continue;
            if (next + 1 >= wb + kWave) {  // slide the window (wave-uniform)
                wb = next;
                rpw = row_ptr[wb + lane <= num_rows ? wb + lane : num_rows];
            }
            const int a = __builtin_amdgcn_readlane(rpw, next - wb);
            const int b = __builtin_amdgcn_readlane(rpw, next + 1 - wb);
            if (next < num_rows && (int64_t)next + a < d1 && b - a <= lmax) {
                if (g == gi) {
                    row = next;
                    e = a;
                    ee = b;
                    div = row_div ? row_div[next] : 1.f;  // arrives long before the flush
                }
                ++next;
            } else {
                stop = true;
            }
        }
    };
    auto load_cw = [&](int (&c)[U], float (&w)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int off = row >= 0 && e + u < ee ? (e + u - ebase) * 4 : (int)0x80000000;
            c[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, off, 0, 0);
            w[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vrs, off, 0, 0));
        }
    };
    assign();
    int c[U];
    float w[U];
    load_cw(c, w);
    float wn[U];
    while (__ballot(row >= 0)) {
        float v[U];
        int s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) src.load(c[u], v[u], s[u]);
        // this step's rows; then the next step's state and its columns / weights in flight
        const int crow = row, ce = e, cee = ee;
        const float cdiv = div;
        const bool fin = crow >= 0 && ce + U >= cee;
        if (fin) row = -1;
        e = ce + U;
        assign();
        load_cw(c, wn);  // c is dead once the record offsets are formed
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool live = lok && crow >= 0 && ce + u < cee;
            float *a = &acc_g[live ? src.col(s[u], D, trash) : trash];
            *a = __builtin_fmaf(w[u], v[u], *a);  // one rounding, as in the batched walkers
        }
        if (fin) {  // group-uniform: this group's row is complete in its copy
            wave_lds_fence();
            float *dst = out + (int64_t)crow * D;
            for (int j = l0 * 4; j < D; j += KG * 4)
                store_out4(dst + j, acc_take4(acc_g + j), row_div != nullptr, cdiv, add, nt);
            wave_lds_fence();
        }
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = wn[u];
    }
    return next;
}

template <int KG, int U, bool WIDE, bool EMIT, bool STREAM = false>
__global__ __launch_bounds__(kBlock, EMIT ? MAXK_FWD_EMIT_WAVES : MAXK_FWD_WAVES) void spgemm_fwd_kernel(
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col_idx,
    const float *__restrict__ edge_val, const uint8_t *__restrict__ rec, int RS,
    const float *__restrict__ row_div, float *__restrict__ out, float *__restrict__ slab,
    int32_t *__restrict__ slab_row, int num_rows, int64_t num_e, int D, int DS, int k,
    int chunk, int n_items, int accumulate, uint8_t *__restrict__ esel,
    const uint8_t *__restrict__ trec = nullptr) {
    // accumulate: bit 0 adds onto out (maxk_spgemm_forward_accumulate), bit 1 stores the output
    // rows non-temporally.  STREAM with trec: the caller's transport records (RecordSrc, stride
    // 5k) instead of the packed ones
    constexpr int NC = kWave / KG;  // LDS copies per wave (one per edge group)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    // MAXK_FWD_XCD: XCD x runs the x-th eighth of the items (contiguous rows), so a graph
    // whose vertex order keeps neighbours close finds their records in that XCD's L2
    const int blk = MAXK_FWD_XCD ? xcd_contiguous_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int item = blk * kWavesPerBlock + wid;
    if (item >= n_items) return;  // whole wave; no workgroup barrier below
    float *acc = lds + (size_t)wid * NC * DS;
    for (int j = lane * 4; j < NC * DS; j += kWave * 4)
        *reinterpret_cast<float4 *>(&acc[j]) = make_float4(0.f, 0.f, 0.f, 0.f);
    float *acc_g = acc + (lane / KG) * DS;
    const bool lok_s = lane % KG < k;
    // built where it is used (a descriptor kept live across the kernel goes to scratch)
    auto rec_src = [&]() {
        const uint32_t lc = (uint32_t)(lok_s ? lane % KG : k - 1);
        return RecordSrc{wave_buffer(trec, 0xffffffffu), 4u * lc, 4u * (uint32_t)k + lc,
                         5u * (uint32_t)k};
    };
    const bool tr = (STREAM || MAXK_FWD_RECORDS_DEEP) && !WIDE && !EMIT && trec != nullptr;

    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int r = wave_first_row_token(row_ptr, num_rows, d0);

    // Continuation of row r-1 (its token precedes d0): edges e with e + r in [d0, d1).
    // A row of at most `chunk` edges is never split: the item holding its row token walks all
    // of it, past d1, so only longer (hub) rows leave a continuation and a slab for the fixup
    // (Reddit-sized k = 16 forward 1.596 -> 1.585 ms, ogbn-products-sized k = 8 3.237 -> 3.19
    // ms, proteins unchanged; profiles/r04/tune/fwd_snap_rows_ab.txt).  An item then walks at
    // most 2 * chunk tokens.
    int cont = -1;
    if (r > 0) {
        const int64_t sb = d0 - r;
        int64_t se = (int64_t)row_ptr[r];
        if (d1 - r < se) se = d1 - r;
        const bool whole = (int64_t)row_ptr[r] - row_ptr[r - 1] <= chunk;
        if (sb < se && !whole) {
            const float div = row_div ? row_div[r - 1] : 1.f;  // loaded before the walk
            wave_lds_fence();
            if (tr)
                walk_src<KG, U>(acc_g, col_idx, edge_val, rec_src(), (int)sb, (int)se, D, DS - 1,
                                lok_s, lane);
            else
                EdgeWalker<KG, U, WIDE, EMIT>::run(acc_g, col_idx, edge_val, rec, RS, (int)sb,
                                                   (int)se, k, DS - 1, lane, esel);
            flush_row<NC>(acc, DS, slab + (int64_t)item * D, D, div, row_div != nullptr, lane);
            cont = r - 1;
        }
    }
    if (lane == 0) slab_row[item] = cont;

    // Rows whose token lies in [d0, d1): this item owns them.  row_ptr of 64 consecutive rows
    // sits one per lane (window from row wb), for the short-row test below.
    int wb = r, rpw = 0;
    constexpr bool BATCH = NC > 1 && !WIDE && !EMIT && !STREAM && MAXK_FWD_SHORT > 0;
    if constexpr (BATCH)
        rpw = row_ptr[r + lane <= num_rows ? r + lane : num_rows];
    while (r < num_rows) {
        int64_t rb = row_ptr[r];
        if (rb + r >= d1) break;
        if constexpr (STREAM) {
            // every row of at most MAXK_FWD_STREAM edges by the streaming lane groups; a longer
            // one (or the item's end) stops them, and the wave walks it below
            if (tr) {
                r = stream_rows<KG, U>(acc, DS, r, row_ptr, num_rows, d1, col_idx, edge_val,
                                       rec_src(), row_div, out, D, k, DS - 1, lane, accumulate,
                                       min(MAXK_FWD_STREAM, chunk), num_e);
            } else {
                const uint32_t lc = (uint32_t)(lok_s ? lane % KG : k - 1);
                const PackedSrc src{wave_buffer(rec, 0xffffffffu), 4u * lc,
                                    4u * (uint32_t)k + 2u * lc, (uint32_t)RS};
                r = stream_rows<KG, U>(acc, DS, r, row_ptr, num_rows, d1, col_idx, edge_val, src,
                                       row_div, out, D, k, DS - 1, lane, accumulate,
                                       min(MAXK_FWD_STREAM, chunk), num_e);
            }
            if (r >= num_rows) break;
            rb = row_ptr[r];
            if (rb + r >= d1) break;
        }
        if (BATCH && !tr) {
            // Short-row batch: up to NC consecutive rows, each wholly inside the item and at
            // most MAXK_FWD_SHORT edges long, one per lane group, so a wave keeps NC rows'
            // loads in flight instead of walking one short row at a time (Flickr: avg
            // degree 11).  The test reads the row_ptr window (no load per row): long rows
            // pay only a few shuffles for it.
            if (r + NC >= wb + kWave) {  // slide the window
                wb = r;
                rpw = row_ptr[r + lane <= num_rows ? r + lane : num_rows];
            }
            const int rq = r + lane;
            const int rpj = __shfl(rpw, (r - wb + lane) & (kWave - 1));
            const int rpn = __shfl_down(rpj, 1);
            const bool okj = lane < NC && rq < num_rows && (int64_t)rq + rpn < d1 &&
                             rpn - rpj <= MAXK_FWD_SHORT;
            const uint64_t bal = __ballot(okj);
            const int m = __builtin_ctzll(~bal);  // leading rows that qualify
            if (m >= 2) {
                const int g = lane / KG;
                const int sb_g = __shfl(rpj, g < m ? g : 0);
                const int len_g = g < m ? __shfl(rpn, g) - sb_g : 0;
                const int e0 = __shfl(rpj, 0), e_end = __shfl(rpj, m);
                int maxlen = 0;
                for (int j = 0; j < m; ++j) {
                    const int lj = __shfl(rpn, j) - __shfl(rpj, j);
                    maxlen = lj > maxlen ? lj : maxlen;
                }
                // the batch's divisors, one per lane, loaded before the walk (not one
                // dependent scalar load per row after it)
                const float divq = row_div && lane < m ? row_div[r + lane] : 1.f;
                wave_lds_fence();
                EdgeWalker<KG, U, WIDE, EMIT>::run_rows(acc_g, col_idx, edge_val, rec, RS, e0,
                                                        e_end, sb_g, len_g, (maxlen + U - 1) / U,
                                                        k, DS - 1, lane, esel);
                for (int j = 0; j < m; ++j) {
                    const float div = __shfl(divq, j);
                    flush_row<1>(acc + j * DS, DS, out + (int64_t)(r + j) * D, D, div,
                                 row_div != nullptr, lane, accumulate & 1, accumulate & 2);
                }
                r += m;
                continue;
            }
        }
        int64_t se = (int64_t)row_ptr[r + 1];
        if (d1 - r - 1 < se && se - rb > chunk) se = d1 - r - 1;  // a hub row: split
        const float div = row_div ? row_div[r] : 1.f;  // loaded before the walk
        wave_lds_fence();
        if (rb < se && tr)
            walk_src<KG, U>(acc_g, col_idx, edge_val, rec_src(), (int)rb, (int)se, D, DS - 1,
                            lok_s, lane);
        else if (rb < se)
            EdgeWalker<KG, U, WIDE, EMIT>::run(acc_g, col_idx, edge_val, rec, RS, (int)rb, (int)se,
                                               k, DS - 1, lane, esel);
        flush_row<NC>(acc, DS, out + (int64_t)r * D, D, div, row_div != nullptr, lane,
                      accumulate & 1, accumulate & 2);
        ++r;
    }
}

// Waves of the plain forward one CU holds at once: 7 per SIMD by VGPRs (65-69 VGPRs, the
// kernel-resource-usage remarks), 4 for the deep-batch kernel (~100), 5 for the streaming-rows
// kernel (~80-87), fewer when the LDS copies (NC rows of DS floats per wave) fill the CU's
// 160 KB first.
int fwd_resident_waves(int kg, int DS, int per_simd) {
    const int by_vgpr = per_simd * 4;
    const size_t per_block = (size_t)kWavesPerBlock * (kWave / kg) * DS * sizeof(float);
    const int by_lds = (int)(kPullLdsBytes / per_block) * kWavesPerBlock;
    return by_lds < by_vgpr ? by_lds : by_vgpr;
}

// Long rows (a dense graph, e.g. a Reddit-sized graph's vertex-range shard: 14.4M tokens at
// N = 8, rows of ~490 edges): items of at least two average rows (at most 1024 tokens), so most
// rows are walked whole instead of split into slabs (that shard's forward at 256 / 512 / 1024 /
// 2048 tokens: 0.256 / 0.237 / 0.237 / 0.254 ms; the N = 4 shard at 438 / 1024: 0.449 / 0.440;
// profiles/r05/tune/fwd_chunk_shards/) -- while the items still fill every wave slot (a small
// dense graph keeps the one-round sizing below)
int64_t fwd_long_rows(int64_t num_rows, int64_t num_e, int64_t c, int resident) {
    if (num_rows <= 0 || num_e < kFwdSparseDegree * num_rows) return c;
    const int64_t two_rows = (2 * ceil_div(num_e, num_rows) + 63) / 64 * 64;
    const int64_t want = two_rows < 1024 ? two_rows : 1024;
    if (c >= want || (num_rows + num_e) / want < device_cus() * resident) return c;
    return want;
}

int fwd_chunk(int64_t num_rows, int64_t num_e, int32_t chunk, int resident) {
    if (chunk > 0) return chunk;
    // ~8 waves of work per resident wave slot on the device's CUs (256 on MI355X), within
    // [256, 2048] tokens
    const int64_t total = num_rows + num_e;
    const int64_t cus = device_cus();
    int64_t c = ceil_div(total, cus * 32 * 8);
    if (c >= 256) return (int)fwd_long_rows(num_rows, num_e, c > 2048 ? 2048 : c, resident);
    // A smaller graph has fewer items than wave slots at 256 tokens: size the items so all of
    // them are resident in one round (90 % of the slots, for uneven block placement), since each
    // wave is a chain of dependent gathers and a second round costs a whole item's latency.
    // Flickr-sized (1.08M tokens, 7168 slots): 151 tokens would fill every slot; the forward at
    // 144 / 160 / 176 / 192 / 256 tokens takes 0.0527 / 0.049 / 0.051 / 0.053 / 0.0585 ms
    // (profiles/r04/tune/flickr_chunk_sweep.txt).
    c = ceil_div(total * 10, cus * resident * 9);
    return (int)fwd_long_rows(num_rows, num_e, c < 64 ? 64 : (c > 256 ? 256 : c), resident);
}

// LDS row stride per copy: D padded to 16 B, plus one 16-B group holding the
// trash column (index DS-1, never read by the flush).
inline int copy_stride(int D) { return ((D + 3) / 4) * 4 + 4; }

struct FwdLayout {
    int chunk, n_items, RS, DS, kg;
    // the deep-batch kernel runs: a dense graph (average degree >= kFwdSparseDegree), 32-bit
    // record offsets, no selector stream written (launch_fwd)
    bool deep;
    // the streaming-rows kernel runs (stream_rows): a sparse graph, 32-bit record offsets,
    // no selector stream written, D % 4 == 0, k <= 64 (a lane group holds every l)
    bool stream;
    size_t rec_off, rec_bytes, slab_off, slab_bytes, row_off, total;
};

// emit: the launch writes the edge-selector stream (the U-step kernel, whatever the graph), so
// small graphs' items are sized for that kernel's occupancy
FwdLayout fwd_layout(int64_t num_rows, int64_t num_cols, int64_t num_e, int D, int k, int chunk,
                     bool emit = false) {
    FwdLayout L{};
    L.RS = record_stride(k, num_cols);
    L.DS = copy_stride(D);
    L.kg = fwd_lanes_per_edge(k, num_rows, num_e);
    const bool narrow = num_cols < (1 << 24) && (uint64_t)num_cols * (uint64_t)L.RS < (1ull << 32);
    L.deep = !emit && num_e >= kFwdSparseDegree * num_rows && narrow;
    L.stream = MAXK_FWD_STREAM > 0 && !emit && narrow && L.kg >= 16 && L.kg <= 32 &&
               D % 4 == 0 && num_e < kFwdSparseDegree * num_rows;
    L.chunk = fwd_chunk(num_rows, num_e, chunk,
                        fwd_resident_waves(L.kg, L.DS, L.deep ? 4 : L.stream ? 5 : 7));
    const int64_t n = ceil_div(num_rows + num_e, L.chunk);
    L.n_items = (int)(n > 0 ? n : 1);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    L.rec_off = 0;
    L.rec_bytes = al((size_t)num_cols * L.RS);
    L.slab_off = L.rec_off + L.rec_bytes;
    L.slab_bytes = al((size_t)L.n_items * D * sizeof(float));
    L.row_off = L.slab_off + L.slab_bytes;
    L.total = L.row_off + al((size_t)L.n_items * sizeof(int32_t));
    return L;
}

template <int KG>
void launch_fwd(const FwdLayout &L, hipStream_t s, const int32_t *row_ptr, const int32_t *col_idx,
                const float *edge_val, const uint8_t *rec, const float *row_div, float *out,
                float *slab, int32_t *slab_row, int num_rows, int64_t num_e, int D, int k,
                int accumulate, uint8_t *esel, const uint8_t *trec = nullptr) {
    constexpr int U = MAXK_FWD_U;
    constexpr int NC = kWave / KG;
    const size_t lds = (size_t)kWavesPerBlock * NC * L.DS * sizeof(float);
    const int64_t blocks = ceil_div(L.n_items, kWavesPerBlock);
    const dim3 grid((unsigned)(MAXK_FWD_XCD ? xcd_grid(blocks) : blocks));
    // 32-bit record offsets need c < 2^24 (24-bit multiply) and the table under 4 GiB
    const int64_t num_cols = (int64_t)(L.rec_bytes / L.RS);
    // esel needs the buffer-descriptor path (the caller checks fwd_can_emit)
    if (esel)
        hipLaunchKernelGGL((spgemm_fwd_kernel<KG, U, false, true>), grid, dim3(kBlock), lds, s,
                           row_ptr, col_idx, edge_val, rec, L.RS, row_div, out, slab, slab_row,
                           num_rows, num_e, D, L.DS, k, L.chunk, L.n_items, accumulate, esel);
    else if (L.stream) {
        if constexpr (KG >= 16)
            hipLaunchKernelGGL((spgemm_fwd_kernel<KG, U, false, false, true>), grid, dim3(kBlock),
                               lds, s, row_ptr, col_idx, edge_val, rec, L.RS, row_div, out, slab,
                               slab_row, num_rows, num_e, D, L.DS, k, L.chunk, L.n_items,
                               accumulate, nullptr, trec);
    } else if (L.deep)
        // dense graphs: 16 wave steps of loads per batch (Reddit-sized k = 16 forward 1.613 ->
        // 1.594 ms, k = 32 / 64 and ogbn-proteins 0.3-0.8 % faster; on the sparse products
        // graph, whose rows hold ~50 edges, 16 steps cost occupancy for nothing: 3.23 -> 4.19
        // ms at k = 8; profiles/r04/tune/fwd_batch_depth_ab*.txt)
        hipLaunchKernelGGL((spgemm_fwd_kernel<KG, 2 * U, false, false>), grid, dim3(kBlock), lds,
                           s, row_ptr, col_idx, edge_val, rec, L.RS, row_div, out, slab, slab_row,
                           num_rows, num_e, D, L.DS, k, L.chunk, L.n_items, accumulate, nullptr,
                           trec);
    else if (num_cols < (1 << 24) && L.rec_bytes < (1ull << 32))
        hipLaunchKernelGGL((spgemm_fwd_kernel<KG, U, false, false>), grid, dim3(kBlock), lds, s,
                           row_ptr, col_idx, edge_val, rec, L.RS, row_div, out, slab, slab_row,
                           num_rows, num_e, D, L.DS, k, L.chunk, L.n_items, accumulate, nullptr);
    else
        hipLaunchKernelGGL((spgemm_fwd_kernel<KG, U, true, false>), grid, dim3(kBlock), lds, s,
                           row_ptr, col_idx, edge_val, rec, L.RS, row_div, out, slab, slab_row,
                           num_rows, num_e, D, L.DS, k, L.chunk, L.n_items, accumulate, nullptr);
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" size_t maxk_spgemm_forward_workspace_size(int64_t num_rows, int64_t num_cols,
                                                     int64_t num_e, int32_t dim_origin,
                                                     int32_t dim_k, int32_t chunk_edges) {
    if (num_rows < 0 || num_cols < 0 || num_e < 0 || dim_origin <= 0 || dim_k <= 0) return 0;
    // one workspace serves the plain and the stream-writing launch (their item sizes differ)
    const size_t a = fwd_layout(num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges).total;
    const size_t b =
        fwd_layout(num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges, true).total;
    const size_t c = dense_route(dim_origin, dim_k)
                         ? dense_forward_workspace_size(num_rows, num_cols, num_e, dim_origin,
                                                        chunk_edges)
                         : 0;
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

namespace {
// the forward over transport records applies (maxk_records_ok): the streaming or (dense graphs,
// MAXK_FWD_RECORDS_DEEP) the deep-batch walker, one pass
// over l, records past one line in the packed form (6k > 128, where a 5k-byte stride costs no
// extra line per gather: 160 B at k = 32 spans two lines as the 256-B record does)
bool records_ok(const FwdLayout &L, int64_t num_cols, int k) {
    return (L.stream || (MAXK_FWD_RECORDS_DEEP && L.deep)) && k % 4 == 0 && 6 * k > 128 &&
           k <= L.kg && k <= 32 &&
           (uint64_t)num_cols * 5u * (uint64_t)k < (1ull << 32);
}

int forward_impl(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                 const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div, float *out,
                 int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin,
                 int32_t dim_k, int32_t chunk_edges, void *workspace, size_t workspace_bytes,
                 void *stream, int accumulate, uint8_t *esel = nullptr,
                 const uint8_t *trec = nullptr) {
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range: %lld",
                 (long long)num_rows);
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range: %lld", (long long)num_e);
    MAXK_REQUIRE(dim_origin >= 1 && dim_origin <= kMaxDim, "dim_origin must be in [1,256], got %d",
                 dim_origin);
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= dim_origin, "dim_k must be in [1,dim_origin], got %d",
                 dim_k);
    MAXK_REQUIRE(chunk_edges >= 0, "chunk_edges must be >= 0");
    MAXK_REQUIRE(num_cols * (int64_t)dim_k < (1LL << 31), "num_cols*k too large");
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && out, "row_ptr/out must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (col_idx && edge_val && ((cbsr_val && cbsr_idx) || trec)),
                 "CSR/CBSR pointers must not be NULL");
    MAXK_REQUIRE(num_e == 0 || num_cols > 0, "edges present but num_cols == 0");
    if (!esel && !trec && dense_route(dim_origin, dim_k) && ((uintptr_t)cbsr_val & 15) == 0 &&
        ((uintptr_t)cbsr_idx & 3) == 0 && ((uintptr_t)out & 15) == 0) {
        // k >= D / 2: dense rows carry no more bytes than the CBSR (dense_route.hip)
        MAXK_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-B aligned");
        return dense_forward(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out,
                             num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace,
                             workspace_bytes, as_stream(stream), accumulate);
    }
    const FwdLayout L =
        fwd_layout(num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges, esel != nullptr);
    MAXK_REQUIRE(workspace && workspace_bytes >= L.total,
                 "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    MAXK_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-B aligned");

    char *ws = reinterpret_cast<char *>(workspace);
    uint8_t *rec = reinterpret_cast<uint8_t *>(ws + L.rec_off);
    float *slab = reinterpret_cast<float *>(ws + L.slab_off);
    int32_t *slab_row = reinterpret_cast<int32_t *>(ws + L.row_off);
    hipStream_t s = as_stream(stream);
    const int D = dim_origin, k = dim_k;
    if (trec) {
        MAXK_REQUIRE(records_ok(L, num_cols, k), "transport records need the streaming forward "
                     "(a sparse graph), k %% 4 == 0 in [24, 32] and num_cols * 5k < 2^32");
    } else if (MAXK_FWD_RECORDS && !esel && num_cols > 0 && records_ok(L, num_cols, k) &&
               ((uintptr_t)cbsr_val & 3) == 0) {
        // the same walk over 5k-byte records packed here (they fit the record table): the
        // ogbn-products-sized graph at k = 32, forward 4.885 -> 4.813 ms, bitwise equal
        // (profiles/r05/tune/transport_records/)
        const int vpw = kPackBlock / (k / 4);
        const int64_t groups = ceil_div(num_cols, (int64_t)vpw);
        hipLaunchKernelGGL(cbsr_records_kernel,
                           dim3((unsigned)(groups < MAXK_PACK_GRID ? groups : MAXK_PACK_GRID)),
                           dim3(kPackBlock), 0, s, cbsr_val, cbsr_idx, rec, (int)num_cols, k, D);
        MAXK_LAUNCHED("cbsr_records_kernel");
        trec = rec;
    } else if (num_cols > 0 && MAXK_PACK4 && k % 4 == 0 && ((uintptr_t)cbsr_val & 15) == 0 &&
        ((uintptr_t)cbsr_idx & 3) == 0) {
        const int vpw = kPackBlock / (k / 4);
        const int64_t groups = ceil_div(num_cols, (int64_t)vpw);
        hipLaunchKernelGGL(cbsr_pack4_kernel,
                           dim3((unsigned)(groups < MAXK_PACK_GRID ? groups : MAXK_PACK_GRID)),
                           dim3(kPackBlock), 0,
                           s, cbsr_val, cbsr_idx, rec, (int)num_cols, k, L.RS, D, L.DS - 1);
        MAXK_LAUNCHED("cbsr_pack4_kernel");
    } else if (num_cols > 0) {
        const int vpw = k >= kPackBlock / kPackMaxV ? kPackBlock / k : kPackMaxV;
        const int64_t groups = ceil_div(num_cols, (int64_t)vpw);
        hipLaunchKernelGGL(cbsr_pack_kernel,
                           dim3((unsigned)(groups < MAXK_PACK_GRID ? groups : MAXK_PACK_GRID)),
                           dim3(kPackBlock), 0,
                           s, cbsr_val, cbsr_idx, rec, (int)num_cols, k, L.RS, D, L.DS - 1);
        MAXK_LAUNCHED("cbsr_pack_kernel");
    }
    const int nr = (int)num_rows;
    // Output rows past the Infinity Cache's size are stored non-temporally, so they do not push
    // the record lines (the forward's random reads) out: ogbn-products k=8 forward emitting the
    // selector stream 3.62 -> 3.28 ms, k=16 3.79 -> 3.61, plain forwards and Reddit (238 MB of
    // output) unchanged (profiles/r03/tune/fwd_out_nt.txt).  A cache-sized output keeps plain
    // stores, so whatever reads it next can still find it there.  MAXK_FWD_OUT_NT: 0 never,
    // 1 always, 2 (default) by size.
    const bool big = (double)num_rows * D * 4 > (double)kInfinityCacheBytes;
    const int flags = (accumulate ? 1 : 0) |
                      ((MAXK_FWD_OUT_NT == 1 || (MAXK_FWD_OUT_NT == 2 && big)) ? 2 : 0);
    switch (L.kg) {
#define MAXK_CASE(KGV)                                                                     \
    case KGV:                                                                              \
        launch_fwd<KGV>(L, s, row_ptr, col_idx, edge_val, rec, row_div, out, slab,         \
                        slab_row, nr, num_e, D, k, flags, esel, trec);                     \
        break;
        MAXK_CASE(8)
        MAXK_CASE(16)
        MAXK_CASE(32)
        MAXK_CASE(64)
#undef MAXK_CASE
        default:
            set_error("unsupported lane group %d", L.kg);
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED("spgemm_fwd_kernel");
    return launch_slab_fixup<0>(slab, slab_row, out, D, L.n_items, s);
}
}  // namespace

extern "C" int maxk_spgemm_forward(const int32_t *row_ptr, const int32_t *col_idx,
                                   const float *edge_val, const float *cbsr_val,
                                   const uint8_t *cbsr_idx, const float *row_div, float *out,
                                   int64_t num_rows, int64_t num_cols, int64_t num_e,
                                   int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                   void *workspace, size_t workspace_bytes, void *stream) {
    clear_error();
    return forward_impl(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out, num_rows,
                        num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace,
                        workspace_bytes, stream, 0);
}

namespace {
// The forward writing the edge-selector stream (accumulate: adding onto out).
int forward_sel(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div, float *out,
                int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin,
                int32_t dim_k, int32_t chunk_edges, void *workspace, size_t workspace_bytes,
                void *stream, uint8_t *edge_sel, int accumulate) {
    MAXK_REQUIRE(num_e == 0 || edge_sel, "edge_sel must not be NULL");
    const bool direct = dim_k <= kWave && num_cols < (1 << 24) &&
                        (uint64_t)record_stride(dim_k, num_cols) * (uint64_t)num_cols < (1ull << 32);
    if (int rc = forward_impl(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out,
                              num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace,
                              workspace_bytes, stream, accumulate, direct ? edge_sel : nullptr))
        return rc;
    if (direct || num_e == 0) return MAXK_OK;
    // past 32-bit record offsets the walker takes 64-bit addresses and does not emit: gather
    return maxk_edge_selectors(col_idx, cbsr_idx, num_e, dim_k, edge_sel, stream);
}
}  // namespace

extern "C" int maxk_spgemm_forward_sel(const int32_t *row_ptr, const int32_t *col_idx,
                                       const float *edge_val, const float *cbsr_val,
                                       const uint8_t *cbsr_idx, const float *row_div, float *out,
                                       int64_t num_rows, int64_t num_cols, int64_t num_e,
                                       int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                       void *workspace, size_t workspace_bytes, void *stream,
                                       uint8_t *edge_sel) {
    clear_error();
    return forward_sel(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out, num_rows,
                       num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace, workspace_bytes,
                       stream, edge_sel, 0);
}

extern "C" int maxk_spgemm_forward_accumulate_sel(
    const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val, const float *cbsr_val,
    const uint8_t *cbsr_idx, const float *row_div, float *out, int64_t num_rows, int64_t num_cols,
    int64_t num_e, int32_t dim_origin, int32_t dim_k, int32_t chunk_edges, void *workspace,
    size_t workspace_bytes, void *stream, uint8_t *edge_sel) {
    clear_error();
    if (num_e == 0) return MAXK_OK;  // adds zeros, writes no selectors
    return forward_sel(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out, num_rows,
                       num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace, workspace_bytes,
                       stream, edge_sel, 1);
}

extern "C" int maxk_spgemm_forward_accumulate(const int32_t *row_ptr, const int32_t *col_idx,
                                              const float *edge_val, const float *cbsr_val,
                                              const uint8_t *cbsr_idx, const float *row_div,
                                              float *out, int64_t num_rows, int64_t num_cols,
                                              int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                              int32_t chunk_edges, void *workspace,
                                              size_t workspace_bytes, void *stream) {
    clear_error();
    if (num_e == 0) return MAXK_OK;  // adds zeros
    return forward_impl(row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out, num_rows,
                        num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace,
                        workspace_bytes, stream, 1);
}

extern "C" int maxk_records_ok(int64_t num_rows, int64_t num_cols, int64_t num_e,
                               int32_t dim_origin, int32_t dim_k) {
    if (num_rows <= 0 || num_cols <= 0 || num_e <= 0 || dim_origin <= 0 || dim_k <= 0 ||
        dim_k > dim_origin || dim_origin > kMaxDim)
        return 0;
    return records_ok(fwd_layout(num_rows, num_cols, num_e, dim_origin, dim_k, 0), num_cols,
                      dim_k)
               ? 1
               : 0;
}

extern "C" int maxk_cbsr_records(const float *cbsr_val, const uint8_t *cbsr_idx, uint8_t *rec,
                                 int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                                 void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(dim_origin >= 1 && dim_origin <= kMaxDim, "dim_origin must be in [1,256]");
    MAXK_REQUIRE(dim_k >= 4 && dim_k <= dim_origin && dim_k % 4 == 0 && dim_k <= 128,
                 "transport records need dim_k %% 4 == 0 in [4, min(dim_origin, 128)], got %d",
                 dim_k);
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(cbsr_val && cbsr_idx && rec, "pointers must not be NULL");
    MAXK_REQUIRE(((uintptr_t)rec & 3) == 0 && ((uintptr_t)cbsr_val & 3) == 0,
                 "records and values must be 4-B aligned");
    const int vpw = kPackBlock / (dim_k / 4);
    const int64_t groups = ceil_div(num_rows, (int64_t)vpw);
    hipLaunchKernelGGL(cbsr_records_kernel,
                       dim3((unsigned)(groups < MAXK_PACK_GRID ? groups : MAXK_PACK_GRID)),
                       dim3(kPackBlock), 0, as_stream(stream), cbsr_val, cbsr_idx, rec,
                       (int)num_rows, dim_k, dim_origin);
    MAXK_LAUNCHED("cbsr_records_kernel");
    return MAXK_OK;
}

extern "C" int maxk_spgemm_forward_records(const int32_t *row_ptr, const int32_t *col_idx,
                                           const float *edge_val, const uint8_t *rec,
                                           const float *row_div, float *out, int64_t num_rows,
                                           int64_t num_cols, int64_t num_e, int32_t dim_origin,
                                           int32_t dim_k, int32_t chunk_edges, void *workspace,
                                           size_t workspace_bytes, void *stream,
                                           int32_t accumulate) {
    clear_error();
    if (accumulate && num_e == 0) return MAXK_OK;  // adds zeros
    MAXK_REQUIRE(num_e == 0 || rec, "rec must not be NULL");
    MAXK_REQUIRE(((uintptr_t)rec & 3) == 0, "records must be 4-B aligned");
    if (num_e == 0) {  // nothing to walk: zero rows
        MAXK_REQUIRE(num_rows >= 0 && dim_origin >= 1 && dim_origin <= kMaxDim,
                     "num_rows / dim_origin out of range");
        MAXK_REQUIRE(num_rows == 0 || out, "out must not be NULL");
        return num_rows == 0 ? MAXK_OK
                             : zero_words(out, num_rows * (int64_t)dim_origin, as_stream(stream));
    }
    return forward_impl(row_ptr, col_idx, edge_val, nullptr, nullptr, row_div, out, num_rows,
                        num_cols, num_e, dim_origin, dim_k, chunk_edges, workspace,
                        workspace_bytes, stream, accumulate ? 1 : 0, nullptr, rec);
}
