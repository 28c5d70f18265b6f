// Backward outer-product sampled SpMM (SSpMM) for gfx950:
//   grad_cbsr[c, l] = sum_{e=(r->c)} val[e] * G[r, sel[c, l]] / row_div[r]
//
// Semantics: kernels/spmm_maxk_backward.cu:15-115 (push from the CSR of A, which
// yields the A^T product) and the /out_degrees of maxk_spgemm_function.py:154-155.
//
// Every edge needs the k values of its source row's G picked by its destination's
// selectors, summed per destination c.  Four forms of that sum:
//  * pull (maxk_sspmm_backward_pull, the default for k % 4 == 0 on dense graphs):
//    per tile (row slice, destination bucket) the edges' values are gathered straight from
//    G / row_div into an fp64 LDS accumulator; no per-edge contribution rows
//    (pull_tile_kernel below).
//  * atomic (maxk_sspmm_backward): the push, each G row staged once in LDS and one global
//    fp32 atomic per (edge, l) into grad_cbsr (zeroed first).  MI355X executes float
//    atomics memory-side and they are bound by request count: ~6 ms for Reddit-sized at
//    any k in 2..16.
//  * two-phase: phase 1 (the push) stores each edge's contribution row in CSR edge order
//    (non-temporal 16-B buffer stores, so the 7.3 GB stream does not evict the
//    selector table every edge gathers from), then
//    - bsort (maxk_sspmm_backward_bsort): phase 1 writes each window of CSR edges' rows
//      ordered by destination bucket; per bucket of destinations the rows are read as runs
//      and summed in an fp64 LDS accumulator (bucket_sum_kernel below; the plain "bucket"
//      mode over CSR-ordered rows left the library in r06);
//    - csc (maxk_sspmm_backward_csc): per destination, the rows are gathered through the
//      CSC permutation and summed in a fixed order; bitwise deterministic.
// Phase 1 and the csc phase 2 use the token-stream work partition of common.h (one wave
// per item of C tokens, hub rows split, short rows batched); loads-in-flight depth per
// launch from the average degree (pick_depth).
#include <algorithm>

#include "common.h"

namespace maxk {
namespace {

enum { kAtomic = 0, kStore = 1, kStoreX4 = 2, kStoreX4W = 3, kStoreX4S = 4 };

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A contribution row's 16 B in phase 2.  NT: rows of whole 128-B lines (k % 32 == 0) are read
// once, so non-temporally -- ogbn-products-sized csc backward k = 32 7.85 -> 7.77 ms, with the
// selector stream 6.71 -> 6.60, k = 64 15.14 -> 14.75; rows sharing a line (k <= 16) need
// the line kept for the other row, and lose 3-6 % that way (Reddit-sized csc k = 16 3.86 ->
// 4.10, products k = 16 5.17 -> 5.37, bsort k = 8 3.06 -> 3.15; profiles/r06/tune/t_load_nt/).
template <bool NT>
__device__ __forceinline__ float4 t_load4(const float4 *p) {
    if constexpr (NT)
        return __builtin_bit_cast(float4,
                                  __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p)));
    return *p;
}

// kStoreX4 (k % 4 == 0): LR = pow2ceil(k/4) lanes per edge, each lane owning 4
// consecutive l: one u32 selector load, four LDS reads, one 16-B store; 64/LR
// edges per wave step (4x fewer memory instructions per edge than one l per
// lane).  All memory goes through wave-uniform buffer descriptors with 32-bit
// offsets (wave_buffer, common.h), which keeps 64-bit address math out of the loop:
//  * col_idx / edge_val over the segment [sb, se): the lane's offset is fixed per
//    batch and the step's part is the instruction's immediate; past se the loads
//    return 0 (column 0, weight 0), so nothing is clamped;
//  * the selector table: offset c*k + 4q, one 24-bit multiply-add (kStoreX4W, for
//    tables past 2^24 columns, a 32-bit multiply);
//  * T rows [sb, se): past se, or for lanes q >= k/4 (offset pushed past 2^31), the
//    hardware drops the store, so no store is predicated.
// Cache policy of the T stores: MAXK_T_AUX (0 plain, 2 nt, 16 sc1).  Store lag as in
// push_edges below.
// ES (edge selectors, maxk_sspmm_backward_csc_sel): the selectors come as a per-edge stream
// esel[e * k + l] (= cbsr_idx[col_idx[e], l]) read in CSR order beside the weights, instead
// of a gather of the destination's row of cbsr_idx per edge: no column loads and no random
// selector line per edge (an ogbn-products-sized table is 20-80 MB, and each gather moved a
// whole 128-B line from the Infinity Cache).
template <int LR, int U, bool WIDE, bool ES = false>
__device__ __forceinline__ void push_x4(const float *g_lds, const int32_t *__restrict__ col_idx,
                                        const float *__restrict__ edge_val,
                                        const uint8_t *__restrict__ cbsr_idx,
                                        float *__restrict__ T, int sb, int se, int k, int lane,
                                        const uint8_t *__restrict__ esel = nullptr) {
    constexpr int G = kWave / LR;
    constexpr int GU = G * U;
    const int grp = lane / LR;
    const int q = lane % LR;
    const int k4 = k >> 2;
    const int n = se - sb;  // wave-uniform, <= chunk
    const auto crs = wave_buffer(col_idx + sb, (uint32_t)n * 4u);
    const auto vrs = wave_buffer(edge_val + sb, (uint32_t)n * 4u);
    // ES: the segment's selector stream; else the table (offsets < num_cols*k < 2^31)
    const auto srs = ES ? wave_buffer(esel + (size_t)(uint32_t)sb * k, (uint32_t)n * k)
                        : wave_buffer(cbsr_idx, 0xffffffffu);
    const auto trs = wave_buffer(T + (size_t)(uint32_t)sb * k, (uint32_t)n * k * 4u);  // <= 2 MiB
    const uint32_t qsel = 4u * (uint32_t)(q < k4 ? q : k4 - 1);
    const uint32_t qst = q < k4 ? 16u * q : 0x80000000u;  // store offset term; past the end if idle
    const uint32_t kb = 4u * (uint32_t)k;                    // T row bytes
    auto sel_off = [&](int c) -> int {
        return WIDE ? (int)((uint32_t)c * (uint32_t)k + qsel)
                    : (int)(__umul24((uint32_t)c, (uint32_t)k) + qsel);
    };
    int c[U];
    float w[U];
    {
        const int lo = grp * 4;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ES) c[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, lo + u * G * 4, 0, 0);
            w[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vrs, lo + u * G * 4, 0, 0));
        }
    }
    u32x4 xp[U];
    uint32_t sto = 0;  // T byte offset of the pending batch's step 0 for this lane
    bool pending = false;
    for (int base = 0;; base += GU) {  // base: edge offset inside the segment
        const bool has_next = base + GU < n;  // wave-uniform
        int cn[U];
        float wn[U];
        if (has_next) {
            const int lo = (base + GU + grp) * 4;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ES)
                    cn[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(crs, lo + u * G * 4, 0, 0);
                wn[u] = __uint_as_float(
                    __builtin_amdgcn_raw_buffer_load_b32(vrs, lo + u * G * 4, 0, 0));
            }
        }
        uint32_t sv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            sv[u] = __builtin_amdgcn_raw_buffer_load_b32(
                srs, ES ? (int)((uint32_t)(base + u * G + grp) * (uint32_t)k + qsel)
                        : sel_off(c[u]), 0, 0);
        if (pending) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(xp[u], trs, (int)(sto + u * G * kb), 0,
                                                       MAXK_T_AUX);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t s = sv[u];
            xp[u].x = __float_as_uint(w[u] * g_lds[s & 255u]);
            xp[u].y = __float_as_uint(w[u] * g_lds[(s >> 8) & 255u]);
            xp[u].z = __float_as_uint(w[u] * g_lds[(s >> 16) & 255u]);
            xp[u].w = __float_as_uint(w[u] * g_lds[s >> 24]);
        }
        sto = (uint32_t)(base + grp) * kb + qst;
        pending = true;
        if (!has_next) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ES) c[u] = cn[u];
            w[u] = wn[u];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(xp[u], trs, (int)(sto + u * G * kb), 0, MAXK_T_AUX);
}

// Walk edges [sb, se) (sb < se) of one staged row.  All loads are
// unconditional (clamped addresses).
//  kAtomic: one predicated global fp32 atomic per (edge, l).
//  kStore (k <= KG): contribution rows go to T in CSR edge order with a
//    one-batch store lag.  On gfx950 stores count in vmcnt with the loads, so a
//    wait for a load drains every OLDER store: per batch the order is
//    [prefetch col/val of batch i+1] [selector loads of batch i] [stores of
//    batch i-1] [wait selectors] -> the stores in flight are always younger than
//    the loads being waited for.  Masked lanes store to the dummy row of T, so
//    no store is predicated (a predicated store becomes a branch + full wait).
template <int KG, int U, int MODE>
__device__ __forceinline__ void push_edges(const float *g_lds, const int32_t *__restrict__ col_idx,
                                           const float *__restrict__ edge_val,
                                           const uint8_t *__restrict__ cbsr_idx,
                                           float *__restrict__ dst, int dummy, int sb, int se,
                                           int k, int lane, const uint8_t *__restrict__ esel) {
    if constexpr (MODE == kStoreX4S) {
        push_x4<KG, U, false, true>(g_lds, col_idx, edge_val, cbsr_idx, dst, sb, se, k, lane,
                                    esel);
        return;
    }
    if constexpr (MODE == kStoreX4 || MODE == kStoreX4W) {
        push_x4<KG, U, MODE == kStoreX4W>(g_lds, col_idx, edge_val, cbsr_idx, dst, sb, se, k, lane);
        return;
    }
    constexpr int G = kWave / KG;
    constexpr int GU = G * U;
    const int grp = lane / KG;
    const int l0 = lane % KG;
    const int last = se - 1;
    int c[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = sb + u * G + grp;
        const int ec = e < se ? e : last;
        c[u] = col_idx[ec];
        w[u] = edge_val[ec];
    }
    if (MODE == kStore && k <= KG) {
        const bool lok = l0 < k;
        const int lc = lok ? l0 : k - 1;
        float xp[U] = {};
        int rp[U];  // T row of each pending store (dummy for masked lanes)
        bool pending = false;
        for (int base = sb;; base += GU) {
            const bool has_next = base + GU < se;  // wave-uniform
            int cn[U];
            float wn[U];
            if (has_next) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = base + GU + u * G + grp;
                    const int ec = e < se ? e : last;
                    cn[u] = col_idx[ec];
                    wn[u] = edge_val[ec];
                }
            }
            int s[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                s[u] = cbsr_idx[c[u] * k + lc];
            }
            if (pending) {
#pragma unroll
                for (int u = 0; u < U; ++u) dst[(size_t)(uint32_t)rp[u] * k + lc] = xp[u];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = base + u * G + grp;
                xp[u] = w[u] * g_lds[s[u]];
                rp[u] = (e < se && lok) ? e : dummy;
            }
            pending = true;
            if (!has_next) break;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                c[u] = cn[u];
                w[u] = wn[u];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) dst[(size_t)(uint32_t)rp[u] * k + lc] = xp[u];
        return;
    }
    for (int base = sb;; base += GU) {
        const bool has_next = base + GU < se;  // wave-uniform
        for (int lb = 0; lb < k; lb += KG) {
            const int l = lb + l0;
            const bool lok = l < k;
            const int lc = lok ? l : k - 1;
            int s[U];
#pragma unroll
            for (int u = 0; u < U; ++u) s[u] = cbsr_idx[c[u] * k + lc];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = base + u * G + grp;
                const float x = w[u] * g_lds[s[u]];
                if (MODE == kAtomic) {
                    if (e < se && lok) atomicAdd(&dst[c[u] * k + l], x);
                } else {
                    dst[(size_t)(uint32_t)((e < se && lok) ? e : dummy) * k + (lok ? l : 0)] = x;
                }
            }
        }
        if (!has_next) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + GU + u * G + grp;
            const int ec = e < se ? e : last;
            c[u] = col_idx[ec];
            w[u] = edge_val[ec];
        }
    }
}

template <int KG, int U, int MODE>
__global__ __launch_bounds__(kBlock, MAXK_BWD_WAVES) void sspmm_bwd_kernel(
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col_idx,
    const float *__restrict__ edge_val, const float *__restrict__ grad,
    const float *__restrict__ row_div, const uint8_t *__restrict__ cbsr_idx,
    float *__restrict__ dst, int num_rows, int64_t num_e, int D, int k, int chunk, int n_items,
    const uint8_t *__restrict__ esel) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    // MAXK_P1_XCD: XCD-contiguous items, as in the forward (an ordered graph's destinations,
    // whose selectors every edge reads, then stay close within one XCD)
    const int blk = MAXK_P1_XCD ? xcd_contiguous_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int item = blk * kWavesPerBlock + wid;
    if (item >= n_items) return;
    float *g_lds = lds[wid];
    *reinterpret_cast<float4 *>(&g_lds[lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);

    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int r = wave_first_row_token(row_ptr, num_rows, d0);
    // Rows q = r-1 (continuation), r, r+1, ...: the item's edges of row q are
    // [max(rb, d0-q-1), min(re, d1-q-1)).  row_ptr / row_div of 64 consecutive rows sit
    // one per lane (read with readlane), and each row's G values (4 per lane, columns
    // lane + 64*i) are loaded while the previous row's edges are pushed: no per-row
    // dependent load before a row can start.
    int q = r > 0 ? r - 1 : 0;
    int wb = q;
    int rpw = row_ptr[wb + lane < num_rows ? wb + lane : num_rows];
    float dvw = row_div ? row_div[wb + lane < num_rows ? wb + lane : num_rows - 1] : 1.f;
    auto load_g = [&](int row, float (&g)[4]) {
        const float *gr = grad + (int64_t)(row < num_rows ? row : num_rows - 1) * D;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = lane + kWave * i;
            g[i] = gr[j < D ? j : D - 1];
        }
    };
    float gn[4];
    load_g(q, gn);
    for (; q < num_rows; ++q) {
        if (q + 1 - wb >= kWave) {  // slide the window
            wb = q;
            rpw = row_ptr[wb + lane < num_rows ? wb + lane : num_rows];
            if (row_div) dvw = row_div[wb + lane < num_rows ? wb + lane : num_rows - 1];
        }
        const int rb = __builtin_amdgcn_readlane(rpw, q - wb);
        const int re = __builtin_amdgcn_readlane(rpw, q + 1 - wb);
        if ((int64_t)q + rb >= d1) break;
        float g[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = gn[i];
        if (q + 1 < num_rows) load_g(q + 1, gn);
        const int64_t sb64 = d0 - q - 1 > rb ? d0 - q - 1 : rb;
        const int64_t se64 = d1 - q - 1 < re ? d1 - q - 1 : re;
        if (sb64 >= se64) continue;
        const float div = __builtin_bit_cast(
            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dvw), q - wb));
        wave_lds_fence();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = lane + kWave * i;
            if (j < D) g_lds[j] = row_div ? g[i] / div : g[i];
        }
        wave_lds_fence();
        push_edges<KG, U, MODE>(g_lds, col_idx, edge_val, cbsr_idx, dst, (int)num_e, (int)sb64,
                                (int)se64, k, lane, esel);
    }
}

// ---- phase 2: grad_cbsr[c, :] = sum over the CSC slots t of c of T[eid[t], :] -------

// Sum the contribution rows T[eid[t]] (k floats each) for t in [tb, te) into
// dst[0:k], in a fixed order.  VEC (k in {4,8,...,256}): LR = k/4 lanes per row
// (16-B loads), 64/LR rows per wave step, U steps in flight; the row groups are
// combined by xor butterflies.  Scalar: KG = pow2ceil(k) lanes per row.
template <bool VEC, int KG, int U, bool NT = false, typename EidAt>
__device__ __forceinline__ void segment_sum(const float *__restrict__ T, EidAt eid, int64_t tb,
                                            int64_t te, int k, float *__restrict__ dst, int lane) {
    if constexpr (VEC) {
        const int LR = k / 4, RI = kWave / LR;
        const int g = lane / LR, q = lane % LR;
        const float4 *__restrict__ T4 = reinterpret_cast<const float4 *>(T);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int64_t base = tb; base < te; base += (int64_t)RI * U) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t t = base + u * RI + g;
                const int e = eid(t < te ? t : tb);
                v[u] = t_load4<NT>(&T4[(size_t)(uint32_t)e * LR + q]);
                if (t >= te) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a.x += v[u].x;
                a.y += v[u].y;
                a.z += v[u].z;
                a.w += v[u].w;
            }
        }
        for (int off = LR; off < kWave; off <<= 1) {
            a.x += __shfl_xor(a.x, off);
            a.y += __shfl_xor(a.y, off);
            a.z += __shfl_xor(a.z, off);
            a.w += __shfl_xor(a.w, off);
        }
        if (g == 0) reinterpret_cast<float4 *>(dst)[q] = a;
    } else {
        constexpr int G = kWave / KG;
        const int grp = lane / KG;
        for (int l = lane % KG; l - lane % KG < k; l += KG) {  // one pass unless k > 64
            const bool lok = l < k;
            const int lc = lok ? l : k - 1;
            float a = 0.f;
            for (int64_t base = tb; base < te; base += (int64_t)G * U) {
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t t = base + u * G + grp;
                    const int e = eid(t < te ? t : tb);
                    v[u] = T[(size_t)(uint32_t)e * k + lc];
                    if (t >= te) v[u] = 0.f;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) a += v[u];
            }
            for (int off = KG; off < kWave; off <<= 1) a += __shfl_xor(a, off);
            if (grp == 0 && lok) dst[l] = a;
        }
    }
}

// Grouped destinations (low average in-degree, e.g. the halo columns of an N = 8 shard, ~6
// slots each, where segment_sum spends one wave step and a 3-stage butterfly per destination).
// Each lane group of LR = k/4 lanes walks one destination's slots U at a time into its own
// float4 (in slot order: bitwise the same run to run), stores the row the step it ends and takes
// the item's next destination, so 64/LR destinations are in flight per wave; the next step's
// gathers are issued before this step's sums.  Destinations are taken in order while owned by
// the item (token < d1) and holding at most lmax of its slots; returns the first one not taken
// (the caller sums a longer one with the whole wave).  k % 4 == 0.
template <int U, bool NT = false, typename EidAt>
__device__ __forceinline__ int csc_groups(const float *__restrict__ T, EidAt eid_at,
                                          const int32_t *__restrict__ col_ptr, int c,
                                          int num_cols, int64_t d1, int k, int lmax,
                                          float *__restrict__ grad_cbsr, int lane) {
    const int LR = k / 4, NG = kWave / LR;
    const int g = lane / LR, q = lane % LR;
    const float4 *__restrict__ T4 = reinterpret_cast<const float4 *>(T);
    int wb = c;  // col_ptr window: destinations [wb, wb + 64), one per lane
    int cpw = col_ptr[wb + lane <= num_cols ? wb + lane : num_cols];
    int next = c;       // the next destination to hand out (wave-uniform)
    bool stop = false;  // it is not the item's or is too long (wave-uniform)
    int dst = -1;       // this group's destination and its slot range [t, te)
    int64_t t = 0, te = 0;
    auto assign = [&]() {
        const uint64_t idle = __ballot(dst < 0);
        for (int gi = 0; gi < NG && !stop; ++gi) {
            if (!((idle >> (gi * LR)) & 1ull)) continue;
            if (next + 1 >= wb + kWave) {  // slide the window (wave-uniform)
                wb = next;
                cpw = col_ptr[wb + lane <= num_cols ? wb + lane : num_cols];
            }
            const int64_t cb = __builtin_amdgcn_readlane(cpw, next - wb);
            int64_t se = __builtin_amdgcn_readlane(cpw, next + 1 - wb);
            if (d1 - next - 1 < se) se = d1 - next - 1;
            if (next < num_cols && next + cb < d1 && se - cb <= lmax) {
                if (g == gi) {
                    dst = next;
                    t = cb;
                    te = se;
                }
                ++next;
            } else {
                stop = true;
            }
        }
    };
    auto gather = [&](float4 (&v)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (dst >= 0 && t + u < te) v[u] = t_load4<NT>(&T4[(size_t)(uint32_t)eid_at(t + u) * LR + q]);
        }
    };
    assign();
    float4 v[U];
    gather(v);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    while (__ballot(dst >= 0)) {
        const int cdst = dst;
        const bool fin = cdst >= 0 && t + U >= te;
        if (fin) dst = -1;
        t += U;
        assign();
        float4 vn[U];
        gather(vn);  // the next step's rows in flight while this step's are summed
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a.x += v[u].x;
            a.y += v[u].y;
            a.z += v[u].z;
            a.w += v[u].w;
            v[u] = vn[u];
        }
        if (fin) {
            reinterpret_cast<float4 *>(grad_cbsr + (int64_t)cdst * k)[q] = a;
            a = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    return next;
}

// STAGED (chunk <= kCscStage): the item's CSC slots are one contiguous range of csc_eid,
// starting at d0 - c (the tokens before d0 hold c destination tokens), so the wave copies
// up to `chunk` of them into LDS with coalesced loads before its first segment: every T-row
// gather then waits for one load instead of two dependent ones (a destination of ogbn-products
// averages 50 slots, two U-steps, so each step used to wait for its eid loads first).
constexpr int kCscStage = 2048;
// GROUP (VEC, STAGED): destinations of at most kCscGroupMax slots go through csc_groups.
constexpr int kCscGroupMax = 64;
template <bool VEC, int KG, int U, bool STAGED, bool GROUP = false, bool NT = false>
__global__ __launch_bounds__(kBlock) void csc_sum_kernel(const int32_t *__restrict__ col_ptr,
                                                         const int32_t *__restrict__ eid,
                                                         const float *__restrict__ T,
                                                         float *__restrict__ grad_cbsr,
                                                         float *__restrict__ slab,
                                                         int32_t *__restrict__ slab_row,
                                                         int num_cols, int64_t num_e, int k,
                                                         int chunk, int n_items) {
    extern __shared__ int32_t s_eid[];  // STAGED: [kWavesPerBlock][chunk]
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int blk = !MAXK_XCD_SUM      ? (int)blockIdx.x
                    : MAXK_XCD_SUM_RUN ? xcd_window_block(blockIdx.x, gridDim.x, MAXK_XCD_SUM_RUN)
                                       : xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int item = blk * kWavesPerBlock + wid;
    if (item >= n_items) return;
    const int64_t total = (int64_t)num_cols + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int c = wave_first_row_token(col_ptr, num_cols, d0);
    const int64_t p_lo = d0 - c;  // the item's first CSC slot
    int32_t *se_lds = s_eid + (STAGED ? wid * chunk : 0);
    if constexpr (STAGED) {
        const int n_pos = (int)(num_e - p_lo < chunk ? num_e - p_lo : chunk);
        for (int i = lane; i < n_pos; i += kWave) se_lds[i] = eid[p_lo + i];
        wave_lds_fence();
    }
    auto eid_at = [&](int64_t t) -> int {
        if constexpr (STAGED)
            return se_lds[(int)(t - p_lo)];
        else
            return eid[t];
    };
    int cont = -1;
    if (c > 0) {
        const int64_t sb = p_lo;
        int64_t se = (int64_t)col_ptr[c];
        if (d1 - c < se) se = d1 - c;
        if (sb < se) {
            segment_sum<VEC, KG, U, NT>(T, eid_at, sb, se, k, slab + (int64_t)item * k, lane);
            cont = c - 1;
        }
    }
    if (lane == 0) slab_row[item] = cont;
    for (; c < num_cols; ++c) {
        if constexpr (GROUP) {
            c = csc_groups<U, NT>(T, eid_at, col_ptr, c, num_cols, d1, k, kCscGroupMax, grad_cbsr,
                              lane);
            if (c >= num_cols) break;
        }
        const int64_t cb = col_ptr[c];
        if (cb + c >= d1) break;
        int64_t se = (int64_t)col_ptr[c + 1];
        if (d1 - c - 1 < se) se = d1 - c - 1;
        segment_sum<VEC, KG, U, NT>(T, eid_at, cb, se, k, grad_cbsr + (int64_t)c * k, lane);
    }
}

// ---- phase 2, bucketed: grad_cbsr[c, :] = sum of T[e, :] over the entries of c's bucket ----
// The bucket-ordered entry list (bucket_eid: per bucket of 2^shift destinations, the CSR
// edge ids into it in CSR order) is cut into equal parts of `part` entries, one
// 1024-thread workgroup each, so a heavy bucket (power-law in-degrees: the largest
// Reddit-sized bucket holds 1.2x the mean) never sets the kernel time alone.  A part
// walks the buckets it meets; per bucket it sums into an fp64 LDS accumulator
// [2^shift, k + 1] and stores the bucket's rows directly when it holds all of the bucket's
// entries, else one fp32 partial to its slab slot (slot 0: the part's first bucket, 1: its
// last); bucket_fixup_kernel adds the partials in part order and zero-fills empty buckets.
// Entries are read in order, LR = pow2ceil(k/4) lanes per T row (16-B loads), 64/LR
// consecutive entries per wave instruction: neighbouring entries of one source row are
// neighbouring T rows, so one line request serves several of them (a Reddit-sized bucket
// of 1024 destinations holds ~2.2 edges of every source row).  Sums go through ds_add_f64:
// on gfx950 it costs about a ds_write (8.8 cycles per wave instruction), ds_add_f32 costs
// 193 (tools/lds_atomic_probe.hip).  fp64 partial sums make the fp32 result independent of
// the order of the adds except in rare rounding ties.  U steps of loads in flight, the
// next step's entry ids prefetched.
template <int LR, int U>
__global__ __launch_bounds__(1024) void bucket_sum_kernel(
    const float *__restrict__ T, const int32_t *__restrict__ bucket_ptr,
    const int32_t *__restrict__ bucket_eid, const uint16_t *__restrict__ bucket_dst,
    float *__restrict__ grad_cbsr, float *__restrict__ slab, int num_cols, int n_buckets,
    int num_e, int k, int shift, int part) {
    __shared__ double acc[kBucketAccDoubles];
    __shared__ int s_j0;
    constexpr int EPI = kWave / LR;  // entries per wave instruction
    constexpr int STEP = EPI * U;    // entries per wave step
    const int tid = threadIdx.x;
    const int lane = lane_id(), w = tid / kWave;
    const int g = lane / LR, q = lane % LR;
    const int kq = k >> 2;
    const bool qok = q < kq;
    const int nacc = k << shift;  // floats of one bucket (output / slab slot)
    const int ks = k + 1;         // LDS row stride (doubles)
    const int nlds = ks << shift;
    const int p = blockIdx.x;
    const int p0 = p * part, p1 = num_e - p0 > part ? p0 + part : num_e;
    if (tid == 0) {  // first bucket of the part: the last j with bucket_ptr[j] <= p0
        int lo = 0, hi = n_buckets - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (bucket_ptr[mid] <= p0) lo = mid; else hi = mid - 1;
        }
        s_j0 = lo;
    }
    __syncthreads();
    const int j0 = s_j0;
    const float4 *__restrict__ T4 = reinterpret_cast<const float4 *>(T);
    for (int j = j0; j < n_buckets; ++j) {
        const int b0 = bucket_ptr[j], b1 = bucket_ptr[j + 1];
        if (b0 >= p1) break;
        if (b0 == b1) continue;  // empty bucket: zero-filled by the fixup
        const int s0 = b0 > p0 ? b0 : p0, s1 = b1 < p1 ? b1 : p1;
        for (int i = tid; i < nlds; i += 1024) acc[i] = 0.0;
        __syncthreads();
        int base = s0 + w * STEP;
        int e[U], d[U];
        auto load_ids = [&](int b) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = b + u * EPI + g;
                const int tc = t < s1 ? t : s1 - 1;
                e[u] = bucket_eid[tc];
                d[u] = t < s1 ? (int)bucket_dst[tc] : -1;
            }
        };
        if (base < s1) load_ids(base);
        for (; base < s1; base += 16 * STEP) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = T4[(size_t)(uint32_t)e[u] * (uint32_t)kq + (qok ? q : 0)];
            int dc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) dc[u] = d[u];
            if (base + 16 * STEP < s1) load_ids(base + 16 * STEP);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (dc[u] >= 0 && qok) {
                    double *a = &acc[dc[u] * ks + 4 * q];
                    atomicAdd(a + 0, (double)v[u].x);
                    atomicAdd(a + 1, (double)v[u].y);
                    atomicAdd(a + 2, (double)v[u].z);
                    atomicAdd(a + 3, (double)v[u].w);
                }
            }
        }
        __syncthreads();
        const int64_t c0 = (int64_t)j << shift;
        const int rows = num_cols - c0 < (1 << shift) ? (int)(num_cols - c0) : (1 << shift);
        const bool whole = b0 >= p0 && b1 <= p1;
        float *o = whole ? grad_cbsr + c0 * k
                         : slab + ((size_t)p * 2 + (j == j0 ? 0 : 1)) * (size_t)nacc;
        for (int i = tid; i < rows * k; i += 1024) {
            const int r = i / k;
            o[i] = (float)acc[i + r];  // row r starts at r * (k + 1)
        }
        __syncthreads();
    }
}

// Buckets no single part holds whole: the sum of their parts' slab partials in part order;
// empty buckets: zeros.  One thread per 4 floats; blockIdx.x = bucket, blockIdx.y = tile.
__global__ __launch_bounds__(kBlock) void bucket_fixup_kernel(
    const int32_t *__restrict__ bucket_ptr, const float *__restrict__ slab,
    float *__restrict__ grad_cbsr, int num_cols, int k, int shift, int part) {
    const int j = blockIdx.x;
    const int b0 = bucket_ptr[j], b1 = bucket_ptr[j + 1];
    const int plo = b0 / part, phi = b1 > 0 ? (b1 - 1) / part : 0;
    if (b0 != b1 && plo == phi) return;  // stored whole by its part
    const int64_t c0 = (int64_t)j << shift;
    const int rows = num_cols - c0 < (1 << shift) ? (int)(num_cols - c0) : (1 << shift);
    const int n4 = rows * k / 4;  // k % 4 == 0
    const int i = blockIdx.y * kBlock + threadIdx.x;
    if (i >= n4) return;
    float4 *o = reinterpret_cast<float4 *>(grad_cbsr + c0 * k) + i;
    if (b0 == b1) {
        *o = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const size_t nacc4 = ((size_t)k << shift) / 4;
    const float4 *sl = reinterpret_cast<const float4 *>(slab);
    const int lo_slot = plo * part < b0 ? 1 : 0;  // bucket j is the last bucket of part plo
    float4 a = sl[((size_t)plo * 2 + lo_slot) * nacc4 + i];
    for (int p = plo + 1; p <= phi; ++p) {
        const float4 b = sl[(size_t)p * 2 * nacc4 + i];
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
    }
    *o = a;
}

// ---- window-sorted phase 1 ("bsort", maxk_sspmm_backward_bsort) ---------------------------
// On a large sparse graph every contribution row the bucketed phase 2 (or csc) reads lies on
// its own random line: at k = 8 a 32-B row costs a 128-B line, so phase 2 runs at the
// fabric's random-line rate whatever k.  Here the edges are cut into windows
// of W consecutive CSR edges (W * k * 4 B fill the 160 KiB LDS stage), one 1024-thread
// workgroup per window: its waves compute the window's rows into LDS in CSR order, then the
// workgroup writes them out to T[window] ordered by destination bucket (win_src: T row
// w0 + i holds edge w0 + win_src[w0 + i]; a stable sort on the bucket, from maxk_bsort_plan).
// A bucket's rows of one window are then one contiguous run (ogbn-products k = 8, W = 5120,
// 1196 buckets: ~4 rows, 137 B), read by bucket_sum_kernel through the plan's positions.  The
// writes stay coalesced: the reorder happens in LDS.
// One workgroup per CU (the stage fills the LDS), so every wave must keep its loads in flight
// across its share of the window: the share is walked in flat batches of edges whatever rows
// they belong to (the source row of each edge from the plan's edge_row), each edge's k values
// gathered straight from G (its rows sit in L2: a window spans ~100 rows on ogbn-products), and
// batch i + 2's weights / selectors / rows and batch i + 1's gathers are issued before batch i
// is computed.  Per-row G staging in LDS as in sspmm_bwd_kernel cost one exposed load latency
// per row segment at this occupancy (2.68 vs 1.45 ms for the CSR-order phase 1, products k=8).
constexpr int kBsortThreads = 1024;
constexpr int kBsortWaves = kBsortThreads / kWave;
constexpr int kBsortStageFloats = 160 * 1024 / 4;
constexpr int kBsortPer = kBsortStageFloats / 4 / kBsortThreads;  // 16-B stage units per thread
static_assert(kBsortStageFloats % (4 * kBsortThreads) == 0, "whole units per thread");

template <int LR, int U, bool ES>
__global__ __launch_bounds__(kBsortThreads) void bsort_push_kernel(
    const int32_t *__restrict__ edge_row, const int32_t *__restrict__ col_idx,
    const float *__restrict__ edge_val, const float *__restrict__ grad,
    const float *__restrict__ row_div, const uint8_t *__restrict__ cbsr_idx,
    const uint8_t *__restrict__ esel, const uint16_t *__restrict__ win_src,
    float *__restrict__ T, int num_e, int D, int k, int W) {
    __shared__ __attribute__((aligned(16))) float stage[kBsortStageFloats];
    constexpr int G = kWave / LR;  // edges per wave instruction
    constexpr int GU = G * U;      // edges per batch
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int b = MAXK_P1_XCD ? xcd_contiguous_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int64_t w0l = (int64_t)b * W;
    if (w0l >= num_e) return;  // whole workgroup: padding blocks of the XCD grid
    const int w0 = (int)w0l;
    const int w1 = num_e - w0 > W ? w0 + W : num_e;
    const int per = (w1 - w0 + kBsortWaves - 1) / kBsortWaves;
    const int e0 = w0 + wid * per;
    const int n = (e0 + per < w1 ? e0 + per : w1) - e0;  // this wave's edges (may be <= 0)
    // the write-out's source rows, loaded now so they are in by the time it runs
    const int kq = k >> 2;
    const int nrow = w1 - w0;
    int src[kBsortPer];
#pragma unroll
    for (int j = 0; j < kBsortPer; ++j) {
        const int i = threadIdx.x + j * kBsortThreads;
        src[j] = i < nrow * kq ? (int)win_src[w0 + i / kq] : 0;
    }
    if (n > 0) {
        const int grp = lane / LR;
        const int q = lane % LR;
        const int k4 = k >> 2;
        const bool active = q < k4;
        const uint32_t qsel = 4u * (uint32_t)(active ? q : k4 - 1);
        // past the share's end the buffer loads return 0: weight 0, row 0, selector 0
        const auto vrs = wave_buffer(edge_val + e0, (uint32_t)n * 4u);
        const auto rrs = wave_buffer(edge_row + e0, (uint32_t)n * 4u);
        const auto crs = wave_buffer(col_idx + (ES ? 0 : e0), ES ? 0u : (uint32_t)n * 4u);
        const auto srs = ES ? wave_buffer(esel + (size_t)(uint32_t)e0 * k, (uint32_t)n * k)
                            : wave_buffer(cbsr_idx, 0xffffffffu);
        float *st = stage + (size_t)(e0 - w0) * k + 4 * q;
        struct Batch {  // per lane and wave instruction u: weight, source row, 4 selectors
            float w[U];
            int r[U];
            uint32_t s[U];
        };
        struct Vals {  // the 4 gathered G values and the row's divisor
            float v[U][4];
            float dv[U];
        };
        auto load_batch = [&](int base, Batch &a) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int o = (base + u * G + grp) * 4;
                a.w[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vrs, o, 0, 0));
                a.r[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(rrs, o, 0, 0);
                if (ES) {
                    a.s[u] = __builtin_amdgcn_raw_buffer_load_b32(
                        srs, (int)((uint32_t)(base + u * G + grp) * (uint32_t)k + qsel), 0, 0);
                } else {
                    const uint32_t c = __builtin_amdgcn_raw_buffer_load_b32(crs, o, 0, 0);
                    a.s[u] = __builtin_amdgcn_raw_buffer_load_b32(srs, (int)(c * (uint32_t)k + qsel),
                                                                  0, 0);
                }
            }
        };
        auto gather = [&](const Batch &a, Vals &g) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float *gr = grad + (int64_t)a.r[u] * D;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = (int)((a.s[u] >> (8 * j)) & 255u);
                    g.v[u][j] = gr[c < D ? c : 0];
                }
                g.dv[u] = row_div ? row_div[a.r[u]] : 1.f;
            }
        };
        auto compute = [&](int base, const Batch &a, const Vals &g) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float x[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = (int)((a.s[u] >> (8 * j)) & 255u);
                    const float gv = row_div ? g.v[u][j] / g.dv[u] : g.v[u][j];
                    x[j] = a.w[u] * (c < D ? gv : 0.f);  // a selector >= D reads 0
                }
                const int e = base + u * G + grp;
                if (active && e < n)
                    *reinterpret_cast<float4 *>(st + (size_t)e * k) =
                        make_float4(x[0], x[1], x[2], x[3]);
            }
        };
        Batch a0, a1;
        Vals g0;
        load_batch(0, a0);
        gather(a0, g0);
        if (GU < n) load_batch(GU, a1);
        for (int base = 0; base < n; base += GU) {
            Batch a2;
            Vals g1;
            if (base + 2 * GU < n) load_batch(base + 2 * GU, a2);
            if (base + GU < n) gather(a1, g1);
            compute(base, a0, g0);
            a0 = a1;
            a1 = a2;
            g0 = g1;
        }
    }
    __syncthreads();
    // write-out in bucket order: T row w0 + i <- staged row win_src[w0 + i], 16 B per thread,
    // non-temporal (the 1-4 GB stream would evict the lines phase 1 re-reads)
    const auto trs = wave_buffer(T + (size_t)w0 * k, (uint32_t)nrow * k * 4u);
    const float4 *st4 = reinterpret_cast<const float4 *>(stage);
#pragma unroll
    for (int j = 0; j < kBsortPer; ++j) {
        const int i = threadIdx.x + j * kBsortThreads;
        const int p = i / kq;
        const int sr = src[j] < nrow ? src[j] : nrow - 1;
        const float4 v = st4[sr * kq + (i - p * kq)];
        if (i < nrow * kq)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), trs, i * 16, 0,
                                                   MAXK_T_AUX);
    }
}

// ---- pull: the backward without contribution rows -------------------------------------
// grad_cbsr[c, :] = sum over the edges (r -> c) of w * G'[r, sel[c, :]], G' = G / row_div.
// The pull plan (maxk_pull_plan) sorts the edges into tiles: tile t = (row slice s,
// destination bucket j), t = s * n_buckets + j, CSR order inside a tile, each entry
// carrying its source row, weight and column within the bucket.  Workgroup t sums tile t
// into an fp64 LDS accumulator [2^shift, k + 1] (as bucket_sum_kernel, ds_add_f64) and
// stores it, fp32, to tile_out[t]; pull_reduce_kernel adds a bucket's slices in slice
// order.  The k values of an entry are gathered straight from G': workgroups start in tile
// order, so the ones in flight read one slice of G' rows (~3.5 MB, the size of an XCD's
// L2), and a source row's entries in a tile (~2 at Reddit scale) are neighbours in one
// wave instruction.  This replaces the 7.4 GB write + ~10 GB read of T by ~1.2 GB of
// entries and 2 x slices x 15 MB of tile partials (Reddit k=16).
__global__ __launch_bounds__(kBlock) void gprime_kernel(const float *__restrict__ G,
                                                        const float *__restrict__ row_div,
                                                        float *__restrict__ Gp, int64_t n4,
                                                        int D4) {
    const int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    if (i >= n4) return;
    const float dv = row_div[i / D4];
    float4 v = reinterpret_cast<const float4 *>(G)[i];
    v.x /= dv;
    v.y /= dv;
    v.z /= dv;
    v.w /= dv;
    reinterpret_cast<float4 *>(Gp)[i] = v;
}

// LR = pow2ceil(k/4) lanes per entry, lane q owning l = 4q..4q+3: per entry one 8-B entry
// load, one u32 selector read (from LDS when the bucket's selector rows fit next to the
// accumulator, SEL_LDS), four gathers and four LDS adds; 64/LR entries per wave
// instruction, U instructions per wave step, the next step's entries prefetched.
// Entry = {row within the slice | column within the bucket << 16, weight bits}.
template <int LR, int U, bool SEL_LDS, int VPL>
__global__ __launch_bounds__(1024) void pull_tile_kernel(
    const float *__restrict__ Gp, const uint8_t *__restrict__ cbsr_idx,
    const int32_t *__restrict__ tile_ptr, const uint2 *__restrict__ ent,
    float *__restrict__ tile_out, int64_t num_cols, int n_buckets, int rows_per_slice, int D,
    int k, int shift) {
    extern __shared__ double acc[];  // [(k + 1) << shift], then (SEL_LDS) [k << shift] bytes
    constexpr int EPI = kWave / LR;
    constexpr int STEP = EPI * U;
    const int tid = threadIdx.x;
    const int lane = lane_id(), w = tid / kWave;
    const int g = lane / LR, q = lane % LR;
    const bool qok = q < k / VPL;
    const int ks = k + 1;
    const int t = blockIdx.x;
    const int j = t % n_buckets;
    const float *__restrict__ Gs = Gp + (size_t)(t / n_buckets) * rows_per_slice * D;
    const int s0 = tile_ptr[t], s1 = tile_ptr[t + 1];
    const int64_t c0 = (int64_t)j << shift;
    const uint8_t *__restrict__ selg = cbsr_idx + c0 * k;
    uint8_t *sel_lds = reinterpret_cast<uint8_t *>(acc + (ks << shift));
    for (int i = tid; i < (ks << shift); i += 1024) acc[i] = 0.0;
    if (SEL_LDS) {
        const int rows = num_cols - c0 < (1 << shift) ? (int)(num_cols - c0) : (1 << shift);
        const int nb = rows * k;  // c0 * k is a multiple of 16 (shift >= 4), as is sel_lds
        for (int i = tid; i < nb / 16; i += 1024)
            reinterpret_cast<uint4 *>(sel_lds)[i] = reinterpret_cast<const uint4 *>(selg)[i];
        for (int i = (nb & ~15) + tid; i < nb; i += 1024) sel_lds[i] = selg[i];
    }
    __syncthreads();
    int base = s0 + w * STEP;
    uint2 en[U];
    // kShfl: 8-B loads with one entry per lane fetch the step's STEP entries (NL = STEP / 64
    // loads); each lane group then takes its entry from the loading lane with ds_bpermute:
    // NL memory instructions per step for the entries instead of U (the texture addresser,
    // not LDS, is the busy unit; Reddit k=8 / 16 / 32: -3.5 / -5.8 / -5.3 %).  With more than
    // 8 lanes per entry the two shuffles per instruction outweigh the loads saved (k=64 +4 %).
    constexpr bool kShfl = MAXK_PULL_SHFL && LR <= 8;
    constexpr int NL = (STEP + kWave - 1) / kWave;
    uint2 my[NL];
    auto load_ids = [&](int b) {
        if constexpr (kShfl) {
#pragma unroll
            for (int m = 0; m < NL; ++m) {
                const int e = b + m * kWave + lane;
                my[m] = ent[e < s1 ? e : s1 - 1];
                if (e >= s1 || m * kWave + lane >= STEP) my[m].x = 0xffff0000u;  // no entry
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * EPI + g;
                en[u] = ent[e < s1 ? e : s1 - 1];
                if (e >= s1) en[u].x = 0xffff0000u;  // no entry: row 0 (a valid gather), column 0xffff
            }
        }
    };
    if (base < s1) load_ids(base);
    for (; base < s1; base += 16 * STEP) {
        if constexpr (kShfl) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int m = (u * EPI) / kWave;  // compile-time after unrolling
                const int src = (u * EPI + g - m * kWave) * 4;
                en[u].x = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)my[m].x);
                en[u].y = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)my[m].y);
            }
        }
        uint32_t sv[U];
        int dc[U];
        float wc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t key = en[u].x;
            dc[u] = (key >> 16) == 0xffffu ? -1 : (int)(key >> 16);
            // VPL (4 or 1) consecutive selectors of the entry's destination, lane q's share
            const int bo = (dc[u] < 0 ? 0 : dc[u]) * k + (qok ? q : 0) * VPL;
            const uint8_t *sb8 = SEL_LDS ? sel_lds : selg;
            sv[u] = VPL == 4 ? *reinterpret_cast<const uint32_t *>(sb8 + bo) : (uint32_t)sb8[bo];
        }
        float v[U][VPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float *gr = Gs + (en[u].x & 0xffffu) * (uint32_t)D;
#pragma unroll
            for (int i = 0; i < VPL; ++i) {  // a selector >= D (D < 256) contributes 0
                const uint32_t c = (sv[u] >> (8 * i)) & 255u;
                const bool in = c < (uint32_t)D;
                const float x = gr[in ? c : 0u];
                v[u][i] = in ? x : 0.0f;
            }
            wc[u] = __uint_as_float(en[u].y);
        }
        if (base + 16 * STEP < s1) load_ids(base + 16 * STEP);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (dc[u] >= 0 && qok) {
                double *a = &acc[dc[u] * ks + VPL * q];
#pragma unroll
                for (int i = 0; i < VPL; ++i) atomicAdd(a + i, (double)(wc[u] * v[u][i]));
            }
        }
    }
    __syncthreads();
    float *o = tile_out + (size_t)t * ((size_t)k << shift);
    if (MAXK_PULL_F4_FLUSH && k % 4 == 0) {  // 16-B stores: 4x fewer store instructions
        for (int i4 = tid; i4 < (k << shift) / 4; i4 += 1024) {
            const double *a = &acc[i4 * 4 + (i4 * 4) / k];  // 4 l of one row (k % 4 == 0)
            reinterpret_cast<float4 *>(o)[i4] =
                make_float4((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
        }
    } else {
        for (int i = tid; i < (k << shift); i += 1024) o[i] = (float)acc[i + i / k];
    }
}

// ---- pull, quantile-slot form (k % 4 == 0) ----------------------------------------------
// The gathers of pull_tile_kernel are bound by the cache lines one wave instruction touches
// (the texture addresser and L1 take a line per cycle, not a lane): an instruction carries
// 64 / LR entries x LR lanes, each lane one value of its entry's source row, so the ~2
// entries of one row in an instruction land on ~6 of the row's eight 128-B lines, four
// instructions per step.  pull_sel_kernel therefore re-orders every destination's k
// selectors once per call: sorted ascending, and laid out so that a lane's four bytes
// (instructions i = 0..3) hold sorted positions i * k/4 + q.  Instruction i then gathers
// only the i-th quarter of every row's selected columns, ~2 lines of a row instead of ~6 (a
// model of the tile stream: 9.2 -> 5.2 distinct lines per entry at Reddit's ~2.2 entries per
// row and tile).  lmap keeps each slot's original l; pull_reduce_kernel writes the sums back
// in CBSR order.  Slot of sorted position p: lane q = p % (k/4), instruction i = p / (k/4)
// -> slot 4q + i.  Equal selectors (never produced by top-k) rank by l, so the map is a
// permutation of the k slots whatever the input.
__global__ __launch_bounds__(kBlock) void pull_sel_kernel(const uint8_t *__restrict__ sel,
                                                          uint8_t *__restrict__ sel_q,
                                                          uint8_t *__restrict__ lmap,
                                                          int64_t num_cols, int k, int kp,
                                                          int vpl) {
    __shared__ uint32_t bm[kBlock / 4 * 8];  // 256-bit column set per destination
    __shared__ uint8_t s_out[kBlock], l_out[kBlock];
    const int nd = kBlock / k;  // destinations per block (k % 4 == 0, k <= 256)
    const int tid = threadIdx.x;
    const int d = tid / k, l = tid % k;
    const int64_t c0 = (int64_t)blockIdx.x * nd;
    const int64_t c = c0 + d;
    const bool act = d < nd && c < num_cols;
    for (int i = tid; i < nd * 8; i += kBlock) bm[i] = 0u;
    __syncthreads();
    const uint32_t s = act ? sel[c * k + l] : 0u;
    if (act) atomicOr(&bm[d * 8 + (s >> 5)], 1u << (s & 31));
    __syncthreads();
    if (act) {
        int distinct = 0, rank = 0;
        for (int wd = 0; wd < 8; ++wd) {
            const uint32_t b = bm[d * 8 + wd];
            distinct += __popc(b);
            if (wd < (int)(s >> 5)) rank += __popc(b);
        }
        rank += __popc(bm[d * 8 + (s >> 5)] & ((1u << (s & 31)) - 1u));
        if (distinct < k) {  // repeated selectors: rank by (selector, l)
            rank = 0;
            for (int m = 0; m < k; ++m) {
                const uint32_t sm = sel[c * k + m];
                rank += (sm < s) || (sm == s && m < l);
            }
        }
        // part h = rank / kp (pull_q_kernel's parts), then the quantile slot inside it
        // lane q of a part holds sorted positions i * (kp / vpl) + q, i < vpl, in slots
        // vpl * q + i
        const int ql = kp / vpl, h = rank / kp, r = rank % kp;
        const int slot = h * kp + vpl * (r % ql) + r / ql;
        s_out[d * k + slot] = (uint8_t)s;
        l_out[d * k + slot] = (uint8_t)l;
    }
    __syncthreads();
    const int64_t nb = (num_cols - c0 < nd ? num_cols - c0 : nd) * (int64_t)k;
    if (tid < nb) {
        sel_q[c0 * k + tid] = s_out[tid];
        lmap[c0 * k + tid] = l_out[tid];
    }
}

// pull_sel_kernel with four selectors per thread (k % 4 == 0, 4-byte aligned selectors): one
// u32 load and store per thread instead of a byte each, and a destination's 256-bit column
// set read once per four ranks (ogbn-products-sized, k=32: 2.45M destinations).
__global__ __launch_bounds__(kBlock) void pull_sel4_kernel(const uint8_t *__restrict__ sel,
                                                           uint8_t *__restrict__ sel_q,
                                                           uint8_t *__restrict__ lmap,
                                                           int64_t num_cols, int k, int kp,
                                                           int vpl) {
    __shared__ uint32_t bm[kBlock * 8];  // 256-bit column set per destination (k >= 4)
    __shared__ uint32_t s_out[kBlock], l_out[kBlock];
    const int tpd = k / 4;      // threads per destination
    const int nd = kBlock / tpd;  // destinations per block
    const int tid = threadIdx.x;
    const int d = tid / tpd, l0 = (tid % tpd) * 4;
    const int64_t c0 = (int64_t)blockIdx.x * nd;
    const int64_t c = c0 + d;
    const bool act = d < nd && c < num_cols;
    for (int i = tid; i < nd * 8; i += kBlock) bm[i] = 0u;
    __syncthreads();
    const uint32_t w4 = act ? *reinterpret_cast<const uint32_t *>(sel + c * k + l0) : 0u;
    if (act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t sj = (w4 >> (8 * j)) & 255u;
            atomicOr(&bm[d * 8 + (sj >> 5)], 1u << (sj & 31));
        }
    }
    __syncthreads();
    if (act) {
        uint32_t wds[8];
        int distinct = 0;
#pragma unroll
        for (int wd = 0; wd < 8; ++wd) {
            wds[wd] = bm[d * 8 + wd];
            distinct += __popc(wds[wd]);
        }
        uint8_t *so = reinterpret_cast<uint8_t *>(s_out), *lo = reinterpret_cast<uint8_t *>(l_out);
        const int ql = kp / vpl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t sj = (w4 >> (8 * j)) & 255u;
            const int l = l0 + j;
            int rank = 0;
            if (distinct == k) {
                const int hi = (int)(sj >> 5);
#pragma unroll
                for (int wd = 0; wd < 8; ++wd) {
                    rank += wd < hi ? __popc(wds[wd]) : 0;
                    rank += wd == hi ? __popc(wds[wd] & ((1u << (sj & 31)) - 1u)) : 0;
                }
            } else {  // repeated selectors: rank by (selector, l)
                for (int m = 0; m < k; ++m) {
                    const uint32_t sm = sel[c * k + m];
                    rank += (sm < sj) || (sm == sj && m < l);
                }
            }
            const int h = rank / kp, r = rank % kp;
            const int slot = h * kp + vpl * (r % ql) + r / ql;
            so[d * k + slot] = (uint8_t)sj;
            lo[d * k + slot] = (uint8_t)l;
        }
    }
    __syncthreads();
    const int64_t nbytes = (num_cols - c0 < nd ? num_cols - c0 : nd) * (int64_t)k;
    if ((int64_t)tid * 4 < nbytes) {
        reinterpret_cast<uint32_t *>(sel_q + c0 * k)[tid] = s_out[tid];
        reinterpret_cast<uint32_t *>(lmap + c0 * k)[tid] = l_out[tid];
    }
}

// One tile's entry loop of pull_q_kernel: adds the tile's n_e entries (ers)
// into the fp64 accumulator, gathering from the slice's G' rows (grs).
template <int LR, int U, bool FULLD, int VPL>
__device__ __forceinline__ void pull_q_entries(double *acc, const uint8_t *sel_lds,
                                               __amdgpu_buffer_rsrc_t grs,
                                               __amdgpu_buffer_rsrc_t ers, int n_e, int D,
                                               int kp, int shift) {
    constexpr int EPI = kWave / LR;                 // entries per wave instruction
    constexpr int STEP = EPI * U;                   // entries per wave step
    constexpr int NL = (STEP + kWave - 1) / kWave;  // entry loads per step (one per lane)
    const int tid = threadIdx.x;
    const int lane = lane_id(), w = tid / kWave;
    // Lane -> (entry g, lane-in-entry q).  The texture path serves a 16-lane quarter in four
    // lane columns {c, c+4, c+8, c+12}, and lanes of one cache line that sit in one quad
    // cost extra cycles (tools/ta_probe.hip, L1-resident: 4 lines per quarter cost 4.2
    // cycles spread one lane per quad, 8.7 with a quad per line).  In one instruction the
    // LR lanes of an entry gather LR consecutive sorted columns, often one line, so they
    // are spread over the quads and gathered into columns: a column holds four consecutive
    // lanes-in-entry of one entry (LR >= 4) or all LR lanes of 4/LR neighbouring entries
    // (LR < 4; neighbours in CSR order share a source row most often).
    constexpr int EPQ = LR < 16 ? 16 / LR : 1;  // entries per 16-lane quarter
    const int lc = (lane % 16) % 4, lm = (lane % 16) / 4;  // column, lane's place in it
    constexpr bool TR = MAXK_PULL_TRANSPOSE && LR <= 16;  // an entry within a quarter
    const int g = !TR ? lane / LR
                  : LR >= 4 ? (lane / 16) * EPQ + lc / (LR / 4 > 0 ? LR / 4 : 1)
                            : (lane / 16) * EPQ + lc * (4 / LR) + lm / LR;
    const int q = !TR ? lane % LR
                  : LR >= 4 ? (lc % (LR / 4 > 0 ? LR / 4 : 1)) * 4 + lm
                            : lm % LR;
    const bool qok = q < kp / VPL;
    const int ks = pull_ks(kp, shift);
    const uint32_t Db = (uint32_t)D * 4u;
    const int stride = 16 * STEP;  // 16 waves
    const int base = w * STEP;     // entry offsets relative to the tile's first entry
    // Every step is issued the same way: no load sits under a branch, since the compiler
    // merges the counters of the two sides of a branch conservatively and then waits for
    // loads it could leave in flight.  Entries past the tile read 0 (past the descriptor),
    // their gathers get offsets past the G' descriptor (0, no memory access), their weight
    // 0, and their adds (+0.0) go to a lane-private row of the accumulator.  The loop runs
    // an even number of steps; the last issue is never consumed.
    const int nsteps = base < n_e ? (n_e - base + stride - 1) / stride : 0;
    const int idle = (w * kWave + lane) & ((1 << shift) - 1);

    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 myA[NL], myB[NL];
    float vA[U][VPL], vB[U][VPL];
    int dA[U], dB[U];
    float wA[U], wB[U];
    auto load_ent = [&](u32x2(&my)[NL], int n) {
#pragma unroll
        for (int m = 0; m < NL; ++m)
            my[m] = __builtin_amdgcn_raw_buffer_load_b64(
                ers, (int)((uint32_t)(base + n * stride + m * kWave + lane) * 8u), 0, 0);
    };
    // step n: entries from my (then reloaded for step n + 2), selectors, gathers into v
    auto issue = [&](u32x2(&my)[NL], float(&v)[U][VPL], int(&dc)[U], float(&wc)[U], int n) {
        uint32_t ex[U], ey[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = (u * EPI) / kWave;  // compile-time after unrolling
            const int src = (u * EPI + g - m * kWave) * 4;
            ex[u] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)my[m][0]);
            ey[u] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)my[m][1]);
        }
        load_ent(my, n + 2);
        uint64_t sv[U];
        bool ok[U];
        const int eb = base + n * stride + g;  // this lane group's entry of instruction 0
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ok[u] = eb + u * EPI < n_e && qok;
            const int d = ok[u] ? (int)(ex[u] >> 16) : idle;
            dc[u] = d * ks + VPL * q * ok[u];
            const uint8_t *sp = sel_lds + d * kp + (ok[u] ? q * VPL : 0);
            if constexpr (VPL == 8)
                sv[u] = *reinterpret_cast<const uint64_t *>(sp);
            else if constexpr (VPL == 4)
                sv[u] = *reinterpret_cast<const uint32_t *>(sp);
            else
                sv[u] = *reinterpret_cast<const uint16_t *>(sp);
            wc[u] = ok[u] ? __uint_as_float(ey[u]) : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = ok[u] ? (ex[u] & 0xffffu) * Db : 0x80000000u;
#pragma unroll
            for (int i = 0; i < VPL; ++i) {
                const uint32_t c = VPL == 8 ? (uint32_t)(sv[u] >> (8 * i)) & 255u
                                            : ((uint32_t)sv[u] >> (8 * i)) & 255u;
                uint32_t off = ro + c * 4u;
                if (!FULLD) off = c < (uint32_t)D ? off : 0x80000000u;  // past the buffer: 0
                v[u][i] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(grs, (int)off, 0, 0));
            }
        }
    };
    auto consume = [&](float(&v)[U][VPL], int(&dc)[U], float(&wc)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double *a = &acc[dc[u]];
#pragma unroll
            for (int i = 0; i < VPL; ++i) atomicAdd(a + i, (double)(wc[u] * v[u][i]));
        }
    };
    if (nsteps > 0) {
        load_ent(myA, 0);
        load_ent(myB, 1);
        // keep step 1's entries ahead of step 0's gathers: the loop head waits for them with
        // step 0's gathers still in flight only if they were issued first
        __builtin_amdgcn_sched_barrier(0);
        issue(myA, vA, dA, wA, 0);
        // sched_barrier: the machine scheduler would otherwise hoist a consume's multiplies
        // and the next issue's shuffles above the gathers, waiting for loads meant to stay in
        // flight
        for (int n = 0; n < nsteps; n += 2) {
            issue(myB, vB, dB, wB, n + 1);
            __builtin_amdgcn_sched_barrier(0);
            consume(vA, dA, wA);
            __builtin_amdgcn_sched_barrier(0);
            issue(myA, vA, dA, wA, n + 2);
            __builtin_amdgcn_sched_barrier(0);
            consume(vB, dB, wB);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// Where tile t's pieces live: its slice's first row and row count, its bucket's first column.
struct PullTile {
    int64_t r0, nrows, c0;
    int s0, s1;
};
// Tile t = slice * n_buckets + bucket; its entries are [tile_ptr[i], tile_ptr[i + 1]), i = t
// for a full plan, i = t's position in the tile list for a listed one (pull_q_kernel).
__device__ __forceinline__ PullTile pull_tile_of(int t, int i, const int32_t *__restrict__ tile_ptr,
                                                 int n_buckets, int rows_per_slice,
                                                 int64_t num_rows, int shift) {
    PullTile p;
    p.r0 = (int64_t)(t / n_buckets) * rows_per_slice;
    p.nrows = num_rows - p.r0 < rows_per_slice ? num_rows - p.r0 : rows_per_slice;
    p.c0 = (int64_t)(t % n_buckets) << shift;
    p.s0 = tile_ptr[i];
    p.s1 = tile_ptr[i + 1];
    return p;
}

// Part h of each destination's slot-ordered selectors (kp bytes of its k-byte row) for the
// bucket starting at column c0, loaded to registers (up to kSelRegs 16-B pieces per
// thread) and then stored to LDS.
constexpr int kSelRegs = 2;
struct PullSel {
    uint4 v[kSelRegs];
};
__device__ __forceinline__ PullSel pull_sel_load(const uint8_t *__restrict__ sel_q, int64_t c0,
                                                 int64_t num_cols, int k, int kp, int h,
                                                 int shift) {
    PullSel r;
    const int tid = threadIdx.x;
    const int rows = num_cols - c0 < (1 << shift) ? (int)(num_cols - c0) : (1 << shift);
    const uint8_t *__restrict__ selg = sel_q + c0 * k + h * kp;
    // piece i: destination i / ppr, bytes [16 * (i % ppr), +16) of its kp (ppr = kp / 16), or
    // for kp < 16 whole 16-B groups of 16 / kp destinations packed from their kp-byte parts
#pragma unroll
    for (int m = 0; m < kSelRegs; ++m) {
        const int i = tid + m * 1024;
        uint4 x = make_uint4(0u, 0u, 0u, 0u);
        if (kp % 16 == 0) {
            const int ppr = kp / 16;
            if (i < rows * ppr)
                x = *reinterpret_cast<const uint4 *>(selg + (int64_t)(i / ppr) * k + (i % ppr) * 16);
        } else {  // kp % 16 != 0 (kp % 4 == 0): 4-byte words, 4 per piece
            uint32_t wd[4];
            const int wpr = kp / 4;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int wi = i * 4 + b;
                wd[b] = wi < rows * wpr
                            ? *reinterpret_cast<const uint32_t *>(selg + (int64_t)(wi / wpr) * k +
                                                                  (wi % wpr) * 4)
                            : 0u;
            }
            x = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
        r.v[m] = x;
    }
    return r;
}
__device__ __forceinline__ void pull_sel_store(uint8_t *sel_lds, const PullSel &r, int kp,
                                               int shift) {
    const int n16 = (kp << shift) / 16;
#pragma unroll
    for (int m = 0; m < kSelRegs; ++m) {
        const int i = threadIdx.x + m * 1024;
        if (i < n16) reinterpret_cast<uint4 *>(sel_lds)[i] = r.v[m];
    }
}

// tile_out[t] is [2^shift, k] in slot order; part h fills slots [h * kp, (h + 1) * kp).
__device__ __forceinline__ void pull_flush(const double *acc, float *__restrict__ tile_out, int t,
                                           int h, int k, int kp, int shift) {
    const int ks = pull_ks(kp, shift);
    float *o = tile_out + (size_t)t * ((size_t)k << shift) + h * kp;
    const int w4 = kp / 4;
    for (int i4 = threadIdx.x; i4 < (kp << shift) / 4; i4 += 1024) {
        const int c = i4 / w4, s4 = i4 % w4;
        const double *a = &acc[c * ks + 4 * s4];
        *reinterpret_cast<float4 *>(o + (size_t)c * k + 4 * s4) =
            make_float4((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
    }
}

// Parts: with H = k / kp parts, destination c's slots split by sorted position into H
// groups of kp (part h: the h-th kp smallest selectors), and one workgroup sums one part of
// one tile: the accumulator holds kp slots per destination, so a bucket holds H times the
// destinations and a source row meets ~H times fewer buckets; each part's gathers cover
// only its share of a row's columns (the h-th kp order statistics of every entry).  The
// tile's entries are read H times (kp: maxk_pull_shift, transpose.hip).
// One 1024-thread workgroup per (tile, part), as pull_tile_kernel (fp64 LDS accumulator of
// the bucket, its slot-ordered selector rows copied next to it), with:
//  * quantile slots (pull_sel_kernel): lane q's u32 selector word holds its four
//    instructions' columns;
//  * a two-step software pipeline: step n's gathers are issued before step n-1's adds, and
//    the entries two steps ahead, so a wave keeps 2 x 4U gathers in flight and never waits
//    on loads it has just issued (the one-step loop waited for every load at its head);
//  * the G' gathers through a wave-uniform buffer descriptor over the slice's rows with
//    32-bit offsets (no 64-bit address math per value); a selector >= D (possible only
//    when D < 256, !FULLD) gets an offset past the descriptor, and the hardware returns 0;
//  * tiles in XCD order (MAXK_PULL_XCD): XCD x runs the x-th eighth of the tile sequence
//    in order, so each XCD's L2 holds the one slice it works on instead of every XCD
//    pulling every slice.
template <int LR, int U, bool FULLD, int VPL>
__global__ __launch_bounds__(1024) void pull_q_kernel(
    const float *__restrict__ Gp, const uint8_t *__restrict__ sel_q,
    const int32_t *__restrict__ tile_ptr, const uint2 *__restrict__ ent,
    float *__restrict__ tile_out, int64_t num_cols, int n_buckets, int n_tiles,
    int rows_per_slice, int64_t num_rows, int D, int k, int kp, int shift,
    const int32_t *__restrict__ tile_list) {
    // tile_list (maxk_sspmm_backward_pull_tiles): only the listed tiles run; tile_ptr then
    // holds their entry ranges and tile_out their partials, both by list position
    extern __shared__ double acc[];  // [ks << shift], then [kp << shift] selector bytes
    const int tid = threadIdx.x;
    const int ks = pull_ks(kp, shift);
    const int H = k / kp;
    const int tp = MAXK_PULL_XCD ? xcd_contiguous_block(blockIdx.x, gridDim.x) : blockIdx.x;
    if (tp >= n_tiles * H) return;  // the XCD grid's padding
    const int ti = tp / H, h = tp % H;
    const int t = tile_list ? tile_list[ti] : ti;
    const PullTile p = pull_tile_of(t, ti, tile_ptr, n_buckets, rows_per_slice, num_rows, shift);
    uint8_t *sel_lds = reinterpret_cast<uint8_t *>(acc + (ks << shift));
    for (int i = tid; i < (ks << shift); i += 1024) acc[i] = 0.0;
    pull_sel_store(sel_lds, pull_sel_load(sel_q, p.c0, num_cols, k, kp, h, shift), kp, shift);
    __syncthreads();
    const auto grs =
        wave_buffer(Gp + p.r0 * D, (uint32_t)(p.nrows > 0 ? p.nrows : 0) * (uint32_t)D * 4u);
    const auto ers = wave_buffer(ent + p.s0, (uint32_t)(p.s1 - p.s0) * 8u);
    pull_q_entries<LR, U, FULLD, VPL>(acc, sel_lds, grs, ers, p.s1 - p.s0, D, kp, shift);
    __syncthreads();
    pull_flush(acc, tile_out, ti, h, k, kp, shift);
}

// grad_cbsr rows of bucket j = the sum of its slices' tiles, in slice order.  With lmap
// (pull_q_kernel's slot order, k % 4 == 0) slot f of row c goes to l = lmap[c * k + f].
// Listed tiles (bucket_ptr != nullptr, k % 4 == 0): bucket j's tiles are the list positions
// bucket_tiles[bucket_ptr[j] .. bucket_ptr[j + 1]), in slice order (none: the sum is 0);
// accumulate adds the sum onto grad_cbsr instead of storing it.
__global__ __launch_bounds__(kBlock) void pull_reduce_kernel(const float *__restrict__ tile_out,
                                                             const uint8_t *__restrict__ lmap,
                                                             float *__restrict__ grad_cbsr,
                                                             int64_t num_cols, int n_buckets,
                                                             int slices, int k, int shift,
                                                             const int32_t *__restrict__ bucket_ptr,
                                                             const int32_t *__restrict__ bucket_tiles,
                                                             int accumulate) {
    const int j = blockIdx.x;
    const int64_t c0 = (int64_t)j << shift;
    const int rows = num_cols - c0 < (1 << shift) ? (int)(num_cols - c0) : (1 << shift);
    const int i = blockIdx.y * kBlock + threadIdx.x;
    const int nf = rows * k;  // floats of this bucket; tiles and c0 * k are 16-B aligned
    if (i * 4 >= nf) return;
    const size_t n4 = ((size_t)k << shift) / 4;
    const float4 *to = reinterpret_cast<const float4 *>(tile_out);
    if (i * 4 + 4 > nf) {  // k % 4 != 0: the bucket's last 1..3 floats
        const int f0 = i * 4;
        for (int f = f0; f < nf; ++f) {
            float a = tile_out[(size_t)j * n4 * 4 + f];
            for (int s = 1; s < slices; ++s) a += tile_out[((size_t)s * n_buckets + j) * n4 * 4 + f];
            grad_cbsr[c0 * k + f] = a;
        }
        return;
    }
    float4 a;
    if (bucket_ptr) {
        a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int q = bucket_ptr[j]; q < bucket_ptr[j + 1]; ++q) {
            const float4 b = to[(size_t)bucket_tiles[q] * n4 + i];
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
    } else {
        a = to[(size_t)j * n4 + i];
        for (int s = 1; s < slices; ++s) {
            const float4 b = to[((size_t)s * n_buckets + j) * n4 + i];
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
    }
    if (lmap) {  // four slots of one row (k % 4 == 0) back to their l
        const size_t f0 = (size_t)c0 * k + (size_t)i * 4;
        const uint32_t m = *reinterpret_cast<const uint32_t *>(lmap + f0);
        float *row = grad_cbsr + (f0 / k) * k;
        if (accumulate) {
            a.x += row[m & 255u];
            a.y += row[(m >> 8) & 255u];
            a.z += row[(m >> 16) & 255u];
            a.w += row[m >> 24];
        }
        row[m & 255u] = a.x;
        row[(m >> 8) & 255u] = a.y;
        row[(m >> 16) & 255u] = a.z;
        row[m >> 24] = a.w;
        return;
    }
    reinterpret_cast<float4 *>(grad_cbsr + c0 * k)[i] = a;
}

// Auto item size: ~`per_slot` items per resident wave slot on the device's CUs, in [256, 2048].
int bwd_chunk(int64_t num_rows, int64_t num_e, int32_t chunk, int per_slot) {
    if (chunk > 0) return chunk;
    const int64_t total = num_rows + num_e;
    int64_t c = ceil_div(total, device_cus() * 32 * per_slot);
    c = c < 256 ? 256 : (c > 2048 ? 2048 : c);
    return (int)c;
}

int n_items_for(int64_t rows, int64_t num_e, int chunk) {
    const int64_t n = ceil_div(rows + num_e, chunk);
    return (int)(n > 0 ? n : 1);
}

// Loads in flight per lane ("depth" U): one wave step covers `per_step` edges (or
// contribution rows), a batch U steps.  Deep batches keep more bytes in flight on long
// rows; on short rows they are mostly masked lanes.  Largest U in [lo, hi] (powers of
// two) whose batch still fits an average row (measured: products deg 50 -> 4, Reddit /
// proteins deg 500-600 -> 16 for phase 1; 4 / 8 for phase 2).
int pick_depth(int64_t num_e, int64_t rows, int per_step, int lo, int hi) {
    const int64_t avg = rows > 0 ? num_e / rows : 0;
    int u = lo;
    while (u < hi && (int64_t)per_step * u * 2 <= avg) u <<= 1;
    return u;
}

template <int MODE>
int launch_push(hipStream_t s, const int32_t *row_ptr, const int32_t *col_idx,
                const float *edge_val, const float *grad, const float *row_div,
                const uint8_t *cbsr_idx, float *dst, int nr, int64_t num_cols, int64_t num_e,
                int D, int k, int chunk, const uint8_t *esel = nullptr) {
    const int n_items = n_items_for(nr, num_e, chunk);
    const int64_t blocks = ceil_div(n_items, kWavesPerBlock);
    const dim3 grid((unsigned)(MAXK_P1_XCD ? xcd_grid(blocks) : blocks));
    if (MODE == kStore && ((MAXK_BWD_X4 && k % 4 == 0) || esel)) {
        const int lr = lanes_per_edge(k / 4);
        const int u = MAXK_X4_U > 0 ? MAXK_X4_U : pick_depth(num_e, nr, kWave / lr, 4, 16);
        const bool wide = num_cols >= (1 << 24);  // selector offsets need a 32-bit multiply
        switch (lr) {
#define MAXK_GO(LRV, UV, MV)                                                                 \
    hipLaunchKernelGGL((sspmm_bwd_kernel<LRV, UV, MV>), grid, dim3(kBlock), 0, s, row_ptr,   \
                       col_idx, edge_val, grad, row_div, cbsr_idx, dst, nr, num_e, D, k,     \
                       chunk, n_items, esel)
#define MAXK_CASE(LRV)                          \
    case LRV:                                   \
        if (esel && u <= 4)                     \
            MAXK_GO(LRV, 4, kStoreX4S);         \
        else if (esel && u <= 8)                \
            MAXK_GO(LRV, 8, kStoreX4S);         \
        else if (esel)                          \
            MAXK_GO(LRV, 16, kStoreX4S);        \
        else if (wide)                          \
            MAXK_GO(LRV, 8, kStoreX4W);         \
        else if (u <= 4)                        \
            MAXK_GO(LRV, 4, kStoreX4);          \
        else if (u <= 8)                        \
            MAXK_GO(LRV, 8, kStoreX4);          \
        else                                    \
            MAXK_GO(LRV, 16, kStoreX4);         \
        break;
            MAXK_CASE(1)
            MAXK_CASE(2)
            MAXK_CASE(4)
            MAXK_CASE(8)
            MAXK_CASE(16)
            MAXK_CASE(32)
            MAXK_CASE(64)
#undef MAXK_CASE
#undef MAXK_GO
            default:
                set_error("unsupported lane group");
                return MAXK_ERR_INVALID;
        }
        MAXK_LAUNCHED("sspmm_bwd_kernel");
        return MAXK_OK;
    }
    switch (lanes_per_edge(k)) {
#define MAXK_CASE(KGV)                                                                        \
    case KGV:                                                                                 \
        hipLaunchKernelGGL((sspmm_bwd_kernel<KGV, (KGV >= 8 ? MAXK_BWD_U : 4), MODE>), grid,  \
                           dim3(kBlock), 0, s, row_ptr, col_idx, edge_val, grad, row_div,     \
                           cbsr_idx, dst, nr, num_e, D, k, chunk, n_items, nullptr);          \
        break;
        MAXK_CASE(1)
        MAXK_CASE(2)
        MAXK_CASE(4)
        MAXK_CASE(8)
        MAXK_CASE(16)
        MAXK_CASE(32)
        MAXK_CASE(64)
#undef MAXK_CASE
        default:
            set_error("unsupported lane group");
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED("sspmm_bwd_kernel");
    return MAXK_OK;
}

bool vec_sum(int k) { return k >= 4 && (k & (k - 1)) == 0; }

struct CscLayout {
    int chunk, n_items;
    size_t t_bytes, slab_off, row_off, total;
};

CscLayout csc_layout(int64_t num_cols, int64_t num_e, int k, int chunk) {
    CscLayout L{};
    L.chunk = bwd_chunk(num_cols, num_e, chunk, MAXK_P2_ITEMS);
    L.n_items = n_items_for(num_cols, num_e, L.chunk);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    L.t_bytes = al((size_t)(num_e + 1) * k * sizeof(float));  // + dummy row for masked lanes
    L.slab_off = L.t_bytes;
    L.row_off = L.slab_off + al((size_t)L.n_items * k * sizeof(float));
    L.total = L.row_off + al((size_t)L.n_items * sizeof(int32_t));
    return L;
}

int check_common(int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t D, int32_t k,
                 int32_t chunk) {
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(D >= 1 && D <= kMaxDim, "dim_origin must be in [1,256], got %d", D);
    MAXK_REQUIRE(k >= 1 && k <= D, "dim_k must be in [1,dim_origin], got %d", k);
    MAXK_REQUIRE(chunk >= 0, "chunk_edges must be >= 0");
    MAXK_REQUIRE(num_cols * (int64_t)k < (1LL << 31), "num_cols*k too large");
    return MAXK_OK;
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" size_t maxk_sspmm_backward_workspace_size(int64_t num_rows, int64_t num_cols,
                                                     int64_t num_e, int32_t dim_origin,
                                                     int32_t dim_k, int32_t chunk_edges) {
    (void)num_rows; (void)num_cols; (void)num_e; (void)dim_origin; (void)dim_k;
    (void)chunk_edges;
    return 0;
}

extern "C" int maxk_sspmm_backward(const int32_t *row_ptr, const int32_t *col_idx,
                                   const float *edge_val, const float *grad_out,
                                   const float *row_div, const uint8_t *cbsr_idx,
                                   float *grad_cbsr, int64_t num_rows, int64_t num_cols,
                                   int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                   int32_t chunk_edges, void *workspace, size_t workspace_bytes,
                                   void *stream) {
    (void)workspace; (void)workspace_bytes;
    clear_error();
    if (int rc = check_common(num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges)) return rc;
    hipStream_t s = as_stream(stream);
    if (num_cols > 0) {
        MAXK_REQUIRE(grad_cbsr != nullptr, "grad_cbsr must not be NULL");
        if (int rc = zero_words(grad_cbsr, num_cols * dim_k, s)) return rc;
    }
    if (num_rows == 0 || num_e == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && col_idx && edge_val && grad_out && cbsr_idx,
                 "CSR/grad/selector pointers must not be NULL");
    MAXK_REQUIRE(num_cols > 0, "edges present but num_cols == 0");
    return launch_push<kAtomic>(s, row_ptr, col_idx, edge_val, grad_out, row_div, cbsr_idx,
                                grad_cbsr, (int)num_rows, num_cols, num_e, dim_origin, dim_k,
                                bwd_chunk(num_rows, num_e, chunk_edges, MAXK_P1_ITEMS));
}

extern "C" size_t maxk_sspmm_backward_csc_workspace_size(int64_t num_rows, int64_t num_cols,
                                                         int64_t num_e, int32_t dim_origin,
                                                         int32_t dim_k, int32_t chunk_edges) {
    (void)num_rows; (void)dim_origin;
    if (num_cols < 0 || num_e < 0 || dim_k <= 0) return 0;
    return csc_layout(num_cols, num_e, dim_k, chunk_edges).total;
}

namespace maxk {
namespace {
// edge_sel (k % 4 == 0): phase 1 reads each edge's selectors from this per-edge stream instead
// of gathering them from cbsr_idx (push_x4, ES).
int csc_impl(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
             const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
             const uint8_t *edge_sel, const int32_t *col_ptr, const int32_t *csc_eid,
             float *grad_cbsr, int64_t num_rows, int64_t num_cols, int64_t num_e,
             int32_t dim_origin, int32_t dim_k, int32_t chunk_edges, void *workspace,
             size_t workspace_bytes, void *stream) {
    if (int rc = check_common(num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges)) return rc;
    hipStream_t s = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    MAXK_REQUIRE(grad_cbsr && col_ptr, "grad_cbsr/col_ptr must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (row_ptr && col_idx && edge_val && grad_out &&
                                (cbsr_idx || edge_sel) && csc_eid),
                 "CSR/grad/selector/transpose pointers must not be NULL");
    const CscLayout L = csc_layout(num_cols, num_e, dim_k, chunk_edges);
    MAXK_REQUIRE(workspace && workspace_bytes >= L.total,
                 "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    char *ws = reinterpret_cast<char *>(workspace);
    float *T = reinterpret_cast<float *>(ws);
    float *slab = reinterpret_cast<float *>(ws + L.slab_off);
    int32_t *slab_row = reinterpret_cast<int32_t *>(ws + L.row_off);
    const int k = dim_k;
    if (num_e > 0 && num_rows > 0) {
        if (int rc = launch_push<kStore>(s, row_ptr, col_idx, edge_val, grad_out, row_div,
                                         cbsr_idx, T, (int)num_rows, num_cols, num_e,
                                         dim_origin, k,
                                         bwd_chunk(num_rows, num_e, chunk_edges, MAXK_P1_ITEMS),
                                         edge_sel))
            return rc;
    }
    const int64_t blocks = ceil_div(L.n_items, kWavesPerBlock);
    const dim3 grid((unsigned)(MAXK_XCD_SUM ? xcd_grid(blocks) : blocks));
    const int nc = (int)num_cols;
    const bool staged = MAXK_CSC_STAGE && L.chunk <= kCscStage;
    const size_t lds = (size_t)kWavesPerBlock * L.chunk * sizeof(int32_t);
    // T rows of whole 128-B lines: non-temporal reads (t_load4)
    const bool nt = MAXK_T_LOAD_NT && k % 32 == 0;
    if (staged && vec_sum(k) && k >= 16 && k <= 64 &&
        num_e < (int64_t)MAXK_CSC_GROUP_DEG * num_cols) {
        // few slots per destination: lane groups per destination (csc_groups)
        if (nt)
            hipLaunchKernelGGL((csc_sum_kernel<true, 64, MAXK_CSC_GROUP_U, true, true, true>),
                               grid, dim3(kBlock), lds, s, col_ptr, csc_eid, T, grad_cbsr, slab,
                               slab_row, nc, num_e, k, L.chunk, L.n_items);
        else
            hipLaunchKernelGGL((csc_sum_kernel<true, 64, MAXK_CSC_GROUP_U, true, true>), grid,
                               dim3(kBlock), lds, s, col_ptr, csc_eid, T, grad_cbsr, slab,
                               slab_row, nc, num_e, k, L.chunk, L.n_items);
    } else if (vec_sum(k)) {
        const int rows_per_step = kWave / (k / 4);
        const int u = MAXK_SUM_U > 0 ? MAXK_SUM_U
                                     : pick_depth(num_e, num_cols, rows_per_step, 2, 8);
#define MAXK_SUM_LAUNCH(UV)                                                                  \
    if (staged && nt)                                                                        \
        hipLaunchKernelGGL((csc_sum_kernel<true, 64, UV, true, false, true>), grid,          \
                           dim3(kBlock), lds, s, col_ptr, csc_eid, T, grad_cbsr, slab,       \
                           slab_row, nc, num_e, k, L.chunk, L.n_items);                      \
    else if (staged)                                                                         \
        hipLaunchKernelGGL((csc_sum_kernel<true, 64, UV, true>), grid, dim3(kBlock), lds, s, \
                           col_ptr, csc_eid, T, grad_cbsr, slab, slab_row, nc, num_e, k,     \
                           L.chunk, L.n_items);                                              \
    else                                                                                     \
        hipLaunchKernelGGL((csc_sum_kernel<true, 64, UV, false>), grid, dim3(kBlock), 0, s,  \
                           col_ptr, csc_eid, T, grad_cbsr, slab, slab_row, nc, num_e, k,     \
                           L.chunk, L.n_items)
        if (u <= 2)
            MAXK_SUM_LAUNCH(2);
        else if (u <= 4)
            MAXK_SUM_LAUNCH(4);
        else
            MAXK_SUM_LAUNCH(8);
#undef MAXK_SUM_LAUNCH
    } else {
        switch (lanes_per_edge(k)) {
#define MAXK_CASE(KGV)                                                                        \
    case KGV:                                                                                 \
        if (staged)                                                                           \
            hipLaunchKernelGGL((csc_sum_kernel<false, KGV, 4, true>), grid, dim3(kBlock), lds, \
                               s,                                                             \
                               col_ptr, csc_eid, T, grad_cbsr, slab, slab_row, nc, num_e, k,  \
                               L.chunk, L.n_items);                                           \
        else                                                                                  \
            hipLaunchKernelGGL((csc_sum_kernel<false, KGV, 4, false>), grid, dim3(kBlock), 0, \
                               s, col_ptr, csc_eid, T, grad_cbsr, slab, slab_row, nc, num_e,  \
                               k, L.chunk, L.n_items);                                        \
        break;
            MAXK_CASE(1)
            MAXK_CASE(2)
            MAXK_CASE(4)
            MAXK_CASE(8)
            MAXK_CASE(16)
            MAXK_CASE(32)
            MAXK_CASE(64)
#undef MAXK_CASE
            default:
                set_error("unsupported lane group");
                return MAXK_ERR_INVALID;
        }
    }
    MAXK_LAUNCHED("csc_sum_kernel");
    return launch_slab_fixup<1>(slab, slab_row, grad_cbsr, k, L.n_items, s);
}

// edge_sel[e * k + l] = cbsr_idx[col_idx[e] * k + l]: wb = 16, 4 or 1 bytes per thread (the
// widest that divides k and both arrays' alignment)
__global__ __launch_bounds__(kBlock) void edge_sel_kernel(const int32_t *__restrict__ col_idx,
                                                          const uint8_t *__restrict__ cbsr_idx,
                                                          uint8_t *__restrict__ edge_sel,
                                                          int64_t n_words, int k, int wb) {
    // grid-stride: the launch caps its grid (num_e * k one-byte words can pass the
    // 2^32 - 1 threads of one grid dimension)
    const int wpe = k / wb;  // words per edge
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n_words; i += stride) {
        const int64_t e = i / wpe;
        const int w = (int)(i % wpe);
        const size_t src = (size_t)(uint32_t)col_idx[e] * k + (size_t)w * wb;
        if (wb == 16)
            reinterpret_cast<uint4 *>(edge_sel)[i] =
                *reinterpret_cast<const uint4 *>(cbsr_idx + src);
        else if (wb == 4)
            reinterpret_cast<uint32_t *>(edge_sel)[i] =
                *reinterpret_cast<const uint32_t *>(cbsr_idx + src);
        else
            edge_sel[i] = cbsr_idx[src];
    }
}
}  // namespace
}  // namespace maxk

extern "C" int maxk_sspmm_backward_csc(const int32_t *row_ptr, const int32_t *col_idx,
                                       const float *edge_val, const float *grad_out,
                                       const float *row_div, const uint8_t *cbsr_idx,
                                       const int32_t *col_ptr, const int32_t *csc_eid,
                                       float *grad_cbsr, int64_t num_rows, int64_t num_cols,
                                       int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                       int32_t chunk_edges, void *workspace,
                                       size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_e == 0 || cbsr_idx, "cbsr_idx must not be NULL");
    return csc_impl(row_ptr, col_idx, edge_val, grad_out, row_div, cbsr_idx, nullptr, col_ptr,
                    csc_eid, grad_cbsr, num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges,
                    workspace, workspace_bytes, stream);
}

extern "C" int maxk_sspmm_backward_csc_sel(const int32_t *row_ptr, const int32_t *col_idx,
                                           const float *edge_val, const float *grad_out,
                                           const float *row_div, const uint8_t *edge_sel,
                                           const int32_t *col_ptr, const int32_t *csc_eid,
                                           float *grad_cbsr, int64_t num_rows, int64_t num_cols,
                                           int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                           int32_t chunk_edges, void *workspace,
                                           size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(dim_k % 4 == 0, "edge selectors need dim_k %% 4 == 0, got %d", dim_k);
    MAXK_REQUIRE(num_e == 0 || edge_sel, "edge_sel must not be NULL");
    MAXK_REQUIRE(((uintptr_t)edge_sel & 3) == 0, "edge_sel must be 4-B aligned");
    return csc_impl(row_ptr, col_idx, edge_val, grad_out, row_div, nullptr, edge_sel, col_ptr,
                    csc_eid, grad_cbsr, num_rows, num_cols, num_e, dim_origin, dim_k, chunk_edges,
                    workspace, workspace_bytes, stream);
}

// edge_sel_kernel's grid: one thread per word up to 64 workgroups per CU, then grid-stride
extern "C" int64_t maxk_edge_selectors_blocks(int64_t n_words) {
    const int64_t b = ceil_div(n_words < 0 ? 0 : n_words, (int64_t)kBlock);
    const int64_t cap = device_cus() * 64;
    return b < cap ? b : cap;
}

extern "C" int maxk_edge_selectors(const int32_t *col_idx, const uint8_t *cbsr_idx,
                                   int64_t num_e, int32_t dim_k, uint8_t *edge_sel, void *stream) {
    clear_error();
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= kMaxDim, "dim_k must be in [1,256], got %d", dim_k);
    MAXK_REQUIRE(num_e >= 0 && num_e * (int64_t)dim_k < (1LL << 40), "num_e out of range");
    if (num_e == 0) return MAXK_OK;
    MAXK_REQUIRE(col_idx && cbsr_idx && edge_sel, "pointers must not be NULL");
    // any k and alignment: the widest word that divides k and both arrays' alignment (the
    // _sel entry points accept 4-B aligned streams, and this is their fallback past 2^24 columns)
    const uintptr_t al = (uintptr_t)edge_sel | (uintptr_t)cbsr_idx;
    const int wb = dim_k % 16 == 0 && (al & 15) == 0 ? 16 : dim_k % 4 == 0 && (al & 3) == 0 ? 4 : 1;
    const int64_t n_words = num_e * (dim_k / wb);
    hipLaunchKernelGGL(edge_sel_kernel, dim3((unsigned)maxk_edge_selectors_blocks(n_words)), dim3(kBlock), 0,
                       as_stream(stream), col_idx, cbsr_idx, edge_sel, n_words, dim_k, wb);
    MAXK_LAUNCHED("edge_sel_kernel");
    return MAXK_OK;
}

// Bucketed phase 2: entries per part (~MAXK_BUCKET_PARTS parts per CU, at least 16384).
int bucket_part(int64_t num_e) {
    int64_t p = ceil_div(num_e, device_cus() * MAXK_BUCKET_PARTS);
    return (int)(p < 16384 ? 16384 : p);
}

static int bucket_phase2(hipStream_t s, const float *T, const int32_t *bucket_ptr,
                         const int32_t *bucket_row, const uint16_t *bucket_dst, int bucket_shift,
                         float *grad_cbsr, void *workspace, int64_t num_cols, int64_t num_e,
                         int k);

// Workspace of the bucketed phase 2 (bsort): T [E + 1, k] floats, then 2 slab rows of
// 2^shift * k floats per part (the parts' first and last buckets)
static size_t bucket_workspace_size(int64_t num_e, int32_t dim_k) {
    if (num_e < 0 || dim_k <= 0) return 0;
    const int shift = maxk_bucket_shift(dim_k);
    const size_t t = ((size_t)(num_e + 1) * dim_k * sizeof(float) + 255) & ~(size_t)255;
    const size_t parts = (size_t)ceil_div(num_e, bucket_part(num_e));
    return t + parts * 2 * ((size_t)dim_k << shift) * sizeof(float);
}

// Phase 2 of the bucketed forms: bucket_sum_kernel over the bucket list (entry i reads T row
// bucket_row[i]) and the fixup of the buckets split over parts.  The slab sits after T in
// the workspace (bucket_workspace_size).
static int bucket_phase2(hipStream_t s, const float *T, const int32_t *bucket_ptr,
                         const int32_t *bucket_row, const uint16_t *bucket_dst, int bucket_shift,
                         float *grad_cbsr, void *workspace, int64_t num_cols, int64_t num_e,
                         int k) {
    const int64_t nb = (num_cols + (1LL << bucket_shift) - 1) >> bucket_shift;
    const int part = bucket_part(num_e);
    const int64_t parts = ceil_div(num_e, part);
    float *slab = reinterpret_cast<float *>(
        reinterpret_cast<char *>(workspace) +
        (((size_t)(num_e + 1) * k * sizeof(float) + 255) & ~(size_t)255));
    const int nc = (int)num_cols, ne = (int)num_e, nbi = (int)nb;
    const int32_t *bucket_eid = bucket_row;
    switch (parts > 0 ? lanes_per_edge(k / 4) : 0) {
        case 0:
            break;
#define MAXK_CASE(LRV)                                                                          \
    case LRV:                                                                                   \
        hipLaunchKernelGGL((bucket_sum_kernel<LRV, MAXK_BUCKET_U>), dim3((unsigned)parts),      \
                           dim3(1024), 0, s, T, bucket_ptr, bucket_eid, bucket_dst, grad_cbsr,  \
                           slab, nc, nbi, ne, k, bucket_shift, part);                           \
        break;
        MAXK_CASE(1)
        MAXK_CASE(2)
        MAXK_CASE(4)
        MAXK_CASE(8)
        MAXK_CASE(16)
        MAXK_CASE(32)
        MAXK_CASE(64)
#undef MAXK_CASE
        default:
            set_error("unsupported lane group");
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED("bucket_sum_kernel");
    hipLaunchKernelGGL(bucket_fixup_kernel,
                       dim3((unsigned)nb, (unsigned)ceil_div(((int64_t)k << bucket_shift) / 4, kBlock)),
                       dim3(kBlock), 0, s, bucket_ptr, slab, grad_cbsr, nc, k, bucket_shift, part);
    MAXK_LAUNCHED("bucket_fixup_kernel");
    return MAXK_OK;
}

extern "C" int32_t maxk_bsort_window(int32_t dim_k) {
    if (dim_k <= 0 || dim_k % 4 != 0 || dim_k > kMaxDim) return -1;
    const int w = kBsortStageFloats / dim_k;
    return w > 65536 ? 65536 : w;
}

extern "C" size_t maxk_sspmm_backward_bsort_workspace_size(int64_t num_rows, int64_t num_cols,
                                                           int64_t num_e, int32_t dim_origin,
                                                           int32_t dim_k) {
    (void)num_rows; (void)num_cols; (void)dim_origin;
    return bucket_workspace_size(num_e, dim_k);
}

extern "C" int maxk_sspmm_backward_bsort(
    const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val, const float *grad_out,
    const float *row_div, const uint8_t *cbsr_idx, const uint8_t *edge_sel,
    const int32_t *bucket_ptr, const int32_t *bucket_pos, const uint16_t *bucket_dst,
    const uint16_t *win_src, const int32_t *edge_row, int32_t bucket_shift, float *grad_cbsr,
    int64_t num_rows,
    int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k, void *workspace,
    size_t workspace_bytes, void *stream) {
    clear_error();
    if (int rc = check_common(num_rows, num_cols, num_e, dim_origin, dim_k, 0)) return rc;
    MAXK_REQUIRE(dim_k % 4 == 0, "window-sorted backward needs dim_k %% 4 == 0, got %d", dim_k);
    MAXK_REQUIRE(bucket_shift >= 0 && bucket_shift <= 16 &&
                     ((int64_t)(dim_k + 1) << bucket_shift) <= kBucketAccDoubles,
                 "bucket_shift %d too large for dim_k %d (2^shift * (k + 1) <= %d)", bucket_shift,
                 dim_k, kBucketAccDoubles);
    hipStream_t s = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    MAXK_REQUIRE(grad_cbsr && bucket_ptr, "grad_cbsr/bucket_ptr must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (row_ptr && edge_val && grad_out && (cbsr_idx || edge_sel) &&
                                (edge_sel || col_idx) && bucket_pos && bucket_dst && win_src &&
                                edge_row),
                 "CSR/grad/selector/plan pointers must not be NULL");
    MAXK_REQUIRE(!edge_sel || ((uintptr_t)edge_sel & 3) == 0, "edge_sel must be 4-B aligned");
    const size_t need = maxk_sspmm_backward_bsort_workspace_size(num_rows, num_cols, num_e,
                                                                 dim_origin, dim_k);
    MAXK_REQUIRE(workspace && workspace_bytes >= need,
                 "workspace too small: need %zu bytes, got %zu", need, workspace_bytes);
    float *T = reinterpret_cast<float *>(workspace);
    const int k = dim_k;
    if (num_e > 0) {
        MAXK_REQUIRE(num_rows > 0, "edges present but num_rows == 0");
        const int W = maxk_bsort_window(k);
        const int64_t nwin = ceil_div(num_e, W);
        const dim3 grid((unsigned)(MAXK_P1_XCD ? xcd_grid(nwin) : nwin));
        const int ne = (int)num_e;
        switch (lanes_per_edge(k / 4)) {
#define MAXK_GO(LRV, ESV)                                                                         \
    hipLaunchKernelGGL((bsort_push_kernel<LRV, MAXK_BSORT_U, ESV>), grid, dim3(kBsortThreads), 0, \
                       s, edge_row, col_idx, edge_val, grad_out, row_div, cbsr_idx, edge_sel,    \
                       win_src, T, ne, dim_origin, k, W)
#define MAXK_CASE(LRV)          \
    case LRV:                   \
        if (edge_sel)           \
            MAXK_GO(LRV, true); \
        else                    \
            MAXK_GO(LRV, false); \
        break;
            MAXK_CASE(1)
            MAXK_CASE(2)
            MAXK_CASE(4)
            MAXK_CASE(8)
            MAXK_CASE(16)
            MAXK_CASE(32)
            MAXK_CASE(64)
#undef MAXK_CASE
#undef MAXK_GO
            default:
                set_error("unsupported lane group");
                return MAXK_ERR_INVALID;
        }
        MAXK_LAUNCHED("bsort_push_kernel");
    }
    return bucket_phase2(s, T, bucket_ptr, bucket_pos, bucket_dst, bucket_shift, grad_cbsr,
                         workspace, num_cols, num_e, k);
}

// ---- pull backward: C entry ------------------------------------------------------------
namespace maxk {
// Parts of pull_q_kernel for k and a plan's bucket shift: the fewest H (k % (4H) == 0) whose
// accumulator [(k/H + 1) << shift] doubles and selector rows [k/H << shift] bytes fit the
// LDS; 0 if none does.
int pull_parts(int k, int shift) {
    for (int H = 1; H <= k / 4; H *= 2) {
        if (k % (4 * H)) break;
        const int kp = k / H;
        if ((((size_t)kp * 8 + kp) << shift) <= kPullLdsBytes) return H;  // unpadded fits
    }
    return 0;
}
}  // namespace maxk

namespace maxk {
namespace {
// Workspace of the pull for `tiles` tile partials of 2^shift destinations each: G' (row_div),
// the partials, slot-ordered selectors and their l map.  The size functions pass the largest
// shift any plan may carry (tiles x 2^shift never shrinks as the shift grows: the columns are
// rounded up to whole buckets), a call its own plan's shift.
size_t pull_workspace(int64_t num_rows, int64_t num_cols, int32_t dim_origin, int32_t dim_k,
                      int64_t tiles, int shift) {
    const size_t gp = ((size_t)num_rows * dim_origin * sizeof(float) + 255) & ~(size_t)255;
    const size_t tb = (size_t)tiles * ((size_t)dim_k << shift) * sizeof(float);
    // slot-ordered selectors and their l map (pull_sel_kernel), k % 4 == 0
    const size_t selq = dim_k % 4 == 0 ? 2 * (((size_t)num_cols * dim_k + 255) & ~(size_t)255) : 0;
    return gp + tb + selq;
}

int pull_impl(const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
              const int32_t *tile_ptr, const uint32_t *ent, int32_t bucket_shift, int32_t slices,
              bool listed, const int32_t *tile_list, int32_t n_list, const int32_t *bucket_ptr,
              const int32_t *bucket_tiles, int32_t accumulate, float *grad_cbsr, int64_t num_rows,
              int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k, void *workspace,
              size_t workspace_bytes, void *stream) {
    if (int rc = check_common(num_rows, num_cols, num_e, dim_origin, dim_k, 0)) return rc;
    MAXK_REQUIRE(dim_k % 4 == 0 || dim_k <= 64,
                 "pull backward needs dim_k %% 4 == 0 or dim_k <= 64, got %d", dim_k);
    MAXK_REQUIRE(dim_origin % 4 == 0, "pull backward needs dim_origin %% 4 == 0, got %d",
                 dim_origin);
    const bool v4 = dim_k % 4 == 0;
    // quantile-slot form with H parts (k % 4 == 0), else the one-l-per-lane pull_tile_kernel
    const int parts = MAXK_PULL_Q && v4 && bucket_shift >= 4 && bucket_shift <= 15
                          ? pull_parts(dim_k, bucket_shift)
                          : 0;
    const int max_shift = std::max(maxk_bucket_shift(dim_k), maxk_pull_shift(dim_k));
    MAXK_REQUIRE(bucket_shift >= 4 && bucket_shift <= 15 && bucket_shift <= max_shift &&
                     (parts > 0 || bucket_shift <= maxk_bucket_shift(dim_k)),
                 "bucket_shift %d out of range [4, min(15, %d)] for dim_k %d", bucket_shift,
                 max_shift, dim_k);
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    MAXK_REQUIRE(slices >= 1 && slices * nb < (1LL << 31), "slices %d out of range", slices);
    const int64_t rps = (num_rows + slices - 1) / slices;
    MAXK_REQUIRE(rps <= 65536, "%d slices leave %lld rows per slice (max 65536)", slices,
                 (long long)rps);
    hipStream_t s = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    MAXK_REQUIRE(grad_cbsr && tile_ptr, "grad_cbsr/tile_ptr must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (grad_out && cbsr_idx && ent),
                 "grad/selector/plan pointers must not be NULL");
    MAXK_REQUIRE(!listed || (parts > 0 && bucket_ptr && n_list >= 0 &&
                             (n_list == 0 || (tile_list && bucket_tiles))),
                 "listed tiles need dim_k %% 4 == 0 and tile_list/bucket_ptr/bucket_tiles");
    const int64_t tiles = listed ? (int64_t)n_list : (int64_t)slices * nb;
    const size_t need = pull_workspace(num_rows, num_cols, dim_origin, dim_k, tiles, bucket_shift);
    MAXK_REQUIRE(workspace && workspace_bytes >= need,
                 "workspace too small: need %zu bytes, got %zu", need, workspace_bytes);
    // accumulate: bit 0 adds onto grad_cbsr; bit 1 (MAXK_PULL_NO_REDUCE) stops at the tile
    // partials, bit 2 (MAXK_PULL_REDUCE_ONLY) runs only the reduce over a workspace the same
    // call with bit 1 filled (listed tiles only: the hybrid runs the two-phase form between)
    const bool front = !(accumulate & MAXK_PULL_REDUCE_ONLY);
    const bool back = !(accumulate & MAXK_PULL_NO_REDUCE);
    MAXK_REQUIRE(listed || (front && back), "reduce-only / no-reduce need listed tiles");
    MAXK_REQUIRE(front || back, "no-reduce and reduce-only together run nothing");
    const int k = dim_k;
    const float *Gp = grad_out;
    const size_t gpb = ((size_t)num_rows * dim_origin * sizeof(float) + 255) & ~(size_t)255;
    if (front && row_div && num_rows > 0 && num_e > 0) {
        const int64_t n4 = num_rows * dim_origin / 4;
        hipLaunchKernelGGL(gprime_kernel, dim3((unsigned)ceil_div(n4, kBlock)), dim3(kBlock), 0,
                           s, grad_out, row_div, reinterpret_cast<float *>(workspace), n4,
                           dim_origin / 4);
        MAXK_LAUNCHED("gprime_kernel");
        Gp = reinterpret_cast<const float *>(workspace);
    }
    float *tile_out = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + gpb);
    const size_t acc_b = ((size_t)(k + 1) << bucket_shift) * sizeof(double);
    const size_t sel_b = ((size_t)k << bucket_shift);
    const bool sel_lds = acc_b + sel_b <= kPullLdsBytes;
    const size_t lds = acc_b + (sel_lds ? sel_b : 0);
    const uint2 *ent2 = reinterpret_cast<const uint2 *>(ent);
    // four l per lane (one u32 selector read) when k % 4 == 0, else one
    const uint8_t *lmap = nullptr;
    if (parts > 0) {  // quantile-slot form (pull_q_kernel), `parts` workgroups per tile
        const int kp = k / parts;
        const size_t lds_q = ((size_t)pull_ks(kp, bucket_shift) * 8 + kp) << bucket_shift;
        const size_t tb = (size_t)tiles * ((size_t)k << bucket_shift) * sizeof(float);
        const size_t nsel = ((size_t)num_cols * k + 255) & ~(size_t)255;
        uint8_t *sel_q = reinterpret_cast<uint8_t *>(tile_out) + tb;
        uint8_t *lm = sel_q + nsel;
        const int nd = kBlock / k;
        // values per lane: 4 (one u32 selector word per lane; 2 lanes per entry for 8-slot
        // parts), 8 for k = 8 (one lane per entry, one u64 selector word; MAXK_PULL_VPL8)
        const int vpl = kp != 8 ? 4 : MAXK_PULL_VPL8 ? MAXK_PULL_VPL8 : parts == 1 ? 8 : 4;
        lmap = lm;
        if (!front) goto reduce;
        if (MAXK_PULL_SEL4 && (reinterpret_cast<uintptr_t>(cbsr_idx) & 3) == 0) {
            const int nd4 = kBlock / (k / 4);
            hipLaunchKernelGGL(pull_sel4_kernel, dim3((unsigned)ceil_div(num_cols, nd4)),
                               dim3(kBlock), 0, s, cbsr_idx, sel_q, lm, num_cols, k, kp, vpl);
            MAXK_LAUNCHED("pull_sel4_kernel");
        } else {
            hipLaunchKernelGGL(pull_sel_kernel, dim3((unsigned)ceil_div(num_cols, nd)),
                               dim3(kBlock), 0, s, cbsr_idx, sel_q, lm, num_cols, k, kp, vpl);
            MAXK_LAUNCHED("pull_sel_kernel");
        }
        const int64_t work = tiles * parts;
        const bool fulld = dim_origin == kMaxDim;
        const unsigned grid = (unsigned)(MAXK_PULL_XCD ? xcd_grid(work) : work);
        if (work == 0) goto reduce;  // no listed tile: the reduce only permutes / accumulates
        switch (vpl == 2   ? (fulld ? -1 : -2)
                : vpl == 8 ? (fulld ? -3 : -4)
                           : lanes_per_edge(kp / 4) * 2 + (fulld ? 1 : 0)) {
#define MAXK_CASE_V(CASE, LRV, FD, VP)                                                        \
    case CASE:                                                                                \
        hipLaunchKernelGGL((pull_q_kernel<LRV, MAXK_PULL_QU, FD, VP>), dim3(grid), dim3(1024), \
                           lds_q, s, Gp, sel_q, tile_ptr, ent2, tile_out, num_cols, (int)nb,   \
                           (int)tiles, (int)rps, num_rows, dim_origin, k, kp, bucket_shift,    \
                           tile_list);                                                          \
        break;
#define MAXK_CASE(LRV) MAXK_CASE_V(LRV * 2 + 1, LRV, true, 4) MAXK_CASE_V(LRV * 2, LRV, false, 4)
            MAXK_CASE(1) MAXK_CASE(2) MAXK_CASE(4) MAXK_CASE(8) MAXK_CASE(16) MAXK_CASE(32)
            MAXK_CASE(64)
            MAXK_CASE_V(-1, 4, true, 2) MAXK_CASE_V(-2, 4, false, 2)
            MAXK_CASE_V(-3, 1, true, 8) MAXK_CASE_V(-4, 1, false, 8)
#undef MAXK_CASE
#undef MAXK_CASE_V
            default:
                set_error("unsupported lane group");
                return MAXK_ERR_INVALID;
        }
        MAXK_LAUNCHED("pull_q_kernel");
    } else switch (lanes_per_edge(v4 ? k / 4 : k) * 4 + (sel_lds ? 1 : 0) + (v4 ? 2 : 0)) {
#define MAXK_CASE(LRV, SL)                                                                    \
    case LRV * 4 + SL + 2:                                                                    \
        hipLaunchKernelGGL((pull_tile_kernel<LRV, MAXK_PULL_U, SL, 4>), dim3((unsigned)tiles), dim3(1024), \
                           lds, s, Gp, cbsr_idx, tile_ptr, ent2, tile_out, num_cols, (int)nb,  \
                           (int)rps, dim_origin, k, bucket_shift);                            \
        break;                                                                                \
    case LRV * 4 + SL:                                                                        \
        hipLaunchKernelGGL((pull_tile_kernel<LRV, MAXK_PULL_U, SL, 1>), dim3((unsigned)tiles), dim3(1024), \
                           lds, s, Gp, cbsr_idx, tile_ptr, ent2, tile_out, num_cols, (int)nb,  \
                           (int)rps, dim_origin, k, bucket_shift);                            \
        break;
        MAXK_CASE(1, 0) MAXK_CASE(1, 1)
        MAXK_CASE(2, 0) MAXK_CASE(2, 1)
        MAXK_CASE(4, 0) MAXK_CASE(4, 1)
        MAXK_CASE(8, 0) MAXK_CASE(8, 1)
        MAXK_CASE(16, 0) MAXK_CASE(16, 1)
        MAXK_CASE(32, 0) MAXK_CASE(32, 1)
        MAXK_CASE(64, 0) MAXK_CASE(64, 1)
#undef MAXK_CASE
        default:
            set_error("unsupported lane group");
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED("pull_tile_kernel");
reduce:
    if (!back) return MAXK_OK;
    hipLaunchKernelGGL(pull_reduce_kernel,
                       dim3((unsigned)nb, (unsigned)ceil_div(ceil_div((int64_t)k << bucket_shift, 4), kBlock)),
                       dim3(kBlock), 0, s, tile_out, lmap, grad_cbsr, num_cols, (int)nb, slices,
                       k, bucket_shift, listed ? bucket_ptr : nullptr,
                       listed ? bucket_tiles : nullptr, accumulate & 1);
    MAXK_LAUNCHED("pull_reduce_kernel");
    return MAXK_OK;
}
}  // namespace
}  // namespace maxk

extern "C" size_t maxk_sspmm_backward_pull_workspace_size(int64_t num_rows, int64_t num_cols,
                                                          int32_t dim_origin, int32_t dim_k,
                                                          int32_t slices) {
    if (num_rows < 0 || num_cols < 0 || dim_origin <= 0 || dim_k <= 0 || slices <= 0) return 0;
    const int shift = std::max(maxk_bucket_shift(dim_k), maxk_pull_shift(dim_k));
    return pull_workspace(num_rows, num_cols, dim_origin, dim_k,
                          (int64_t)slices * maxk_bucket_count(num_cols, shift), shift);
}

extern "C" int maxk_sspmm_backward_pull(const float *grad_out, const float *row_div,
                                        const uint8_t *cbsr_idx, const int32_t *tile_ptr,
                                        const uint32_t *ent, int32_t bucket_shift,
                                        int32_t slices, float *grad_cbsr, int64_t num_rows,
                                        int64_t num_cols, int64_t num_e, int32_t dim_origin,
                                        int32_t dim_k, void *workspace, size_t workspace_bytes,
                                        void *stream) {
    clear_error();
    return pull_impl(grad_out, row_div, cbsr_idx, tile_ptr, ent, bucket_shift, slices, false,
                     nullptr, 0, nullptr, nullptr, 0, grad_cbsr, num_rows, num_cols, num_e, dim_origin, dim_k,
                     workspace, workspace_bytes, stream);
}

extern "C" size_t maxk_sspmm_backward_pull_tiles_workspace_size(int64_t num_rows,
                                                                int64_t num_cols,
                                                                int32_t dim_origin,
                                                                int32_t dim_k, int32_t n_tiles) {
    if (num_rows < 0 || num_cols < 0 || dim_origin <= 0 || dim_k <= 0 || n_tiles < 0) return 0;
    return pull_workspace(num_rows, num_cols, dim_origin, dim_k, n_tiles,
                          std::max(maxk_bucket_shift(dim_k), maxk_pull_shift(dim_k)));
}

extern "C" int maxk_sspmm_backward_pull_tiles(
    const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
    const int32_t *tile_list, const int32_t *tile_ent, int32_t n_tiles,
    const int32_t *bucket_ptr, const int32_t *bucket_tiles, const uint32_t *ent,
    int32_t bucket_shift, int32_t slices, int32_t accumulate, float *grad_cbsr,
    int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k,
    void *workspace, size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(tile_ent, "tile_ent must not be NULL");
    return pull_impl(grad_out, row_div, cbsr_idx, tile_ent, ent, bucket_shift, slices, true,
                     tile_list, n_tiles, bucket_ptr, bucket_tiles, accumulate, grad_cbsr, num_rows, num_cols,
                     num_e, dim_origin, dim_k, workspace, workspace_bytes, stream);
}
