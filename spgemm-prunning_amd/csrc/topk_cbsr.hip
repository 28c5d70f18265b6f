// CBSR encode (MaxK top-k) and CBSR -> dense scatter for gfx950.
//
// Semantics: torch.topk(x, k, dim=1, largest=True, sorted=True) + .to(uint8)
// (maxk_spgemm_function.py:51-57); replaces the uint8 threshold-bisection
// kernel topk (kernels/maxk_kernel.cu:23-96), which is approximate (quantised
// input, index-order output, unfilled slots on ties) -- this one is exact.
//
// Two kernels.  topk_rows4_kernel (k <= MAXK_TOPK_ROWS4_KMAX, 48) puts four rows on one wave,
// 16 lanes per row, and finds the threshold by bisection over DPP row sums (see its comment).
// topk_cbsr_kernel (k > 32): one wavefront per row (D <= 256, so <= 4 elements per lane,
// column j = lane + 64*i for coalesced loads):
//  1. order-preserving 32-bit keys (NaN above +inf, as torch ranks it);
//  2. the k-th largest key T by MSB-first radix select over data-adaptive
//     8-bit digits (wave min/max of the keys in play, then a per-wave 256-bin
//     LDS histogram of the 8 bits below their common prefix + a wave suffix scan;
//     usually one pass).
//     (An earlier bit-by-bit construction, 32 dependent ballot/popcount rounds,
//     was bound by the CU's single scalar unit.)
//  3. select key > T, plus the lowest-column key == T until k are taken;
//  4. compact the k winners into LDS, rank each against the others
//     (broadcast LDS reads) and store in (key desc, column asc) order.
#include "common.h"

namespace maxk {
namespace {

// Rows whose search took other than k winners since the last reset (a kernel bug; read and
// reset by maxk_topk_error_rows).  One counter per device.
__device__ uint32_t g_topk_bad_rows = 0;

__device__ __forceinline__ uint32_t order_key(float x) {
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return 0xffffffffu;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t order_key(uint8_t x) { return x; }


template <typename T>
__global__ __launch_bounds__(kBlock) void topk_cbsr_kernel(const T *__restrict__ x, int64_t ld_x,
                                                           T *__restrict__ out_val,
                                                           uint8_t *__restrict__ out_idx,
                                                           int32_t *__restrict__ out_idx32,
                                                           T *__restrict__ out_dense,
                                                           int num_rows, int D, int k) {
    // winner slots [0, k), padding slots [k, k4) (key 0, column 255: never ranked above a
    // winner), and per-lane scratch slots [kMaxDim, kMaxDim + 64) for lanes not taking
    constexpr int kSlots = kMaxDim + kWave;
    __shared__ __attribute__((aligned(16))) uint32_t s_key[kWavesPerBlock][kSlots];
    __shared__ T s_val[kWavesPerBlock][kSlots];
    __shared__ __attribute__((aligned(16))) uint8_t s_col[kWavesPerBlock][kSlots];
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[kWavesPerBlock][256];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const int stride = gridDim.x * kWavesPerBlock;
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ok[i] = lane + kWave * i < D;
    // grid-stride over rows (a launch of one tiny workgroup per 4 rows is bound by the
    // workgroup dispatch rate); the next row's values are loaded before this row is ranked
    // loads are unconditional (clamped row / column), masked after: no predicated loads
    int col4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) col4[i] = ok[i] ? lane + kWave * i : D - 1;
    int row = blockIdx.x * kWavesPerBlock + wid;
    T vn[4];
    {
        const T *xr = x + (int64_t)(row < num_rows ? row : num_rows - 1) * ld_x;
#pragma unroll
        for (int i = 0; i < 4; ++i) vn[i] = xr[col4[i]];
    }
    for (; row < num_rows; row += stride) {
    T v[4];
    uint32_t key[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[i] = ok[i] ? vn[i] : T(0);
        key[i] = ok[i] ? order_key(v[i]) : 0u;
    }
    const int nrow = row + stride;
    {
        const T *xr = x + (int64_t)(nrow < num_rows ? nrow : row) * ld_x;
#pragma unroll
        for (int i = 0; i < 4; ++i) vn[i] = xr[col4[i]];
    }

    // T = max t such that #{key >= t} >= k  (the k-th largest key), by MSB-first radix
    // select with data-adaptive 8-bit digits: each pass takes the wave min / max of the
    // keys still in play and histograms the 8 bits right below their common prefix
    // (256-bin LDS histogram, integer atomics), then keeps the largest digit whose suffix
    // count still reaches `need`.  Real activations share their top bits (sign, exponent),
    // so a fixed top-byte digit would pile them into one bin; the adaptive digit spreads
    // them, and the pass usually ends the search (the chosen bin holds exactly the keys
    // still needed).
    uint32_t thr = 0, pmask = 0;
    int need = k;  // how many of the keys in play are still to be taken
    int sh = 0;    // selection compares key >> sh with thr (after the final shift)
    uint32_t *hist = s_hist[wid];
    for (;;) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in = ok[i] && (key[i] & pmask) == thr;
            mx = in && key[i] > mx ? key[i] : mx;
            mn = in && key[i] < mn ? key[i] : mn;
        }
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) {
            const uint32_t a = __shfl_xor(mx, off), b = __shfl_xor(mn, off);
            mx = a > mx ? a : mx;
            mn = b < mn ? b : mn;
        }
        const uint32_t diff = mx ^ mn;
        if (diff == 0u) {  // every key in play is equal: it is T, ties decide
            thr = mx;
            sh = 0;
            break;
        }
        const int hb = 31 - __builtin_clz(diff);  // highest bit where keys in play differ
        const int shift = hb >= 7 ? hb - 7 : 0;   // digit = bits [shift, shift + 8)
        reinterpret_cast<uint4 *>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_fence();
#pragma unroll
        for (int i = 0; i < 4; ++i)  // branch-free: keys out of play add 0
            atomicAdd(&hist[(key[i] >> shift) & 255u], (ok[i] && (key[i] & pmask) == thr) ? 1u : 0u);
        wave_lds_fence();
        const uint4 h = reinterpret_cast<const uint4 *>(hist)[lane];  // bins 4*lane .. 4*lane+3
        const uint32_t s3 = h.w, s2 = h.z + s3, s1 = h.y + s2, s0 = h.x + s1;
        uint32_t acc = s0;  // -> sum of s0 over lanes >= this one
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint32_t t = __shfl_down(acc, off);
            acc += lane + off < kWave ? t : 0u;
        }
        const uint32_t above = acc - s0;  // keys with a digit in a higher lane's bins
        const uint32_t nd = (uint32_t)need;
        // largest digit d with #{digit >= d} >= need: the highest lane holding one
        // (s0 >= s1 >= s2 >= s3: the conditions are monotone, m = their count - 1)
        const int m = (int)(above + s0 >= nd) + (int)(above + s1 >= nd) +
                      (int)(above + s2 >= nd) + (int)(above + s3 >= nd) - 1;
        const uint32_t gt_l = above + (uint32_t)(m == 0) * s1 + (uint32_t)(m == 1) * s2 +
                              (uint32_t)(m == 2) * s3;  // #{digit > 4*lane + m}
        const uint32_t ge_l = above + (uint32_t)(m == 0) * s0 + (uint32_t)(m == 1) * s1 +
                              (uint32_t)(m == 2) * s2 + (uint32_t)(m == 3) * s3;
        const uint64_t has = __ballot(m >= 0);
        const int src = 63 - __clzll(has);
        const int dm = __shfl(m, src);
        const uint32_t gt = __shfl(gt_l, src);
        const uint32_t in_bin = __shfl(ge_l, src) - gt;
        need -= (int)gt;
        // keys in play share every bit above shift + 8 (they differ first at bit hb)
        const uint32_t high = shift + 8 >= 32 ? 0u : (mx & (~0u << (shift + 8)));
        thr = high | ((uint32_t)(4 * src + dm) << shift);
        pmask = ~0u << shift;
        sh = shift;
        if (in_bin == (uint32_t)need || shift == 0) break;  // bin fully taken, or T exact
    }
    const int need_eq = need;
    thr >>= sh;

    // select, then compact winners into LDS slots [0, k)
    const int k4 = (k + 3) & ~3;
    for (int p = k + lane; p < k4; p += kWave) {
        s_key[wid][p] = 0u;
        s_col[wid][p] = 255;
    }
    int eq_base = 0, slot_base = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool eq = ok[i] && (key[i] >> sh) == thr;
        const uint64_t me = __ballot(eq);
        const int eq_rank = eq_base + __popcll(me & lt_mask);
        eq_base += __popcll(me);
        const bool take = (ok[i] && (key[i] >> sh) > thr) || (eq && eq_rank < need_eq);
        if (out_dense && ok[i])  // fused masked dense output (wave-uniform pointer test)
            out_dense[(int64_t)row * D + lane + kWave * i] = take ? v[i] : T(0);
        const uint64_t mt = __ballot(take);
        const int ws = slot_base + __popcll(mt & lt_mask);
        const int slot = take && ws < k ? ws : kMaxDim + lane;  // never past the k slots
        s_key[wid][slot] = key[i];
        s_val[wid][slot] = v[i];
        s_col[wid][slot] = (uint8_t)(lane + kWave * i);
        slot_base += __popcll(mt);
    }
    // any other count than k is a search bug: counted for the host (maxk_topk_error_rows)
    if (lane == 0 && slot_base != k) atomicAdd(&g_topk_bad_rows, 1u);
    wave_lds_fence();
    // rank of winner p among the winners: (key desc, column asc); 4 slots per LDS read
    for (int p = lane; p < k; p += kWave) {
        const uint32_t kp = s_key[wid][p];
        const int cp = s_col[wid][p];
        int pos = 0;
        for (int q = 0; q < k4; q += 4) {
            const uint4 kq = *reinterpret_cast<const uint4 *>(&s_key[wid][q]);
            const uint32_t cq = *reinterpret_cast<const uint32_t *>(&s_col[wid][q]);
            pos += (kq.x > kp) || (kq.x == kp && (int)(cq & 255u) < cp);
            pos += (kq.y > kp) || (kq.y == kp && (int)((cq >> 8) & 255u) < cp);
            pos += (kq.z > kp) || (kq.z == kp && (int)((cq >> 16) & 255u) < cp);
            pos += (kq.w > kp) || (kq.w == kp && (int)(cq >> 24) < cp);
        }
        const int64_t o = (int64_t)row * k + pos;
        out_val[o] = s_val[wid][p];
        out_idx[o] = (uint8_t)cp;
        if (out_idx32) out_idx32[o] = cp;
    }
    wave_lds_fence();  // this row's LDS slots are read before the next row overwrites them
    }
}

// ---- four rows per wave: 16 lanes per row ------------------------------------------------
// A row lives on 16 lanes (one DPP row, 16 values per lane: columns 64i + 4q + j), so every
// cross-lane step of a row is a DPP row operation folded into a VALU instruction and one
// wave instruction works on four rows.  Per row: the k-th largest key by a bitwise search
// (no LDS, no histogram atomics), tie-exact selection in column order, winners compacted to
// LDS and ranked (key desc, column asc) against each other.  Loads are unconditional and the
// next row group is prefetched while this one is ranked.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}
// all-reduce over the 16 lanes of a row (row_ror 8, 4, 2, 1)
__device__ __forceinline__ uint32_t row_max(uint32_t x) {
    x = max(x, dpp<0x128>(x));
    x = max(x, dpp<0x124>(x));
    x = max(x, dpp<0x122>(x));
    return max(x, dpp<0x121>(x));
}
__device__ __forceinline__ uint32_t row_min(uint32_t x) {
    x = min(x, dpp<0x128>(x));
    x = min(x, dpp<0x124>(x));
    x = min(x, dpp<0x122>(x));
    return min(x, dpp<0x121>(x));
}
__device__ __forceinline__ uint32_t row_sum(uint32_t x) {
    x += dpp<0x128>(x);
    x += dpp<0x124>(x);
    x += dpp<0x122>(x);
    return x + dpp<0x121>(x);
}
// exclusive prefix (lanes below in the row; row_shr: lane i reads lane i-n, 0 past the row)
__device__ __forceinline__ uint32_t row_prefix_excl(uint32_t x) {
    uint32_t a = x;
    a += dpp<0x111>(a);
    a += dpp<0x112>(a);
    a += dpp<0x114>(a);
    a += dpp<0x118>(a);
    return a - x;
}
// Unconditional loads at clamped columns (masked by ok[] afterwards): a predicated load makes
// the compiler wait for it at the branch merge, which would expose every prefetch.
template <typename T, bool VEC>
__device__ __forceinline__ void load_row16(const T *__restrict__ xr, int D, int q, T (&v)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c0 = 64 * i + 4 * q;
        if constexpr (VEC && sizeof(T) == 4) {
            const float4 f = *reinterpret_cast<const float4 *>(xr + (c0 < D ? c0 : D - 4));
            v[4 * i + 0] = f.x;
            v[4 * i + 1] = f.y;
            v[4 * i + 2] = f.z;
            v[4 * i + 3] = f.w;
        } else if constexpr (VEC) {
            const uint32_t w = *reinterpret_cast<const uint32_t *>(xr + (c0 < D ? c0 : D - 4));
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = (T)((w >> (8 * j)) & 255u);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = xr[c0 + j < D ? c0 + j : D - 1];
        }
    }
}

#if MAXK_TOPK_FENCE_WAIT  // tools only: drain the wave's LDS queue at every fence
#define wave_lds_fence()                                  \
    do {                                                  \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
        maxk::wave_lds_fence();                           \
    } while (0)
#endif
template <typename T, bool VEC, int J>
__global__ __launch_bounds__(kBlock) void topk_rows4_kernel(const T *__restrict__ x, int64_t ld_x,
                                                            T *__restrict__ out_val,
                                                            uint8_t *__restrict__ out_idx,
                                                            int32_t *__restrict__ out_idx32,
                                                            T *__restrict__ out_dense,
                                                            int num_rows, int D, int k,
                                                            int wave_lds_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_topk[];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int sub = lane >> 4, q = lane & 15;
    const int k4 = (k + 3) & ~3;
    uint32_t *wl = lds_topk + (size_t)wid * wave_lds_words;
    uint32_t *wkey = wl + sub * (3 * k4);  // the row's winners: keys, values, columns
    uint32_t *wval = wkey + k4;
    uint32_t *wcol = wval + k4;
    const int stride = gridDim.x * kWavesPerBlock * 4;  // rows per grid step
    bool ok[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) ok[t] = 64 * (t >> 2) + 4 * q + (t & 3) < D;
    int row = (blockIdx.x * kWavesPerBlock + wid) * 4 + sub;
    T vn[16];
    load_row16<T, VEC>(x + (int64_t)(row < num_rows ? row : num_rows - 1) * ld_x, D, q, vn);
    uint32_t n_bad = 0;  // this lane's rows with other than k winners (lane q == 0 counts)
    for (int rbase = (blockIdx.x * kWavesPerBlock + wid) * 4; rbase < num_rows;
         rbase += stride, row += stride) {
        const bool live = row < num_rows;
        T v[16];
        uint32_t key[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            v[t] = vn[t];
            key[t] = ok[t] ? order_key(v[t]) : 0u;
        }
        {
            const int nrow = row + stride;
            load_row16<T, VEC>(x + (int64_t)(nrow < num_rows ? nrow : num_rows - 1) * ld_x, D, q,
                               vn);
        }
        // ---- threshold T = the k-th largest key, built bit by bit from the highest bit where
        // the row's keys differ: T | bit is kept while at least k keys are >= it (one compare
        // per key and a DPP row sum per bit, no LDS).  A candidate with exactly k keys >= it
        // ends the row's search: selecting key >= T then takes exactly k.
        // The search starts at the highest bit where mx and a lower bound lb of the answer
        // differ: lb = max(smallest key, smallest over the row's lanes of the lane's j-th
        // largest key, j = ceil(k / 16)), since 16 lanes x j keys are >= the latter.  The
        // answer lies in [lb, mx] and so shares their common prefix; on Gaussian rows this
        // skips the sign and most exponent bits.
        // m[0..J) = the lane's J largest keys (an insertion network, lowest slot first so
        // every slot reads the previous key's values); the lane's j-th largest with
        // j = ceil(k / 16) <= J bounds the answer from below: 16 lanes x j keys are >= the
        // smallest of them over the row, and 16 j >= k.
        uint32_t mx = 0u, mn = ~0u, m[J];
#pragma unroll
        for (int j = 0; j < J; ++j) m[j] = 0u;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            mx = key[t] > mx ? key[t] : mx;  // columns past D hold key 0
            mn = ok[t] && key[t] < mn ? key[t] : mn;
#pragma unroll
            for (int j = J - 1; j > 0; --j) m[j] = max(m[j], min(m[j - 1], key[t]));
            m[0] = max(m[0], key[t]);
        }
        mx = row_max(mx);
        mn = row_min(mn);
        uint32_t mj = m[0];
#pragma unroll
        for (int j = 1; j < J; ++j) mj = k > 16 * j ? m[j] : mj;
        uint32_t lb = MAXK_TOPK_LB ? row_min(mj) : 0u;
        lb = lb > mn ? lb : mn;
        uint32_t thr;
        int need = k;
        if (MAXK_TOPK_BISECT) {
            // Bisection over the key interval [lb, mx] itself: the answer is the largest c
            // with at least k keys >= c.  Invariant: >= k keys are >= lo, the answer <= hi.
            // The bit search below halves a power-of-two interval instead, which is 2^31
            // wide whenever [lb, mx] straddles a float exponent boundary with a carry (a
            // Gaussian row's does: 0x3F7F... -> 0x4000...); the count of keys >= mid == k
            // ends a row early in both.
            uint32_t lo = lb, hi = mx;
            bool done = lo == hi;  // rows past the end search too (see `take` below)
            for (;;) {
                const bool go = !done;
                if (__ballot(go) == 0) break;
                const uint32_t d = hi - lo;
                const uint32_t mid = lo + (d >> 1) + (d & 1u);  // in (lo, hi]: >= 1
                uint32_t n = 0;  // columns past D hold key 0 < mid: no mask needed
#pragma unroll
                for (int t = 0; t < 16; ++t) n += key[t] >= mid ? 1u : 0u;
                n = row_sum(n);
                if (go) {
                    if (n >= (uint32_t)k) lo = mid;
                    else hi = mid - 1u;
                    if (n == (uint32_t)k || lo == hi) done = true;
                }
            }
            thr = lo;
        } else {
            const uint32_t diff = mx ^ lb;
            int bit = diff ? 31 - __builtin_clz(diff) : -1;
            // common prefix of the keys (all keys are >= it); bit 31 differing -> no prefix
            thr = !diff ? mx : (bit == 31 ? 0u : mx & (~0u << (bit + 1)));
            bool done = diff == 0u;
            for (;;) {
                const bool go = !done && bit >= 0;
                if (__ballot(go) == 0) break;
                const uint32_t c = thr | (1u << (bit & 31));
                uint32_t n = 0;  // columns past D hold key 0 < c (c >= 1): no mask needed
#pragma unroll
                for (int t = 0; t < 16; ++t) n += key[t] >= c ? 1u : 0u;
                n = row_sum(n);
                if (go) {
                    if (n >= (uint32_t)k) thr = c;
                    if (n == (uint32_t)k) done = true;
                    --bit;
                }
            }
        }
        const int sh = 0;
        // keys > thr are taken; `need` of the keys == thr (ties: lowest columns first)
        {
            uint32_t ngt = 0;
#pragma unroll
            for (int t = 0; t < 16; ++t) ngt += (ok[t] && key[t] > thr) ? 1u : 0u;
            need = k - (int)row_sum(ngt);
        }
        const uint32_t T_ = thr >> sh;
        // ---- selection: key > T, plus the lowest-column keys == T until k are taken
        uint32_t neq = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) neq += (ok[t] && (key[t] >> sh) == T_) ? 1u : 0u;
        const uint32_t neq_row = row_sum(neq);  // every lane: DPP reads the whole row
        // Rows past the end (the last row group's dead sub-rows, holding a copy of the last
        // row) run the same exact search and take exactly k winners; they only skip the
        // stores.  Skipping their search (r02) left thr at their lower bound, so "key >= thr"
        // took 32-100 winners whose compaction ran past the row's 3*k4 LDS words into the next
        // wave's winners -- which that wave, one grid-stride round behind, could still be
        // ranking (r02's k = 48 mismatch on row 2186888 of the seed-0 [2449029, 256] Gaussian
        // input).  Searching costs nothing there; a `live` test per key cost 2-3 %.
        const bool ties = neq_row != (uint32_t)need;
        // The selection below takes (k - need) keys above the threshold plus min(need, neq_row)
        // equal ones: exactly k whenever 0 <= need <= neq_row, which the search guarantees.  A
        // row outside that is a bug in the search (r02's dead sub-rows were one): it is counted
        // for the host (maxk_topk_error_rows) and takes no winners at all, so its compaction
        // cannot write past its k LDS slots into another row's or another wave's winners, and
        // the good rows need no per-winner bound check.  Such a row always has ties
        // (neq_row != need: need < 0 wraps past any count), so the check sits in that branch.
        bool take[16];
        if (__ballot(ties) == 0) {
#pragma unroll
            for (int t = 0; t < 16; ++t) take[t] = ok[t] && (key[t] >> sh) >= T_;
        } else {  // rank the equal keys in column order: chunk i, then lane, then j
            uint32_t base = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t c = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) c += (ok[4 * i + j] && (key[4 * i + j] >> sh) == T_);
                uint32_t r = base + row_prefix_excl(c);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = 4 * i + j;
                    const bool eq = ok[t] && (key[t] >> sh) == T_;
                    take[t] = (ok[t] && (key[t] >> sh) > T_) || (eq && r < (uint32_t)need);
                    r += eq ? 1u : 0u;
                }
                base += row_sum(c);
            }
            const bool bad = (uint32_t)need > neq_row;
            if (__ballot(bad) != 0) {  // never taken unless the search is wrong
                n_bad += live && q == 0 && bad ? 1u : 0u;
#pragma unroll
                for (int t = 0; t < 16; ++t) take[t] = take[t] && !bad;
            }
        }
        if (out_dense && live) {  // fused masked dense output
            T *dr = out_dense + (int64_t)row * D;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c0 = 64 * i + 4 * q;
                if constexpr (sizeof(T) == 4 && VEC) {
                    if (c0 < D) {
                        *reinterpret_cast<float4 *>(dr + c0) =
                            make_float4(take[4 * i] ? v[4 * i] : 0.f,
                                        take[4 * i + 1] ? v[4 * i + 1] : 0.f,
                                        take[4 * i + 2] ? v[4 * i + 2] : 0.f,
                                        take[4 * i + 3] ? v[4 * i + 3] : 0.f);
                        continue;
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (c0 + j < D) dr[c0 + j] = take[4 * i + j] ? v[4 * i + j] : T(0);
            }
        }
        // ---- compact the row's winners into LDS, rank them, store
        uint32_t nw = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) nw += take[t] ? 1u : 0u;
        uint32_t slot = row_prefix_excl(nw);  // a row's winners fill slots [0, k) (`bad` above)
        wave_lds_fence();  // the previous group's winners are no longer read
        for (int p = k + q; p < k4; p += 16) {
            wkey[p] = 0u;
            wcol[p] = 255u;
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            if (take[t]) {
                wkey[slot] = key[t];
                wval[slot] = sizeof(T) == 4 ? __builtin_bit_cast(uint32_t, (float)v[t])
                                            : (uint32_t)v[t];
                wcol[slot] = (uint32_t)(64 * (t >> 2) + 4 * q + (t & 3));
                ++slot;
            }
        }
        wave_lds_fence();
        if (live) {
            for (int p = q; p < k; p += 16) {
                const uint32_t kp = wkey[p], cp = wcol[p];
                int pos = 0;
                for (int o = 0; o < k4; o += 4) {
                    const uint4 kq = *reinterpret_cast<const uint4 *>(&wkey[o]);
                    const uint4 cq = *reinterpret_cast<const uint4 *>(&wcol[o]);
                    pos += (kq.x > kp) || (kq.x == kp && cq.x < cp);
                    pos += (kq.y > kp) || (kq.y == kp && cq.y < cp);
                    pos += (kq.z > kp) || (kq.z == kp && cq.z < cp);
                    pos += (kq.w > kp) || (kq.w == kp && cq.w < cp);
                }
                const int64_t o = (int64_t)row * k + pos;
                const uint32_t vb = wval[p];
                if constexpr (sizeof(T) == 4)
                    out_val[o] = __builtin_bit_cast(float, vb);
                else
                    out_val[o] = (T)vb;
                out_idx[o] = (uint8_t)cp;
                if (out_idx32) out_idx32[o] = (int32_t)cp;
            }
        }
        wave_lds_fence();  // winners read before the next group's histogram overwrites them
    }
    if (n_bad) atomicAdd(&g_topk_bad_rows, n_bad);  // maxk_topk_error_rows
}

#ifdef wave_lds_fence
#undef wave_lds_fence
#endif
// dense[r, :] = 0; dense[r, idx[r, l]] = val[r, l] + add[r, idx[r, l]]   (val and add
// optional).  One wave per row, grid-stride: one workgroup per 4 rows would be bound by
// workgroup dispatch on large graphs.  A row's reads all land in LDS before its stores, so
// dense may alias add (in-place MaxK gradient).
#if MAXK_SCATTER_ROWS4
// Four rows per wave, 16 lanes per row for the k (index, value) pairs; the four 1 KB rows are
// then stored one per wave instruction (16 B per lane).  One row per wave left each wave a
// chain of dependent byte loads, an LDS round trip and a store per row.
__global__ __launch_bounds__(kBlock) void cbsr_scatter_dense_kernel(
    const float *__restrict__ val, const uint8_t *__restrict__ idx, const float *add,
    float *dense, int num_rows, int D, int k) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][4][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int sub = lane >> 4, sl = lane & 15;
    float(*buf)[kMaxDim] = lds[wid];
    const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 4;
    for (int64_t g0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * 4; g0 < num_rows;
         g0 += stride) {
        const int64_t row = g0 + sub;
        float4 *b4 = reinterpret_cast<float4 *>(&buf[sub][sl * 16]);
#pragma unroll
        for (int i = 0; i < 4; ++i) b4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        wave_lds_fence();
        if (row < num_rows) {
            for (int l = sl; l < k; l += 16) {
                const int j = idx[row * k + l];
                float x = val ? val[row * k + l] : 0.f;
                if (add) x += add[row * D + j];
                buf[sub][j] = x;
            }
        }
        wave_lds_fence();
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int64_t r = g0 + rr;
            if (r >= num_rows) break;
            float *dst = dense + r * D;
            if ((D & 3) == 0) {
                for (int j = lane * 4; j < D; j += kWave * 4)
                    *reinterpret_cast<float4 *>(&dst[j]) =
                        *reinterpret_cast<const float4 *>(&buf[rr][j]);
            } else {
                for (int j = lane; j < D; j += kWave) dst[j] = buf[rr][j];
            }
        }
        wave_lds_fence();
    }
}
#else
__global__ __launch_bounds__(kBlock) void cbsr_scatter_dense_kernel(
    const float *__restrict__ val, const uint8_t *__restrict__ idx, const float *add,
    float *dense, int num_rows, int D, int k) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    float *buf = lds[wid];
    for (int row = blockIdx.x * kWavesPerBlock + wid; row < num_rows;
         row += gridDim.x * kWavesPerBlock) {
        *reinterpret_cast<float4 *>(&buf[lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
        wave_lds_fence();
        for (int l = lane; l < k; l += kWave) {
            const int j = idx[(int64_t)row * k + l];
            float x = val ? val[(int64_t)row * k + l] : 0.f;
            if (add) x += add[(int64_t)row * D + j];
            buf[j] = x;
        }
        wave_lds_fence();
        float *dst = dense + (int64_t)row * D;
        if ((D & 3) == 0) {
            for (int j = lane * 4; j < D; j += kWave * 4)
                *reinterpret_cast<float4 *>(&dst[j]) = *reinterpret_cast<const float4 *>(&buf[j]);
        } else {
            for (int j = lane; j < D; j += kWave) dst[j] = buf[j];
        }
        wave_lds_fence();
    }
}
#endif

template <typename T>
int topk_launch(const T *x, int64_t ld_x, T *val, uint8_t *idx, int32_t *idx32, T *dense,
                int64_t num_rows, int32_t D, int32_t k, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(D >= 1 && D <= kMaxDim, "dim_origin must be in [1,256], got %d", D);
    MAXK_REQUIRE(k >= 1 && k <= D, "dim_k must be in [1,dim_origin], got %d", k);
    MAXK_REQUIRE(ld_x >= D, "ld_x (%lld) < dim_origin (%d)", (long long)ld_x, D);
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(x && val && idx, "x/val/idx must not be NULL");
    if (MAXK_TOPK_ROWS4 && k <= MAXK_TOPK_ROWS4_KMAX) {  // at k=64 its k^2 ranking ties one
                                                         // row per wave
        const int k4 = (k + 3) & ~3;
        const int words = 4 * 3 * k4;  // per wave: 4 rows of winners (key, value, column)
        const size_t lds = (size_t)kWavesPerBlock * words * 4;
        const bool vec = D % 4 == 0 && ld_x % 4 == 0 &&
                         (reinterpret_cast<uintptr_t>(x) % (4 * sizeof(T))) == 0;
        const int64_t blocks = ceil_div(num_rows, 4 * kWavesPerBlock);
        const dim3 grid((unsigned)(blocks < MAXK_TOPK_BLOCKS ? blocks : MAXK_TOPK_BLOCKS));
        // J = lane keys kept for the lower bound: 2 up to k = 32, 4 up to 64
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, grid, dim3(kBlock), lds, as_stream(stream), x, ld_x, val, idx,
                               idx32, dense, (int)num_rows, D, k, words);
        };
        if (k <= 32)
            vec ? go(topk_rows4_kernel<T, true, 2>) : go(topk_rows4_kernel<T, false, 2>);
        else
            vec ? go(topk_rows4_kernel<T, true, 4>) : go(topk_rows4_kernel<T, false, 4>);
        MAXK_LAUNCHED("topk_rows4_kernel");
        return MAXK_OK;
    }
    const int64_t blocks = ceil_div(num_rows, kWavesPerBlock);
    const dim3 grid((unsigned)(blocks < MAXK_TOPK_BLOCKS ? blocks : MAXK_TOPK_BLOCKS));
    hipLaunchKernelGGL(topk_cbsr_kernel<T>, grid, dim3(kBlock), 0, as_stream(stream), x, ld_x, val,
                       idx, idx32, dense, (int)num_rows, D, k);
    MAXK_LAUNCHED("topk_cbsr_kernel");
    return MAXK_OK;
}

// The reference uint8 top-k's intended per-row convention (kernels/maxk_kernel.cu:23-94, behind
// cuda_topk_maxk / cuda_topk_maxk_float), one wave per row of 256 bytes (four per lane).  Not
// the CUDA kernel's as-built output, which thresholds every row on its block's first row per
// lane (:42, :44-48) through a shared-memory race (oracle topk_u8_reference_as_built; unpinned):
//  * threshold: 8 bisection steps on [0, 255] over the row's own bytes > mid (ballots); fewer than k:
//    high = mid, else low = mid; mid = (low + high) / 2;
//  * selection: the bytes strictly above mid in ascending column order, 32 columns per step
//    (column 32 s + l on lane l), at most k; the step's count is the exclusive prefix of its
//    lane 31, so a pick in column 32 s + 31 is overwritten by the next step's first pick, as in
//    the reference; slots never filled stay 0.
// The row's output is assembled in LDS (the overwrite order kept) and stored once.
__global__ __launch_bounds__(kBlock) void topk_u8_reference_kernel(const uint8_t *__restrict__ x,
                                                                   uint8_t *__restrict__ val,
                                                                   uint8_t *__restrict__ idx,
                                                                   int num_rows, int k) {
    __shared__ uint8_t s_out[kWavesPerBlock][2 * 256];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    uint8_t *sv = s_out[wid], *si = s_out[wid] + 256;
    for (int row = blockIdx.x * kWavesPerBlock + wid; row < num_rows;
         row += gridDim.x * kWavesPerBlock) {
        const uint32_t w = reinterpret_cast<const uint32_t *>(x + (int64_t)row * 256)[lane];
        int low = 0, high = 255, mid = 127;
        for (int it = 0; it < 8; ++it) {
            int count = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                count += __popcll(__ballot((int)((w >> (8 * b)) & 255u) > mid));
            if (count < k)
                high = mid;
            else
                low = mid;
            mid = (low + high) / 2;
        }
        for (int i = lane; i < 2 * k; i += kWave) s_out[wid][i < k ? i : 256 + i - k] = 0;
        wave_lds_fence();
        int total = 0;
        for (int ext = 0; ext < 8 && total < k; ++ext) {
            const int c = ext * 32 + (lane & 31);  // lanes 32..63 mirror 0..31 and do not pick
            const uint32_t src = (uint32_t)__shfl((int)w, c >> 2);
            const int v = (int)((src >> (8 * (c & 3))) & 255u);
            const bool choose = lane < 32 && v > mid;
            const uint64_t mask = __ballot(choose);
            const int loc = __popcll(mask & ((1ull << lane) - 1));
            if (choose && total + loc < k) {
                sv[total + loc] = (uint8_t)v;
                si[total + loc] = (uint8_t)c;
            }
            wave_lds_fence();
            total += __popcll(mask & 0x7fffffffull);  // lane 31's exclusive prefix
        }
        for (int i = lane; i < k; i += kWave) {
            val[(int64_t)row * k + i] = sv[i];
            idx[(int64_t)row * k + i] = si[i];
        }
        wave_lds_fence();
    }
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" int maxk_topk_cbsr(const float *x, int64_t ld_x, float *cbsr_val, uint8_t *cbsr_idx,
                              int32_t *idx32, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                              void *stream) {
    return topk_launch<float>(x, ld_x, cbsr_val, cbsr_idx, idx32, nullptr, num_rows, dim_origin,
                              dim_k, stream);
}

extern "C" int maxk_topk_cbsr_dense(const float *x, int64_t ld_x, float *cbsr_val,
                                    uint8_t *cbsr_idx, float *dense, int64_t num_rows,
                                    int32_t dim_origin, int32_t dim_k, void *stream) {
    if (num_rows > 0 && !dense) {
        clear_error();
        MAXK_REQUIRE(dense, "dense must not be NULL");
    }
    return topk_launch<float>(x, ld_x, cbsr_val, cbsr_idx, nullptr, dense, num_rows, dim_origin,
                              dim_k, stream);
}

extern "C" int maxk_topk_cbsr_u8(const uint8_t *x, int64_t ld_x, uint8_t *cbsr_val,
                                 uint8_t *cbsr_idx, int32_t *idx32, int64_t num_rows,
                                 int32_t dim_origin, int32_t dim_k, void *stream) {
    return topk_launch<uint8_t>(x, ld_x, cbsr_val, cbsr_idx, idx32, nullptr, num_rows, dim_origin,
                                dim_k, stream);
}

extern "C" int maxk_topk_error_rows(int64_t *rows, int32_t reset, void *stream) {
    clear_error();
    MAXK_REQUIRE(rows, "rows must not be NULL");
    hipStream_t s = as_stream(stream);
    uint32_t v = 0;
    MAXK_HIP(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_topk_bad_rows), sizeof(v), 0,
                                      hipMemcpyDeviceToHost, s));
    MAXK_HIP(hipStreamSynchronize(s));
    if (reset && v) {
        static const uint32_t z = 0;
        MAXK_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_topk_bad_rows), &z, sizeof(z), 0,
                                        hipMemcpyHostToDevice, s));
        MAXK_HIP(hipStreamSynchronize(s));
    }
    *rows = v;
    return MAXK_OK;
}

namespace maxk {
namespace {
int scatter_launch(const float *val, const uint8_t *idx, const float *add, float *dense,
                   int64_t num_rows, int32_t dim_origin, int32_t dim_k, void *stream) {
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(dim_origin >= 1 && dim_origin <= kMaxDim, "dim_origin must be in [1,256]");
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= dim_origin, "dim_k must be in [1,dim_origin]");
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(idx && dense, "pointers must not be NULL");
    const int64_t blocks = ceil_div(num_rows, kWavesPerBlock * (MAXK_SCATTER_ROWS4 ? 4 : 1));
    const dim3 grid((unsigned)(blocks < MAXK_TOPK_BLOCKS ? blocks : MAXK_TOPK_BLOCKS));
    hipLaunchKernelGGL(cbsr_scatter_dense_kernel, grid, dim3(kBlock), 0, as_stream(stream), val,
                       idx, add, dense, (int)num_rows, dim_origin, dim_k);
    MAXK_LAUNCHED("cbsr_scatter_dense_kernel");
    return MAXK_OK;
}
}  // namespace
}  // namespace maxk

extern "C" int maxk_topk_backward(const float *grad_val, const float *grad_dense,
                                  const uint8_t *cbsr_idx, float *grad_x, int64_t num_rows,
                                  int32_t dim_origin, int32_t dim_k, void *stream) {
    clear_error();
    return scatter_launch(grad_val, cbsr_idx, grad_dense, grad_x, num_rows, dim_origin, dim_k,
                          stream);
}

extern "C" int maxk_cbsr_scatter_dense(const float *cbsr_val, const uint8_t *cbsr_idx,
                                       float *dense, int64_t num_rows, int32_t dim_origin,
                                       int32_t dim_k, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows == 0 || cbsr_val, "cbsr_val must not be NULL");
    return scatter_launch(cbsr_val, cbsr_idx, nullptr, dense, num_rows, dim_origin, dim_k, stream);
}

extern "C" int maxk_topk_u8_reference(const uint8_t *x, uint8_t *val, uint8_t *idx,
                                      int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                                      void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(dim_origin == 256, "the reference's uint8 top-k has rows of 256, got %d",
                 dim_origin);
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= 256, "dim_k must be in [1,256], got %d", dim_k);
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(x && val && idx, "pointers must not be NULL");
    MAXK_REQUIRE(((uintptr_t)x & 3) == 0, "x must be 4-B aligned");
    const int64_t blocks = ceil_div(num_rows, kWavesPerBlock);
    hipLaunchKernelGGL(topk_u8_reference_kernel,
                       dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(kBlock), 0,
                       as_stream(stream), x, val, idx, (int)num_rows, dim_k);
    MAXK_LAUNCHED("topk_u8_reference_kernel");
    return MAXK_OK;
}
