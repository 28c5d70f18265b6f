// Dense route for wide top-k (r05): k >= D / 2 at D <= MAXK_DENSE_DMAX.
//
// A vertex's CBSR row (k values + k selectors; 6k bytes as a packed record, plus one LDS
// read-modify-write per selected column and edge in the record walkers) then carries as many
// bytes as its dense row (4D) and more instructions, so the aggregation reads dense rows:
//
//   forward   X = scatter(CBSR) (cbsr_dense_kernel, the record pack's duplicate rule), then
//             out = diag(1/row_div) A X by dense_rows_kernel;
//   backward  Y = A^T diag(1/row_div) G by the same kernel over the graph's transpose with its
//             source rows (maxk_dense_plan), each finished row stored as its k selected
//             columns, grad_cbsr[c, l] = Y[c, sel[c, l]] (selectors >= D read 0, as in every
//             mode); rows split over items are finished by dense_fixup_select_kernel.
//
// dense_rows_kernel reads the CSR as the token stream of common.h (one wave per item of
// `chunk` tokens).  The item's column ids and weights (divided by src_div when given) are staged
// in LDS with coalesced loads.  Lane groups of LR = pow2ceil(D / 4) lanes (a float4 each) take
// whole rows of at most kDenseGroupMax of the item's edges: a group walks its row U edges per
// step into registers, stores it the step it ends and takes the item's next row, so 64 / LR rows
// are in flight per wave and the next step's gathers are issued before this step's sums.  A
// longer row, and the continuation of a row started in an earlier item (its partial goes to the
// item's slab; slab_fixup_kernel adds the slabs in item order), are walked by the whole wave,
// edges interleaved over the groups and the groups combined by xor butterflies.  Sums run in
// edge order per lane: bitwise the same run to run.
#include <atomic>

#include "common.h"

namespace maxk {
namespace {

constexpr int kDenseBlock = 512;     // threads of the scatter kernel
constexpr int kDenseLdsWords = 4096;  // its LDS rows: (4 * kDenseBlock / k) * D <= 4096 floats
constexpr int kDenseGroupMax = 64;   // rows of at most this many item edges go to lane groups
constexpr int kDenseChunkMax = 512;  // item size cap (LDS staging: 8 B per token per wave)

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// X[v, :] = the dense row of vertex v's CBSR: four l per thread (one u32 selector word, one
// float4 of values), 4 * kDenseBlock / k whole vertices per group, rows assembled in LDS and
// stored as one contiguous run.  Duplicate selectors of a vertex: the lowest l carries the sum
// of their values in l order (cbsr_pack4_kernel's rule); selectors >= D are dropped.
__global__ __launch_bounds__(kDenseBlock) void cbsr_dense_kernel(const float *__restrict__ cbsr_val,
                                                             const uint8_t *__restrict__ cbsr_idx,
                                                             float *__restrict__ X, int num_cols,
                                                             int k, int D) {
    __shared__ __attribute__((aligned(16))) float s_x[kDenseLdsWords];
    __shared__ uint32_t s_bits[kDenseBlock * 8];
    __shared__ int s_dup[kDenseBlock];
    const int tpv = k >> 2;
    const int vpw = kDenseBlock / tpv;
    const int t = threadIdx.x;
    const int vl = t / tpv, l0 = (t - vl * tpv) * 4;
    for (int64_t g0 = (int64_t)blockIdx.x * vpw; g0 < num_cols; g0 += (int64_t)gridDim.x * vpw) {
        const int nv = num_cols - g0 < vpw ? (int)(num_cols - g0) : vpw;
        const int64_t v = g0 + vl;
        const bool act = vl < nv;
        for (int i = t; i < vpw * D; i += kDenseBlock) s_x[i] = 0.f;
        for (int i = t; i < vpw * 8; i += kDenseBlock) s_bits[i] = 0u;
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
            const float xv[4] = {x.x, x.y, x.z, x.w};
            const bool any_dup = s_dup[vl] != 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sj = (w >> (8 * j)) & 255u;
                float o = xv[j];
                bool first = true;
                if (any_dup) {  // rare
                    const int l = l0 + j;
                    const uint8_t *ci = cbsr_idx + v * k;
                    const float *cv = cbsr_val + v * k;
                    for (int m = 0; m < l; ++m) first = first && ci[m] != sj;
                    if (first)
                        for (int m = l + 1; m < k; ++m)
                            if (ci[m] == sj) o += cv[m];
                }
                if (first && (int)sj < D) s_x[vl * D + sj] = o;
            }
        }
        __syncthreads();
        float4 *dst = reinterpret_cast<float4 *>(X + g0 * D);
        const float4 *src = reinterpret_cast<const float4 *>(s_x);
        for (int i = t; i < nv * D / 4; i += kDenseBlock) dst[i] = src[i];
        __syncthreads();  // LDS is reused by the next group
    }
}

__device__ __forceinline__ void fma4(float4 &a, float s, const float4 &v) {
    a.x = __builtin_fmaf(s, v.x, a.x);
    a.y = __builtin_fmaf(s, v.y, a.y);
    a.z = __builtin_fmaf(s, v.z, a.z);
    a.w = __builtin_fmaf(s, v.w, a.w);
}

// dst[4q .. 4q + 4) of one row: the sum divided by div (when has_div), added onto dst (add)
__device__ __forceinline__ void store_row4(float *dst, float4 a, bool has_div, float div,
                                           bool add) {
    if (has_div) {
        a.x /= div;
        a.y /= div;
        a.z /= div;
        a.w /= div;
    }
    float4 *p = reinterpret_cast<float4 *>(dst);
    if (add) {
        const float4 o = *p;
        a.x += o.x;
        a.y += o.y;
        a.z += o.z;
        a.w += o.w;
    }
    *p = a;
}

// Rows are owned by the item holding their token.  A row of at most `chunk` edges is walked
// whole by its owner, past the item's end if it must (so an item walks at most 2 * chunk
// tokens; the LDS stage holds that many edges); only a longer (hub) row is split at item ends:
// its owner stores a partial, every later item it reaches stores a partial to its slab, and
// slab_fixup_kernel (forward) / dense_fixup_select_kernel (backward) add the slabs in item
// order.  (Finishing hub rows inside the walk -- the last item to reach one adding the slabs,
// counted with a device-scope atomic -- measured 2.7x slower on Flickr: every device-scope
// release / acquire writes back and invalidates the XCD's L2.)  SEL (the backward): a whole
// row is stored as its k selected
// columns, grad_cbsr[row, l] = row[sel[row, l]] (through a per-group LDS copy of the row); a hub
// row's partials go to out (= Y) and the slabs for dense_fixup_select_kernel.
template <int LR, int U, bool SEL>
__device__ __forceinline__ void dense_rows_body(
    const int32_t *__restrict__ ptr, const int32_t *__restrict__ idx, const float *__restrict__ w,
    const float *__restrict__ src_div, const float *__restrict__ X, int D,
    const float *__restrict__ dst_div, float *__restrict__ out, int add,
    float *__restrict__ slab, int32_t *__restrict__ slab_row, int num_rows, int64_t num_e,
    int chunk, int n_items, const uint8_t *__restrict__ sel, float *__restrict__ grad_cbsr,
    int k) {
    constexpr int NG = kWave / LR;  // lane groups (rows in flight) per wave
    // per wave: ids and scales of 2 * chunk edges, then (SEL) one row copy per lane group
    extern __shared__ __attribute__((aligned(16))) int32_t s_stage[];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int item = (int)blockIdx.x * kWavesPerBlock + wid;
    if (item >= n_items) return;  // whole wave; no workgroup barrier below
    const int g = lane / LR, q = lane % LR;
    const int D4 = D >> 2;
    const bool qok = q < D4;
    const float4 *__restrict__ X4 = reinterpret_cast<const float4 *>(X);
    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int r = wave_first_row_token(ptr, num_rows, d0);
    const int64_t p_lo = d0 - r;  // the item's first edge (the tokens before d0 hold r rows)
    int32_t *s_idx = s_stage + (size_t)wid * (4 * chunk + (SEL ? 4 * kWave : 0));
    float *s_sc = reinterpret_cast<float *>(s_idx + 2 * chunk);
    float *s_buf = s_sc + 2 * chunk;  // SEL: group g's row copy at g * 4 * LR
    const uint32_t *__restrict__ sel32 = reinterpret_cast<const uint32_t *>(sel);
    const int kw = k >> 2;
    // SEL: the group's finished row -> its k selected columns (selw: this lane's selector word)
    auto select_store = [&](int row_, const float4 &a_, uint32_t selw_) {
        float *buf = s_buf + g * 4 * LR;
        if (qok) *reinterpret_cast<float4 *>(buf + 4 * q) = a_;
        wave_lds_fence();
        if (q < kw) {
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int sj = (int)((selw_ >> (8 * j)) & 255u);
                o[j] = sj < D ? buf[sj] : 0.f;
            }
            reinterpret_cast<float4 *>(grad_cbsr + (int64_t)row_ * k)[q] =
                make_float4(o[0], o[1], o[2], o[3]);
        }
        wave_lds_fence();  // the copy is reused by the group's next row
    };
    {
        const int64_t span = 2 * (int64_t)chunk;
        const int n_pos = (int)(num_e - p_lo < span ? num_e - p_lo : span);
        for (int i = lane; i < n_pos; i += kWave) {
            const int c = idx[p_lo + i];
            const float wv = w[p_lo + i];
            s_idx[i] = c;
            s_sc[i] = src_div ? wv / src_div[c] : wv;
        }
        wave_lds_fence();
    }
    // edges [sb, se) of one row by the whole wave: edge sb + j to group j % NG
    auto wave_row = [&](int64_t sb, int64_t se) -> float4 {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int64_t base = sb; base < se; base += (int64_t)NG * U) {
            float4 v[U];
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = base + u * NG + g;
                v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                sc[u] = 0.f;
                if (e < se) {
                    const int i = (int)(e - p_lo);
                    sc[u] = s_sc[i];
                    if (qok) v[u] = X4[(size_t)(uint32_t)s_idx[i] * D4 + q];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) fma4(a, sc[u], v[u]);
        }
        for (int off = LR; off < kWave; off <<= 1) {
            a.x += __shfl_xor(a.x, off);
            a.y += __shfl_xor(a.y, off);
            a.z += __shfl_xor(a.z, off);
            a.w += __shfl_xor(a.w, off);
        }
        return a;
    };

    // continuation of hub row r - 1 (its token precedes d0): this item's part goes to its slab
    int cont = -1;
    if (r > 0) {
        const int64_t rp = ptr[r - 1];
        int64_t se = (int64_t)ptr[r];
        const bool hub = se - rp > chunk;
        if (d1 - r < se) se = d1 - r;
        if (hub && p_lo < se) {
            const float div = dst_div ? dst_div[r - 1] : 1.f;
            const float4 a = wave_row(p_lo, se);
            if (g == 0 && qok)
                store_row4(slab + (int64_t)item * D + 4 * q, a, dst_div != nullptr, div, false);
            cont = r - 1;
        }
    }
    if (lane == 0) slab_row[item] = cont;

    const int lmax = chunk < kDenseGroupMax ? chunk : kDenseGroupMax;
    while (r < num_rows) {
        // whole rows of at most lmax edges by the lane groups
        {
            int wb = r;  // ptr window: rows [wb, wb + 64), one per lane
            int rpw = ptr[wb + lane <= num_rows ? wb + lane : num_rows];
            int next = r;       // the next row to hand out (wave-uniform)
            bool stop = false;  // it is not the item's or is too long (wave-uniform)
            int row = -1;       // this group's row and its edge range [t, te)
            int64_t t = 0, te = 0;
            float div = 1.f;
            auto assign = [&]() {
                const uint64_t idle = __ballot(row < 0);
                for (int gi = 0; gi < NG && !stop; ++gi) {
                    if (!((idle >> (gi * LR)) & 1ull)) continue;
                    if (next + 1 >= wb + kWave) {  // slide the window (wave-uniform)
                        wb = next;
                        rpw = ptr[wb + lane <= num_rows ? wb + lane : num_rows];
                    }
                    const int64_t rb = __builtin_amdgcn_readlane(rpw, next - wb);
                    const int64_t re = __builtin_amdgcn_readlane(rpw, next + 1 - wb);
                    if (next < num_rows && next + rb < d1 && re - rb <= lmax) {
                        if (g == gi) {
                            row = next;
                            t = rb;
                            te = re;
                            div = dst_div ? dst_div[next] : 1.f;  // arrives before the store
                        }
                        ++next;
                    } else {
                        stop = true;
                    }
                }
            };
            auto gather = [&](float4 (&v)[U], float (&sc)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    sc[u] = 0.f;
                    if (row >= 0 && t + u < te) {
                        const int i = (int)(t + u - p_lo);
                        sc[u] = s_sc[i];
                        if (qok) v[u] = X4[(size_t)(uint32_t)s_idx[i] * D4 + q];
                    }
                }
            };
            assign();
            float4 v[U];
            float sc[U];
            gather(v, sc);
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            while (__ballot(row >= 0)) {
                const int crow = row;
                const float cdiv = div;
                const bool fin = crow >= 0 && t + U >= te;
                // SEL: the finished row's selector word, in flight with the next step's gathers
                uint32_t cselw = 0u;
                if (SEL && fin && q < kw) cselw = sel32[(int64_t)crow * kw + q];
                if (fin) row = -1;
                t += U;
                assign();
                float4 vn[U];
                float scn[U];
                gather(vn, scn);  // the next step's rows in flight while this step's are summed
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    fma4(a, sc[u], v[u]);
                    v[u] = vn[u];
                    sc[u] = scn[u];
                }
                if (fin) {
                    if constexpr (SEL)
                        select_store(crow, a, cselw);
                    else if (qok)
                        store_row4(out + (int64_t)crow * D + 4 * q, a, dst_div != nullptr, cdiv,
                                   add != 0);
                    a = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            r = next;
        }
        if (r >= num_rows) break;
        const int64_t rb = ptr[r];
        if (rb + r >= d1) break;
        // a longer row by the whole wave: whole up to chunk edges, else a hub row split at d1
        const int64_t re = (int64_t)ptr[r + 1];
        const bool hub = re - rb > chunk;
        const int64_t se = hub && d1 - r - 1 < re ? d1 - r - 1 : re;
        const float div = dst_div ? dst_div[r] : 1.f;
        const uint32_t selw = SEL && q < kw ? sel32[(int64_t)r * kw + q] : 0u;
        const float4 a = wave_row(rb, se);
        if (g == 0) {
            if (SEL && !hub)
                select_store(r, a, selw);
            else if (qok)
                store_row4(out + (int64_t)r * D + 4 * q, a, dst_div != nullptr, div, add != 0);
        }
        ++r;
    }
}

// The forward walk and the backward's selecting walk as two kernels (two names in profiles)
template <int LR, int U>
__global__ __launch_bounds__(kBlock, U <= 4 ? 6 : 4) void dense_rows_kernel(
    const int32_t *__restrict__ ptr, const int32_t *__restrict__ idx, const float *__restrict__ w,
    const float *__restrict__ X, int D, const float *__restrict__ dst_div, float *__restrict__ out,
    int add, float *__restrict__ slab, int32_t *__restrict__ slab_row, int num_rows,
    int64_t num_e, int chunk, int n_items) {
    dense_rows_body<LR, U, false>(ptr, idx, w, nullptr, X, D, dst_div, out, add, slab, slab_row,
                                  num_rows, num_e, chunk, n_items, nullptr, nullptr, 0);
}
template <int LR, int U>
__global__ __launch_bounds__(kBlock, U <= 4 ? 6 : 4) void dense_select_rows_kernel(
    const int32_t *__restrict__ ptr, const int32_t *__restrict__ idx, const float *__restrict__ w,
    const float *__restrict__ src_div, const float *__restrict__ X, int D, float *__restrict__ Y,
    float *__restrict__ slab, int32_t *__restrict__ slab_row, int num_rows, int64_t num_e,
    int chunk, int n_items, const uint8_t *__restrict__ sel, float *__restrict__ grad_cbsr,
    int k) {
    dense_rows_body<LR, U, true>(ptr, idx, w, src_div, X, D, nullptr, Y, 0, slab, slab_row,
                                 num_rows, num_e, chunk, n_items, sel, grad_cbsr, k);
}

// The backward at k < D / 2 (the destination-ordered walk without a dense Y): lane groups of
// LR = pow2ceil(k) lanes, lane l of a group holding selector l of its destination row for the
// whole row and gathering G[src, sel[c, l]] for each of the row's edges (one dword per lane;
// the group's k columns of one G row share its few lines), summed in registers and stored as
// grad_cbsr[c, l] directly.  Rows, items, staging and hub rows as in dense_rows_kernel; a hub
// row's owner stores its partial to grad_cbsr and later items to their slabs (k floats), added
// by slab_fixup_kernel<1>.  Selectors >= D read 0.
template <int LR, int U>
__global__ __launch_bounds__(kBlock, U <= 4 ? 6 : 4) void pick_rows_kernel(
    const int32_t *__restrict__ ptr, const int32_t *__restrict__ idx, const float *__restrict__ w,
    const float *__restrict__ src_div, const float *__restrict__ G, int D,
    const uint8_t *__restrict__ sel, int k, float *__restrict__ grad_cbsr,
    float *__restrict__ slab, int32_t *__restrict__ slab_row, int num_rows, int64_t num_e,
    int chunk, int n_items) {
    constexpr int NG = kWave / LR;
    extern __shared__ __attribute__((aligned(16))) int32_t s_stage[];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int item = (int)blockIdx.x * kWavesPerBlock + wid;
    if (item >= n_items) return;  // whole wave; no workgroup barrier below
    const int g = lane / LR, q = lane % LR;
    const bool qok = q < k;
    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int r = wave_first_row_token(ptr, num_rows, d0);
    const int64_t p_lo = d0 - r;
    int32_t *s_idx = s_stage + (size_t)wid * 4 * chunk;
    float *s_sc = reinterpret_cast<float *>(s_idx + 2 * chunk);
    {
        const int64_t span = 2 * (int64_t)chunk;
        const int n_pos = (int)(num_e - p_lo < span ? num_e - p_lo : span);
        for (int i = lane; i < n_pos; i += kWave) {
            const int c = idx[p_lo + i];
            const float wv = w[p_lo + i];
            s_idx[i] = c;
            s_sc[i] = src_div ? wv / src_div[c] : wv;
        }
        wave_lds_fence();
    }
    // this lane's column of row c (D: reads 0)
    auto col_of = [&](int c) -> int {
        const int sv = qok ? (int)sel[(int64_t)c * k + q] : D;
        return sv < D ? sv : D;
    };
    auto load = [&](int i, int col) -> float {
        return col < D ? G[(size_t)(uint32_t)s_idx[i] * D + col] : 0.f;
    };
    auto wave_row = [&](int64_t sb, int64_t se, int col) -> float {
        float a = 0.f;
        for (int64_t base = sb; base < se; base += (int64_t)NG * U) {
            float v[U], sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = base + u * NG + g;
                v[u] = 0.f;
                sc[u] = 0.f;
                if (e < se) {
                    const int i = (int)(e - p_lo);
                    sc[u] = s_sc[i];
                    v[u] = load(i, col);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) a = __builtin_fmaf(sc[u], v[u], a);
        }
        for (int off = LR; off < kWave; off <<= 1) a += __shfl_xor(a, off);
        return a;
    };

    int cont = -1;
    if (r > 0) {
        const int64_t rp = ptr[r - 1];
        int64_t se = (int64_t)ptr[r];
        const bool hub = se - rp > chunk;
        if (d1 - r < se) se = d1 - r;
        if (hub && p_lo < se) {
            const float a = wave_row(p_lo, se, col_of(r - 1));
            if (g == 0 && qok) slab[(int64_t)item * k + q] = a;
            cont = r - 1;
        }
    }
    if (lane == 0) slab_row[item] = cont;

    const int lmax = chunk < kDenseGroupMax ? chunk : kDenseGroupMax;
    while (r < num_rows) {
        {
            int wb = r;
            int rpw = ptr[wb + lane <= num_rows ? wb + lane : num_rows];
            int next = r;
            bool stop = false;
            int row = -1, col = D;
            int64_t t = 0, te = 0;
            auto assign = [&]() {
                const uint64_t idle = __ballot(row < 0);
                for (int gi = 0; gi < NG && !stop; ++gi) {
                    if (!((idle >> (gi * LR)) & 1ull)) continue;
                    if (next + 1 >= wb + kWave) {
                        wb = next;
                        rpw = ptr[wb + lane <= num_rows ? wb + lane : num_rows];
                    }
                    const int64_t rb = __builtin_amdgcn_readlane(rpw, next - wb);
                    const int64_t re = __builtin_amdgcn_readlane(rpw, next + 1 - wb);
                    if (next < num_rows && next + rb < d1 && re - rb <= lmax) {
                        if (g == gi) {
                            row = next;
                            t = rb;
                            te = re;
                            col = col_of(next);
                        }
                        ++next;
                    } else {
                        stop = true;
                    }
                }
            };
            auto gather = [&](float (&v)[U], float (&sc)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    v[u] = 0.f;
                    sc[u] = 0.f;
                    if (row >= 0 && t + u < te) {
                        const int i = (int)(t + u - p_lo);
                        sc[u] = s_sc[i];
                        v[u] = load(i, col);
                    }
                }
            };
            assign();
            float v[U], sc[U];
            gather(v, sc);
            float a = 0.f;
            while (__ballot(row >= 0)) {
                const int crow = row;
                const bool fin = crow >= 0 && t + U >= te;
                if (fin) row = -1;
                t += U;
                assign();
                float vn[U], scn[U];
                gather(vn, scn);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    a = __builtin_fmaf(sc[u], v[u], a);
                    v[u] = vn[u];
                    sc[u] = scn[u];
                }
                if (fin) {
                    if (qok) grad_cbsr[(int64_t)crow * k + q] = a;
                    a = 0.f;
                }
            }
            r = next;
        }
        if (r >= num_rows) break;
        const int64_t rb = ptr[r];
        if (rb + r >= d1) break;
        const int64_t re = (int64_t)ptr[r + 1];
        const bool hub = re - rb > chunk;
        const int64_t se = hub && d1 - r - 1 < re ? d1 - r - 1 : re;
        const float a = wave_row(rb, se, col_of(r));
        if (g == 0 && qok) grad_cbsr[(int64_t)r * k + q] = a;  // a hub row's owner: its partial
        ++r;
    }
}

// The rows split over items (the backward): per run of items continuing one row, the owner's
// partial Y[row] plus the slabs in item order (dense_rows_kernel's slab rule, as
// slab_fixup_kernel), then the row's k selected columns into grad_cbsr.  16 lanes per item.
__global__ __launch_bounds__(kBlock) void dense_fixup_select_kernel(
    const float *__restrict__ slab, const int32_t *__restrict__ slab_row,
    const float *__restrict__ Y, const uint8_t *__restrict__ sel, float *__restrict__ grad_cbsr,
    int D, int k, int n_items) {
    __shared__ __attribute__((aligned(16))) float s_row[kBlock / 16][kMaxDim];
    const int item = (int)((blockIdx.x * (int64_t)kBlock + threadIdx.x) / 16);
    const int g = threadIdx.x % 16, gl = threadIdx.x / 16;
    if (item >= n_items) return;
    const int row = slab_row[item];
    if (row < 0 || (item > 0 && slab_row[item - 1] == row)) return;
    int n = 1;
    while (item + n < n_items && slab_row[item + n] == row) ++n;
    for (int j = 4 * g; j < D; j += 64) {
        float4 a = *reinterpret_cast<const float4 *>(Y + (int64_t)row * D + j);
        for (int i = 0; i < n; ++i) {
            const float4 b = *reinterpret_cast<const float4 *>(slab + (int64_t)(item + i) * D + j);
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
        *reinterpret_cast<float4 *>(&s_row[gl][j]) = a;
    }
    wave_lds_fence();
    const uint32_t *sel32 = reinterpret_cast<const uint32_t *>(sel);
    for (int wv = g; wv < (k >> 2); wv += 16) {
        const uint32_t s = sel32[(int64_t)row * (k >> 2) + wv];
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int sj = (int)((s >> (8 * j)) & 255u);
            o[j] = sj < D ? s_row[gl][sj] : 0.f;
        }
        reinterpret_cast<float4 *>(grad_cbsr + (int64_t)row * k)[wv] =
            make_float4(o[0], o[1], o[2], o[3]);
    }
}

// source row of every CSC slot (the CSR row holding edge csc_eid[t]) and its weight
__global__ __launch_bounds__(kBlock) void dense_plan_kernel(const int32_t *__restrict__ row_ptr,
                                                            const float *__restrict__ edge_val,
                                                            const int32_t *__restrict__ csc_eid,
                                                            int num_rows, int64_t num_e,
                                                            int32_t *__restrict__ t_src,
                                                            float *__restrict__ t_w) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < num_e; t += stride) {
        const int e = csc_eid[t];
        int lo = 0, hi = num_rows - 1;  // the last row r with row_ptr[r] <= e
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (row_ptr[mid] <= e) lo = mid; else hi = mid - 1;
        }
        t_src[t] = lo;
        t_w[t] = edge_val[e];
    }
}

int dense_lanes(int D) {
    int lr = 1;
    while (lr * 4 < D) lr <<= 1;
    return lr;
}

// Resident waves of dense_rows_kernel on the whole device (the occupancy API on the kernel
// that launches, times the CUs; MAXK_DENSE_WAVES per CU x 256 CUs when no device answers).
// The occupancy is cached per (device, lane group, kind): the item size, and so the workspace
// size, stays the same for the whole process on each device.
// kind: 0 dense_rows_kernel, 1 its selecting form, 2 pick_rows_kernel
template <int LR>
int rows_blocks_per_cu(int kind) {
    int b = 0;
    const size_t lds = (size_t)kWavesPerBlock * (256 * 16 + (kind == 1 ? 16 * kWave : 0));
    const hipError_t e =
        kind == 2   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                          &b, pick_rows_kernel<LR, MAXK_DENSE_U>, kBlock, lds)
        : kind == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                          &b, dense_select_rows_kernel<LR, MAXK_DENSE_U>, kBlock, lds)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                          &b, dense_rows_kernel<LR, MAXK_DENSE_U>, kBlock, lds);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return b;
}

int64_t dense_slots(int lr, int kind) {
    // workgroups per CU, per device (a process with mixed devices sizes each from
    // its own occupancy and CU count); every thread computes the same value
    constexpr int kDevs = 16;
    static std::atomic<int> cache[kDevs][8][3] = {};
    int li = 0;
    while ((1 << li) < lr) ++li;
    const int dev = device_ordinal();
    int bpc = dev < kDevs ? cache[dev][li][kind].load(std::memory_order_relaxed) : 0;
    if (bpc == 0) {
        switch (lr) {
            case 1: bpc = rows_blocks_per_cu<1>(kind); break;
            case 2: bpc = rows_blocks_per_cu<2>(kind); break;
            case 4: bpc = rows_blocks_per_cu<4>(kind); break;
            case 8: bpc = rows_blocks_per_cu<8>(kind); break;
            case 16: bpc = rows_blocks_per_cu<16>(kind); break;
            case 32: bpc = rows_blocks_per_cu<32>(kind); break;
            default: bpc = rows_blocks_per_cu<64>(kind); break;
        }
        if (bpc <= 0) bpc = -1;  // no device answered: the fixed fallback below
        if (dev < kDevs) cache[dev][li][kind].store(bpc, std::memory_order_relaxed);
    }
    return bpc > 0 ? (int64_t)bpc * kWavesPerBlock * device_cus() : 256LL * MAXK_DENSE_WAVES;
}

// Items sized like the forward's (fwd_chunk): all resident in one round (90 % of the wave slots,
// for uneven block placement) -- each wave is a chain of dependent gathers, and a second round
// costs a whole item's latency (items sized for 24 waves per CU on a kernel holding 20: 0.057
// against 0.044 ms) -- at least 64 and at most kDenseChunkMax tokens (the LDS stage).
int dense_chunk(int64_t tokens, int chunk, int64_t slots) {
    if (chunk > 0) return chunk < kDenseChunkMax ? chunk : kDenseChunkMax;
    int64_t c = ceil_div(tokens * 10, slots * 9);
    return (int)(c < 64 ? 64 : (c > kDenseChunkMax ? kDenseChunkMax : c));
}

struct DenseLayout {
    int chunk, n_items;
    size_t x_off, slab_off, row_off, total;
};

// x_rows: rows of the dense table the route writes (forward: num_cols source rows of X;
// backward: num_cols destination rows of Y)

// kind as rows_blocks_per_cu; width: floats per slab row (D, or k for the pick)
DenseLayout dense_layout(int64_t rows, int64_t x_rows, int64_t num_e, int D, int chunk, int kind,
                         int width) {
    DenseLayout L{};
    L.chunk = dense_chunk(rows + num_e, chunk,
                          dense_slots(kind == 2 ? lanes_per_edge(width) : dense_lanes(D), kind));
    const int64_t n = ceil_div(rows + num_e, L.chunk);
    L.n_items = (int)(n > 0 ? n : 1);
    L.x_off = 0;
    L.slab_off = al256((size_t)x_rows * D * sizeof(float));
    L.row_off = L.slab_off + al256((size_t)L.n_items * width * sizeof(float));
    L.total = L.row_off + al256((size_t)L.n_items * sizeof(int32_t));
    return L;
}

// sel / grad_cbsr given: the backward's selecting store (dense_rows_kernel SEL)
int launch_dense_rows(const DenseLayout &L, hipStream_t s, const int32_t *ptr, const int32_t *idx,
                      const float *w, const float *src_div, const float *X, int D,
                      const float *dst_div, float *out, int add, float *slab, int32_t *slab_row,
                      int rows, int64_t num_e, const uint8_t *sel = nullptr,
                      float *grad_cbsr = nullptr, int k = 0) {
    const dim3 grid((unsigned)ceil_div(L.n_items, kWavesPerBlock));
    const bool select = sel != nullptr;
    const size_t lds = (size_t)kWavesPerBlock * (L.chunk * 16 + (select ? 16 * kWave : 0));
    constexpr int U = MAXK_DENSE_U;
    switch (dense_lanes(D)) {
#define MAXK_CASE(LRV)                                                                          \
    case LRV:                                                                                   \
        if (select)                                                                             \
            hipLaunchKernelGGL((dense_select_rows_kernel<LRV, U>), grid, dim3(kBlock), lds, s,  \
                               ptr, idx, w, src_div, X, D, out, slab, slab_row, rows, num_e,    \
                               L.chunk, L.n_items, sel, grad_cbsr, k);                          \
        else                                                                                    \
            hipLaunchKernelGGL((dense_rows_kernel<LRV, U>), grid, dim3(kBlock), lds, s, ptr,    \
                               idx, w, X, D, dst_div, out, add, slab, slab_row, rows, num_e,    \
                               L.chunk, L.n_items);                                             \
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
            set_error("unsupported dense lane group for D = %d", D);
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED(select ? "dense_select_rows_kernel" : "dense_rows_kernel");
    return MAXK_OK;
}

}  // namespace

// the backward picks selected columns (pick_rows_kernel) below k = D / 2 (MAXK_DENSE_PICK)
bool dense_pick(int D, int k) { return MAXK_DENSE_PICK && 2 * k < D && k <= kWave; }

bool dense_route(int D, int k) {
    return MAXK_DENSE_ROUTE && D % 4 == 0 && D <= MAXK_DENSE_DMAX && k % 4 == 0 && 2 * k >= D;
}

size_t dense_forward_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e, int D,
                                    int chunk) {
    return dense_layout(num_rows, num_cols, num_e, D, chunk, 0, D).total;
}

int dense_forward(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                  const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div,
                  float *out, int64_t num_rows, int64_t num_cols, int64_t num_e, int D, int k,
                  int chunk, void *workspace, size_t workspace_bytes, hipStream_t s,
                  int accumulate) {
    const DenseLayout L = dense_layout(num_rows, num_cols, num_e, D, chunk, 0, D);
    MAXK_REQUIRE(workspace && workspace_bytes >= L.total,
                 "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    char *ws = reinterpret_cast<char *>(workspace);
    float *X = reinterpret_cast<float *>(ws + L.x_off);
    float *slab = reinterpret_cast<float *>(ws + L.slab_off);
    int32_t *slab_row = reinterpret_cast<int32_t *>(ws + L.row_off);
    if (num_cols > 0 && num_e > 0) {
        const int vpw = kDenseBlock / (k / 4);
        const int64_t groups = ceil_div(num_cols, (int64_t)vpw);
        hipLaunchKernelGGL(cbsr_dense_kernel,
                           dim3((unsigned)(groups < MAXK_PACK_GRID ? groups : MAXK_PACK_GRID)),
                           dim3(kDenseBlock), 0, s, cbsr_val, cbsr_idx, X, (int)num_cols, k, D);
        MAXK_LAUNCHED("cbsr_dense_kernel");
    }
    if (int rc = launch_dense_rows(L, s, row_ptr, col_idx, edge_val, nullptr, X, D, row_div, out,
                                   accumulate & 1, slab, slab_row, (int)num_rows, num_e))
        return rc;
    return launch_slab_fixup<0>(slab, slab_row, out, D, L.n_items, s);
}

}  // namespace maxk

using namespace maxk;

extern "C" int maxk_dense_plan(const int32_t *row_ptr, const float *edge_val,
                               const int32_t *csc_eid, int64_t num_rows, int64_t num_e,
                               int32_t *t_src, float *t_w, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31) && num_e >= 0 && num_e < (1LL << 31),
                 "num_rows/num_e out of range");
    if (num_e == 0) return MAXK_OK;
    MAXK_REQUIRE(num_rows > 0, "edges present but num_rows == 0");
    MAXK_REQUIRE(row_ptr && edge_val && csc_eid && t_src && t_w, "pointers must not be NULL");
    const int64_t blocks = ceil_div(num_e, kBlock);
    hipLaunchKernelGGL(dense_plan_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)),
                       dim3(kBlock), 0, as_stream(stream), row_ptr, edge_val, csc_eid,
                       (int)num_rows, num_e, t_src, t_w);
    MAXK_LAUNCHED("dense_plan_kernel");
    return MAXK_OK;
}

extern "C" int maxk_dense_route(int32_t dim_origin, int32_t dim_k) {
    return dense_route(dim_origin, dim_k) ? 1 : 0;
}

extern "C" size_t maxk_sspmm_backward_dense_workspace_size(int64_t num_rows, int64_t num_cols,
                                                           int64_t num_e, int32_t dim_origin,
                                                           int32_t dim_k, int32_t chunk_edges) {
    (void)num_rows;
    if (num_cols < 0 || num_e < 0 || dim_origin <= 0 || dim_k <= 0) return 0;
    const int D = dim_origin, k = dim_k;
    if (dense_pick(D, k)) return dense_layout(num_cols, 0, num_e, D, chunk_edges, 2, k).total;
    return dense_layout(num_cols, num_cols, num_e, D, chunk_edges, 1, D).total;
}

extern "C" int maxk_sspmm_backward_dense(const int32_t *col_ptr, const int32_t *t_src,
                                         const float *t_w, const float *grad_out,
                                         const float *row_div, const uint8_t *cbsr_idx,
                                         float *grad_cbsr, int64_t num_rows, int64_t num_cols,
                                         int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                         int32_t chunk_edges, void *workspace,
                                         size_t workspace_bytes, void *stream) {
    clear_error();
    const int D = dim_origin, k = dim_k;
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31) && num_cols >= 0 &&
                     num_cols < (1LL << 31) && num_e >= 0 && num_e < (1LL << 31),
                 "num_rows/num_cols/num_e out of range");
    MAXK_REQUIRE(D >= 4 && D <= kMaxDim && D % 4 == 0, "dense backward needs dim_origin %% 4 == 0 "
                 "in [4, 256], got %d", D);
    MAXK_REQUIRE(k >= 4 && k <= D && k % 4 == 0, "dense backward needs dim_k %% 4 == 0 in [4, "
                 "dim_origin], got %d", k);
    MAXK_REQUIRE(chunk_edges >= 0, "chunk_edges must be >= 0");
    if (num_cols == 0) return MAXK_OK;
    MAXK_REQUIRE(col_ptr && cbsr_idx && grad_cbsr, "col_ptr/cbsr_idx/grad_cbsr must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (t_src && t_w && grad_out), "plan/grad pointers must not be NULL");
    MAXK_REQUIRE(((uintptr_t)cbsr_idx & 3) == 0 && ((uintptr_t)grad_cbsr & 15) == 0 &&
                     ((uintptr_t)grad_out & 15) == 0,
                 "dense backward needs 4-B aligned selectors and 16-B aligned G / grad_cbsr");
    hipStream_t s = as_stream(stream);
    if (dense_pick(D, k)) {
        const DenseLayout L = dense_layout(num_cols, 0, num_e, D, chunk_edges, 2, k);
        MAXK_REQUIRE(workspace && workspace_bytes >= L.total,
                     "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
        char *ws = reinterpret_cast<char *>(workspace);
        float *slab = reinterpret_cast<float *>(ws + L.slab_off);
        int32_t *slab_row = reinterpret_cast<int32_t *>(ws + L.row_off);
        const dim3 grid((unsigned)ceil_div(L.n_items, kWavesPerBlock));
        const size_t lds = (size_t)kWavesPerBlock * L.chunk * 16;
        constexpr int U = MAXK_DENSE_U;
        switch (lanes_per_edge(k)) {
#define MAXK_CASE(LRV)                                                                         \
    case LRV:                                                                                  \
        hipLaunchKernelGGL((pick_rows_kernel<LRV, U>), grid, dim3(kBlock), lds, s, col_ptr,    \
                           t_src, t_w, row_div, grad_out, D, cbsr_idx, k, grad_cbsr, slab,     \
                           slab_row, (int)num_cols, num_e, L.chunk, L.n_items);               \
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
                set_error("unsupported lane group for k = %d", k);
                return MAXK_ERR_INVALID;
        }
        MAXK_LAUNCHED("pick_rows_kernel");
        return launch_slab_fixup<1>(slab, slab_row, grad_cbsr, k, L.n_items, s);
    }
    const DenseLayout L = dense_layout(num_cols, num_cols, num_e, D, chunk_edges, 1, D);
    MAXK_REQUIRE(workspace && workspace_bytes >= L.total,
                 "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    char *ws = reinterpret_cast<char *>(workspace);
    float *Y = reinterpret_cast<float *>(ws + L.x_off);
    float *slab = reinterpret_cast<float *>(ws + L.slab_off);
    int32_t *slab_row = reinterpret_cast<int32_t *>(ws + L.row_off);
    if (int rc = launch_dense_rows(L, s, col_ptr, t_src, t_w, row_div, grad_out, D, nullptr, Y, 0,
                                   slab, slab_row, (int)num_cols, num_e, cbsr_idx, grad_cbsr,
                                   k))
        return rc;
    hipLaunchKernelGGL(dense_fixup_select_kernel, dim3((unsigned)ceil_div(L.n_items, kBlock / 16)),
                       dim3(kBlock), 0, s, slab, slab_row, Y, cbsr_idx, grad_cbsr, D, k,
                       L.n_items);
    MAXK_LAUNCHED("dense_fixup_select_kernel");
    return MAXK_OK;
}
