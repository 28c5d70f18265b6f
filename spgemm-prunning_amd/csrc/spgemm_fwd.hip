// Forward row-wise-product SpGEMM for gfx950:  out = diag(1/row_div) . A . scatter(CBSR)
//
// Semantics: kernels/spmm_maxk.cu:17-106 (spmm_kernel_opt2_sparse_v3) and the
// /in_degrees of maxk_spgemm_function.py:85-86.  Design (not a translation):
//
//  * Work partition: the CSR is read as one token stream of V row tokens and E
//    edge tokens (row r's token sits at r + row_ptr[r], edge e of row q at
//    e + q + 1).  Work item i = one wavefront = tokens [i*C, (i+1)*C), so every
//    wave gets <= C edges AND <= C rows whatever the degree skew (hub rows are
//    split, runs of empty rows are shared).  The reference's warp4 side file is
//    not needed; the wave finds its first row with a 64-ary search of row_ptr.
//  * Per wave: a 256-float LDS accumulator (one output row).  Lanes are grouped
//    KG = pow2ceil(k) per edge, 64/KG edges per wave step, U steps in flight;
//    each lane gathers cbsr_val[c,l] (f32) + cbsr_idx[c,l] (u8) and does one
//    ds_add_f32 into acc[sel] (LDS atomics: duplicate selectors and edges that
//    hit the same column in one step are both safe).
//  * Write-back: a row whose tokens all sit in this item is stored once with
//    16-B stores, already divided by row_div (no zero-init, no global atomics).
//    A hub row continued from the previous item goes to a per-item slab; a
//    second tiny kernel adds the slabs of each split row in item order
//    (deterministic) onto the owner's partial.
#include "common.h"

namespace maxk {
namespace {

template <int KG, int U>
struct EdgeWalker {
    static constexpr int G = kWave / KG;  // edges per wave step

    // acc[sel[c, l]] += val[e] * cbsr_val[c, l] for e in [sb, se)
    __device__ __forceinline__ static void run(float *acc, const int32_t *__restrict__ col_idx,
                                               const float *__restrict__ edge_val,
                                               const float *__restrict__ cbsr_val,
                                               const uint8_t *__restrict__ cbsr_idx,
                                               int64_t sb, int64_t se, int k, int lane) {
        const int grp = lane / KG;
        const int l0 = lane % KG;
        for (int64_t base = sb; base < se; base += (int64_t)G * U) {
            int c[U];
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = base + u * G + grp;
                const bool ok = e < se;
                c[u] = ok ? col_idx[e] : -1;
                w[u] = ok ? edge_val[e] : 0.f;
            }
            for (int l = l0; l < k; l += KG) {
                float v[U];
                int s[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (c[u] >= 0) {
                        const int q = c[u] * k + l;  // num_cols*k < 2^31 (host check)
                        v[u] = cbsr_val[q];
                        s[u] = cbsr_idx[q];
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (c[u] >= 0) atomicAdd(&acc[s[u]], w[u] * v[u]);
            }
        }
    }
};

// dst[0:D] = acc[0:D] / div ; acc[0:D] = 0   (one wave)
__device__ __forceinline__ void flush_row(float *acc, float *__restrict__ dst, int D, float div,
                                          bool scale, int lane) {
    wave_lds_fence();
    if ((D & 3) == 0) {
        for (int j = lane * 4; j < D; j += kWave * 4) {
            float4 a = *reinterpret_cast<float4 *>(&acc[j]);
            if (scale) {
                a.x = a.x / div;
                a.y = a.y / div;
                a.z = a.z / div;
                a.w = a.w / div;
            }
            *reinterpret_cast<float4 *>(&dst[j]) = a;
            *reinterpret_cast<float4 *>(&acc[j]) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else {
        for (int j = lane; j < D; j += kWave) {
            const float a = acc[j];
            dst[j] = scale ? a / div : a;
            acc[j] = 0.f;
        }
    }
    wave_lds_fence();
}

template <int KG, int U>
__global__ __launch_bounds__(kBlock) void spgemm_fwd_kernel(
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col_idx,
    const float *__restrict__ edge_val, const float *__restrict__ cbsr_val,
    const uint8_t *__restrict__ cbsr_idx, const float *__restrict__ row_div,
    float *__restrict__ out, float *__restrict__ slab, int32_t *__restrict__ slab_row,
    int num_rows, int64_t num_e, int D, int k, int chunk, int n_items) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int item = blockIdx.x * kWavesPerBlock + wid;
    if (item >= n_items) return;  // whole wave; no workgroup barrier below
    float *acc = lds[wid];
    *reinterpret_cast<float4 *>(&acc[lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);

    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;

    int r = wave_first_row_token(row_ptr, num_rows, d0);

    // Continuation of row r-1 (its token precedes d0): edges e with e + r in [d0, d1).
    int cont = -1;
    if (r > 0) {
        const int64_t sb = d0 - r;
        int64_t se = (int64_t)row_ptr[r];
        if (d1 - r < se) se = d1 - r;
        if (sb < se) {
            EdgeWalker<KG, U>::run(acc, col_idx, edge_val, cbsr_val, cbsr_idx, sb, se, k, lane);
            const float div = row_div ? row_div[r - 1] : 1.f;
            flush_row(acc, slab + (int64_t)item * D, D, div, row_div != nullptr, lane);
            cont = r - 1;
        }
    }
    if (lane == 0) slab_row[item] = cont;

    // Rows whose token lies in [d0, d1): this item owns them.
    for (; r < num_rows; ++r) {
        const int64_t rb = row_ptr[r];
        if (rb + r >= d1) break;
        int64_t se = (int64_t)row_ptr[r + 1];
        if (d1 - r - 1 < se) se = d1 - r - 1;
        EdgeWalker<KG, U>::run(acc, col_idx, edge_val, cbsr_val, cbsr_idx, rb, se, k, lane);
        const float div = row_div ? row_div[r] : 1.f;
        flush_row(acc, out + (int64_t)r * D, D, div, row_div != nullptr, lane);
    }
}

// out[row] += sum of the slabs of split rows, in item order.  One wave per item;
// only the first item of each run of equal slab_row does the work.
__global__ __launch_bounds__(kBlock) void spgemm_fwd_fixup_kernel(
    const float *__restrict__ slab, const int32_t *__restrict__ slab_row, float *__restrict__ out,
    int D, int n_items) {
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int item = blockIdx.x * kWavesPerBlock + wid;
    if (item >= n_items) return;
    const int row = slab_row[item];
    if (row < 0) return;
    if (item > 0 && slab_row[item - 1] == row) return;
    for (int j = lane; j < D; j += kWave) {
        float a = out[(int64_t)row * D + j];
        for (int i = item; i < n_items && slab_row[i] == row; ++i) a += slab[(int64_t)i * D + j];
        out[(int64_t)row * D + j] = a;
    }
}

template <int KG>
void launch_fwd(dim3 grid, hipStream_t s, const int32_t *row_ptr, const int32_t *col_idx,
                const float *edge_val, const float *cbsr_val, const uint8_t *cbsr_idx,
                const float *row_div, float *out, float *slab, int32_t *slab_row, int num_rows,
                int64_t num_e, int D, int k, int chunk, int n_items) {
    constexpr int U = KG >= 32 ? 8 : (KG >= 8 ? 8 : 4);
    hipLaunchKernelGGL((spgemm_fwd_kernel<KG, U>), grid, dim3(kBlock), 0, s, row_ptr, col_idx,
                       edge_val, cbsr_val, cbsr_idx, row_div, out, slab, slab_row, num_rows, num_e,
                       D, k, chunk, n_items);
}

int fwd_chunk(int64_t num_rows, int64_t num_e, int32_t chunk) {
    if (chunk > 0) return chunk;
    // ~8 waves of work per resident wave slot on 256 CUs, within [256, 2048] tokens
    const int64_t total = num_rows + num_e;
    int64_t c = ceil_div(total, 256LL * 32 * 8);
    c = c < 256 ? 256 : (c > 2048 ? 2048 : c);
    return (int)c;
}

}  // namespace

size_t spgemm_fwd_items(int64_t num_rows, int64_t num_e, int32_t chunk) {
    const int64_t total = num_rows + num_e;
    const int c = fwd_chunk(num_rows, num_e, chunk);
    const int64_t n = ceil_div(total, c);
    return (size_t)(n > 0 ? n : 1);
}

}  // namespace maxk

using namespace maxk;

extern "C" size_t maxk_spgemm_forward_workspace_size(int64_t num_rows, int64_t num_e,
                                                     int32_t dim_origin, int32_t dim_k,
                                                     int32_t chunk_edges) {
    (void)dim_k;
    if (num_rows < 0 || num_e < 0 || dim_origin <= 0) return 0;
    const size_t n = spgemm_fwd_items(num_rows, num_e, chunk_edges);
    const size_t slab = ((n * (size_t)dim_origin * sizeof(float)) + 255) & ~(size_t)255;
    return slab + n * sizeof(int32_t);
}

extern "C" int maxk_spgemm_forward(const int32_t *row_ptr, const int32_t *col_idx,
                                   const float *edge_val, const float *cbsr_val,
                                   const uint8_t *cbsr_idx, const float *row_div, float *out,
                                   int64_t num_rows, int64_t num_cols, int64_t num_e,
                                   int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                   void *workspace, size_t workspace_bytes, void *stream) {
    clear_error();
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
    MAXK_REQUIRE(num_e == 0 || (col_idx && edge_val && cbsr_val && cbsr_idx),
                 "CSR/CBSR pointers must not be NULL");
    MAXK_REQUIRE(num_e == 0 || num_cols > 0, "edges present but num_cols == 0");
    const size_t need = maxk_spgemm_forward_workspace_size(num_rows, num_e, dim_origin, dim_k,
                                                           chunk_edges);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu bytes, got %zu",
                 need, workspace_bytes);

    const int chunk = fwd_chunk(num_rows, num_e, chunk_edges);
    const int n_items = (int)spgemm_fwd_items(num_rows, num_e, chunk_edges);
    float *slab = reinterpret_cast<float *>(workspace);
    const size_t slab_bytes = (((size_t)n_items * dim_origin * sizeof(float)) + 255) & ~(size_t)255;
    int32_t *slab_row = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(workspace) + slab_bytes);
    hipStream_t s = as_stream(stream);
    const dim3 grid((unsigned)ceil_div(n_items, kWavesPerBlock));
    const int kg = lanes_per_edge(dim_k);
    const int nr = (int)num_rows, D = dim_origin, k = dim_k;
    switch (kg) {
#define MAXK_CASE(KGV)                                                                         \
    case KGV:                                                                                  \
        launch_fwd<KGV>(grid, s, row_ptr, col_idx, edge_val, cbsr_val, cbsr_idx, row_div, out, \
                        slab, slab_row, nr, num_e, D, k, chunk, n_items);                      \
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
            set_error("unsupported lane group %d", kg);
            return MAXK_ERR_INVALID;
    }
    MAXK_LAUNCHED("spgemm_fwd_kernel");
    hipLaunchKernelGGL(spgemm_fwd_fixup_kernel, grid, dim3(kBlock), 0, s, slab, slab_row, out, D,
                       n_items);
    MAXK_LAUNCHED("spgemm_fwd_fixup_kernel");
    return MAXK_OK;
}
