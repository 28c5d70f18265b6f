// Backward outer-product sampled SpMM (SSpMM) for gfx950:
//   grad_cbsr[c, l] = sum_{e=(r->c)} val[e] * G[r, sel[c, l]] / row_div[r]
//
// Semantics: kernels/spmm_maxk_backward.cu:15-115 (push from the CSR of A, which
// yields the A^T product) and the /out_degrees of maxk_spgemm_function.py:154-155.
// Design:
//  * Same token-stream work partition as the forward (common.h): one wave per
//    item of C tokens, so hub rows are split and short rows are batched.
//  * Per row r of the item: the wave stages G[r, :] / row_div[r] into a
//    256-float LDS row (16-B loads), then walks the row's edges with
//    KG = pow2ceil(k) lanes per edge: lane l reads sel[c, l] (u8), takes
//    G_lds[sel] and issues one global fp32 atomic add into grad_cbsr[c, l].
//    A wave step therefore adds 64/KG contiguous k-float rows -- the
//    "contiguous segments" atomic shape of the MI355X guide.
//  * grad_cbsr is zeroed by hipMemsetAsync on the same stream first.
#include "common.h"

namespace maxk {
namespace {

template <int KG, int U>
__device__ __forceinline__ void push_edges(const float *g_lds, const int32_t *__restrict__ col_idx,
                                           const float *__restrict__ edge_val,
                                           const uint8_t *__restrict__ cbsr_idx,
                                           float *__restrict__ grad_cbsr, int64_t sb, int64_t se,
                                           int k, int lane) {
    constexpr int G = kWave / KG;
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
            int s[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (c[u] >= 0) s[u] = cbsr_idx[c[u] * k + l];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (c[u] >= 0) atomicAdd(&grad_cbsr[c[u] * k + l], w[u] * g_lds[s[u]]);
        }
    }
}

// g_lds[0:D] = grad[0:D] / div   (one wave; g_lds[D:256] stays 0)
__device__ __forceinline__ void stage_row(float *g_lds, const float *__restrict__ grad, int D,
                                          float div, bool scale, int lane) {
    wave_lds_fence();
    if ((D & 3) == 0) {
        for (int j = lane * 4; j < D; j += kWave * 4) {
            float4 a = *reinterpret_cast<const float4 *>(&grad[j]);
            if (scale) {
                a.x = a.x / div;
                a.y = a.y / div;
                a.z = a.z / div;
                a.w = a.w / div;
            }
            *reinterpret_cast<float4 *>(&g_lds[j]) = a;
        }
    } else {
        for (int j = lane; j < D; j += kWave) g_lds[j] = scale ? grad[j] / div : grad[j];
    }
    wave_lds_fence();
}

template <int KG, int U>
__global__ __launch_bounds__(kBlock) void sspmm_bwd_kernel(
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col_idx,
    const float *__restrict__ edge_val, const float *__restrict__ grad,
    const float *__restrict__ row_div, const uint8_t *__restrict__ cbsr_idx,
    float *__restrict__ grad_cbsr, int num_rows, int64_t num_e, int D, int k, int chunk,
    int n_items) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int item = blockIdx.x * kWavesPerBlock + wid;
    if (item >= n_items) return;
    float *g_lds = lds[wid];
    *reinterpret_cast<float4 *>(&g_lds[lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);

    const int64_t total = (int64_t)num_rows + num_e;
    const int64_t d0 = (int64_t)item * chunk;
    const int64_t d1 = d0 + chunk < total ? d0 + chunk : total;
    int r = wave_first_row_token(row_ptr, num_rows, d0);

    if (r > 0) {  // continuation of row r-1
        const int64_t sb = d0 - r;
        int64_t se = (int64_t)row_ptr[r];
        if (d1 - r < se) se = d1 - r;
        if (sb < se) {
            const float div = row_div ? row_div[r - 1] : 1.f;
            stage_row(g_lds, grad + (int64_t)(r - 1) * D, D, div, row_div != nullptr, lane);
            push_edges<KG, U>(g_lds, col_idx, edge_val, cbsr_idx, grad_cbsr, sb, se, k, lane);
        }
    }
    for (; r < num_rows; ++r) {
        const int64_t rb = row_ptr[r];
        if (rb + r >= d1) break;
        int64_t se = (int64_t)row_ptr[r + 1];
        if (d1 - r - 1 < se) se = d1 - r - 1;
        if (rb >= se) continue;  // empty row: nothing to push
        const float div = row_div ? row_div[r] : 1.f;
        stage_row(g_lds, grad + (int64_t)r * D, D, div, row_div != nullptr, lane);
        push_edges<KG, U>(g_lds, col_idx, edge_val, cbsr_idx, grad_cbsr, rb, se, k, lane);
    }
}

template <int KG>
void launch_bwd(dim3 grid, hipStream_t s, const int32_t *row_ptr, const int32_t *col_idx,
                const float *edge_val, const float *grad, const float *row_div,
                const uint8_t *cbsr_idx, float *grad_cbsr, int num_rows, int64_t num_e, int D,
                int k, int chunk, int n_items) {
    constexpr int U = KG >= 8 ? 8 : 4;
    hipLaunchKernelGGL((sspmm_bwd_kernel<KG, U>), grid, dim3(kBlock), 0, s, row_ptr, col_idx,
                       edge_val, grad, row_div, cbsr_idx, grad_cbsr, num_rows, num_e, D, k, chunk,
                       n_items);
}

int bwd_chunk(int64_t num_rows, int64_t num_e, int32_t chunk) {
    if (chunk > 0) return chunk;
    const int64_t total = num_rows + num_e;
    int64_t c = ceil_div(total, 256LL * 32 * 8);
    c = c < 256 ? 256 : (c > 2048 ? 2048 : c);
    return (int)c;
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
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(dim_origin >= 1 && dim_origin <= kMaxDim, "dim_origin must be in [1,256], got %d",
                 dim_origin);
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= dim_origin, "dim_k must be in [1,dim_origin], got %d",
                 dim_k);
    MAXK_REQUIRE(chunk_edges >= 0, "chunk_edges must be >= 0");
    MAXK_REQUIRE(num_cols * (int64_t)dim_k < (1LL << 31), "num_cols*k too large");
    hipStream_t s = as_stream(stream);
    if (num_cols > 0) {
        MAXK_REQUIRE(grad_cbsr != nullptr, "grad_cbsr must not be NULL");
        MAXK_HIP(hipMemsetAsync(grad_cbsr, 0, (size_t)num_cols * dim_k * sizeof(float), s));
    }
    if (num_rows == 0 || num_e == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && col_idx && edge_val && grad_out && cbsr_idx,
                 "CSR/grad/selector pointers must not be NULL");
    MAXK_REQUIRE(num_cols > 0, "edges present but num_cols == 0");

    const int chunk = bwd_chunk(num_rows, num_e, chunk_edges);
    const int64_t n64 = ceil_div(num_rows + num_e, chunk);
    const int n_items = (int)(n64 > 0 ? n64 : 1);
    const dim3 grid((unsigned)ceil_div(n_items, kWavesPerBlock));
    const int nr = (int)num_rows, D = dim_origin, k = dim_k;
    switch (lanes_per_edge(dim_k)) {
#define MAXK_CASE(KGV)                                                                      \
    case KGV:                                                                               \
        launch_bwd<KGV>(grid, s, row_ptr, col_idx, edge_val, grad_out, row_div, cbsr_idx,   \
                        grad_cbsr, nr, num_e, D, k, chunk, n_items);                        \
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
