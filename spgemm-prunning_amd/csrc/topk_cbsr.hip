// CBSR encode (MaxK top-k) and CBSR -> dense scatter for gfx950.
//
// Semantics: torch.topk(x, k, dim=1, largest=True, sorted=True) + .to(uint8)
// (maxk_spgemm_function.py:51-57); replaces the uint8 threshold-bisection
// kernel topk (kernels/maxk_kernel.cu:23-96), which is approximate (quantised
// input, index-order output, unfilled slots on ties) -- this one is exact.
//
// One wavefront per row (D <= 256, so <= 4 elements per lane, column
// j = lane + 64*i for coalesced loads):
//  1. order-preserving 32-bit keys (NaN above +inf, as torch ranks it);
//  2. the k-th largest key T by MSB-first bit construction, each bit one
//     ballot/popcount per element slot -- no LDS, no sorting of all D;
//  3. select key > T, plus the lowest-column key == T until k are taken;
//  4. compact the k winners into LDS, rank each against the others
//     (broadcast LDS reads) and store in (key desc, column asc) order.
#include "common.h"

namespace maxk {
namespace {

__device__ __forceinline__ uint32_t order_key(float x) {
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return 0xffffffffu;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t order_key(uint8_t x) { return x; }

template <typename T>
struct KeyBits {
    static constexpr int value = 32;
};
template <>
struct KeyBits<uint8_t> {
    static constexpr int value = 8;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void topk_cbsr_kernel(const T *__restrict__ x, int64_t ld_x,
                                                           T *__restrict__ out_val,
                                                           uint8_t *__restrict__ out_idx,
                                                           int32_t *__restrict__ out_idx32,
                                                           int num_rows, int D, int k) {
    __shared__ uint32_t s_key[kWavesPerBlock][kMaxDim];
    __shared__ T s_val[kWavesPerBlock][kMaxDim];
    __shared__ uint8_t s_col[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int row = blockIdx.x * kWavesPerBlock + wid;
    if (row >= num_rows) return;
    const uint64_t lt_mask = (1ull << lane) - 1ull;

    T v[4];
    uint32_t key[4];
    bool ok[4];
    const T *xr = x + (int64_t)row * ld_x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = lane + kWave * i;
        ok[i] = j < D;
        v[i] = ok[i] ? xr[j] : T(0);
        key[i] = ok[i] ? order_key(v[i]) : 0u;
    }

    // T = max t such that #{key >= t} >= k  (the k-th largest key)
    uint32_t thr = 0;
    for (int bit = KeyBits<T>::value - 1; bit >= 0; --bit) {
        const uint32_t cand = thr | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) cnt += __popcll(__ballot(ok[i] && key[i] >= cand));
        if (cnt >= k) thr = cand;
    }
    int n_gt = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) n_gt += __popcll(__ballot(ok[i] && key[i] > thr));
    const int need_eq = k - n_gt;

    // select, then compact winners into LDS slots [0, k)
    int eq_base = 0, slot_base = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool eq = ok[i] && key[i] == thr;
        const uint64_t me = __ballot(eq);
        const int eq_rank = eq_base + __popcll(me & lt_mask);
        eq_base += __popcll(me);
        const bool take = (ok[i] && key[i] > thr) || (eq && eq_rank < need_eq);
        const uint64_t mt = __ballot(take);
        if (take) {
            const int slot = slot_base + __popcll(mt & lt_mask);
            s_key[wid][slot] = key[i];
            s_val[wid][slot] = v[i];
            s_col[wid][slot] = (uint8_t)(lane + kWave * i);
        }
        slot_base += __popcll(mt);
    }
    wave_lds_fence();
    for (int p = lane; p < k; p += kWave) {
        const uint32_t kp = s_key[wid][p];
        const int cp = s_col[wid][p];
        int pos = 0;
        for (int q = 0; q < k; ++q) {
            const uint32_t kq = s_key[wid][q];
            pos += (kq > kp) || (kq == kp && (int)s_col[wid][q] < cp);
        }
        const int64_t o = (int64_t)row * k + pos;
        out_val[o] = s_val[wid][p];
        out_idx[o] = (uint8_t)cp;
        if (out_idx32) out_idx32[o] = cp;
    }
}

// dense[r, :] = 0; dense[r, idx[r, l]] = val[r, l]   (one wave per row)
__global__ __launch_bounds__(kBlock) void cbsr_scatter_dense_kernel(
    const float *__restrict__ val, const uint8_t *__restrict__ idx, float *__restrict__ dense,
    int num_rows, int D, int k) {
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock][kMaxDim];
    const int wid = threadIdx.x / kWave;
    const int lane = lane_id();
    const int row = blockIdx.x * kWavesPerBlock + wid;
    if (row >= num_rows) return;
    float *buf = lds[wid];
    *reinterpret_cast<float4 *>(&buf[lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
    wave_lds_fence();
    for (int l = lane; l < k; l += kWave) buf[idx[(int64_t)row * k + l]] = val[(int64_t)row * k + l];
    wave_lds_fence();
    float *dst = dense + (int64_t)row * D;
    if ((D & 3) == 0) {
        for (int j = lane * 4; j < D; j += kWave * 4)
            *reinterpret_cast<float4 *>(&dst[j]) = *reinterpret_cast<const float4 *>(&buf[j]);
    } else {
        for (int j = lane; j < D; j += kWave) dst[j] = buf[j];
    }
}

template <typename T>
int topk_launch(const T *x, int64_t ld_x, T *val, uint8_t *idx, int32_t *idx32, int64_t num_rows,
                int32_t D, int32_t k, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(D >= 1 && D <= kMaxDim, "dim_origin must be in [1,256], got %d", D);
    MAXK_REQUIRE(k >= 1 && k <= D, "dim_k must be in [1,dim_origin], got %d", k);
    MAXK_REQUIRE(ld_x >= D, "ld_x (%lld) < dim_origin (%d)", (long long)ld_x, D);
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(x && val && idx, "x/val/idx must not be NULL");
    const dim3 grid((unsigned)ceil_div(num_rows, kWavesPerBlock));
    hipLaunchKernelGGL(topk_cbsr_kernel<T>, grid, dim3(kBlock), 0, as_stream(stream), x, ld_x, val,
                       idx, idx32, (int)num_rows, D, k);
    MAXK_LAUNCHED("topk_cbsr_kernel");
    return MAXK_OK;
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" int maxk_topk_cbsr(const float *x, int64_t ld_x, float *cbsr_val, uint8_t *cbsr_idx,
                              int32_t *idx32, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                              void *stream) {
    return topk_launch<float>(x, ld_x, cbsr_val, cbsr_idx, idx32, num_rows, dim_origin, dim_k,
                              stream);
}

extern "C" int maxk_topk_cbsr_u8(const uint8_t *x, int64_t ld_x, uint8_t *cbsr_val,
                                 uint8_t *cbsr_idx, int32_t *idx32, int64_t num_rows,
                                 int32_t dim_origin, int32_t dim_k, void *stream) {
    return topk_launch<uint8_t>(x, ld_x, cbsr_val, cbsr_idx, idx32, num_rows, dim_origin, dim_k,
                                stream);
}

extern "C" int maxk_cbsr_scatter_dense(const float *cbsr_val, const uint8_t *cbsr_idx,
                                       float *dense, int64_t num_rows, int32_t dim_origin,
                                       int32_t dim_k, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(dim_origin >= 1 && dim_origin <= kMaxDim, "dim_origin must be in [1,256]");
    MAXK_REQUIRE(dim_k >= 1 && dim_k <= dim_origin, "dim_k must be in [1,dim_origin]");
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(cbsr_val && cbsr_idx && dense, "pointers must not be NULL");
    const dim3 grid((unsigned)ceil_div(num_rows, kWavesPerBlock));
    hipLaunchKernelGGL(cbsr_scatter_dense_kernel, grid, dim3(kBlock), 0, as_stream(stream),
                       cbsr_val, cbsr_idx, dense, (int)num_rows, dim_origin, dim_k);
    MAXK_LAUNCHED("cbsr_scatter_dense_kernel");
    return MAXK_OK;
}
