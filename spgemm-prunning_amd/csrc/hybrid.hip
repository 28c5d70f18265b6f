// Hybrid backward plan, pull locality, the "auto" backward rule, pre-divided pull entries and
// the whole hybrid backward -- the C-ABI side of what the Python binding did with PyTorch
// ops (maxk_cuda_kernels/__init__.py hybrid_plan / pull_locality / _bwd_mode /
// _scaled_entries), so a non-Python host replacing cuda_kernel_wrappers.cu:58-76 gets the
// same backward without re-deriving it.
//
// The hybrid plan splits a graph's edges by the tiles (row slice x destination bucket) of its
// pull plan: tiles holding at least density x (rows of their slice) entries are pulled
// (maxk_sspmm_backward_pull_tiles), every other edge goes through the two-phase csc backward.
// Since the CSR is sorted by (row, column), the other edges are a stable compaction of the
// CSR itself -- already a CSR, no sort needed.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.h"

namespace maxk {
namespace {

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// flag[t] = tile t is pulled; cnt_d[t] = its entries if pulled, else 0
__global__ void hybrid_flag_kernel(const int32_t *__restrict__ tile_ptr, int64_t n_tiles, int nb,
                                   int64_t num_rows, int rps, float density,
                                   int32_t *__restrict__ flag, int32_t *__restrict__ cnt_d) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const int64_t cnt = tile_ptr[t + 1] - tile_ptr[t];
    const int64_t s = t / nb;
    int64_t rows_in = num_rows - s * rps;
    rows_in = rows_in > rps ? rps : (rows_in < 1 ? 1 : rows_in);
    const bool d = cnt > 0 && (double)cnt >= (double)density * (double)rows_in;
    flag[t] = d ? 1 : 0;
    cnt_d[t] = d ? (int32_t)cnt : 0;
}

// tile_list / tile_ent of the pulled tiles (pos = exclusive scan of flag, off = of cnt_d)
__global__ void hybrid_list_kernel(const int32_t *__restrict__ flag,
                                   const int32_t *__restrict__ pos,
                                   const int32_t *__restrict__ off,
                                   const int32_t *__restrict__ cnt_d, int64_t n_tiles,
                                   int32_t *__restrict__ tile_list, int32_t *__restrict__ tile_ent,
                                   int64_t *__restrict__ totals) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    if (flag[t]) {
        tile_list[pos[t]] = (int32_t)t;
        tile_ent[pos[t]] = off[t];
    }
    if (t == n_tiles - 1) {  // the end of the last run, and the counts for the host
        const int32_t nt = pos[t] + flag[t];
        const int32_t ne = off[t] + cnt_d[t];
        tile_ent[nt] = ne;
        totals[0] = nt;
        totals[1] = ne;
    }
}

// per bucket: how many of its tiles are pulled
__global__ void hybrid_bucket_count_kernel(const int32_t *__restrict__ flag, int nb, int slices,
                                           int32_t *__restrict__ bcnt) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nb) return;
    int c = 0;
    for (int s = 0; s < slices; ++s) c += flag[(int64_t)s * nb + j];
    bcnt[j] = c;
}

// bucket_tiles[bucket_ptr[j] + rank] = position in tile_list of bucket j's pulled tiles, in
// slice order
__global__ void hybrid_bucket_fill_kernel(const int32_t *__restrict__ flag,
                                          const int32_t *__restrict__ pos,
                                          const int32_t *__restrict__ bucket_ptr, int nb,
                                          int slices, int32_t *__restrict__ bucket_tiles) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nb) return;
    int r = bucket_ptr[j];
    for (int s = 0; s < slices; ++s) {
        const int64_t t = (int64_t)s * nb + j;
        if (flag[t]) bucket_tiles[r++] = pos[t];
    }
}

// the pulled tiles' entries, tile by tile (one workgroup per tile)
__global__ void hybrid_copy_ent_kernel(const int32_t *__restrict__ tile_ptr,
                                       const int32_t *__restrict__ flag,
                                       const int32_t *__restrict__ off, int64_t n_tiles,
                                       const uint2 *__restrict__ ent, uint2 *__restrict__ ent_pull) {
    for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        if (!flag[t]) continue;
        const int b = tile_ptr[t], e = tile_ptr[t + 1];
        uint2 *dst = ent_pull + off[t] - b;
        for (int i = b + (int)threadIdx.x; i < e; i += blockDim.x) dst[i] = ent[i];
    }
}

// one wave per row: edges off the pulled tiles (count, then stable compaction)
template <bool FILL>
__global__ void hybrid_off_kernel(const int32_t *__restrict__ row_ptr,
                                  const int32_t *__restrict__ col_idx,
                                  const float *__restrict__ edge_val,
                                  const int32_t *__restrict__ flag, int64_t num_rows, int nb,
                                  int rps, int shift, int32_t *__restrict__ row_cnt,
                                  const int32_t *__restrict__ off_row_ptr,
                                  int32_t *__restrict__ off_col, float *__restrict__ off_val) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    if (r >= num_rows) return;
    const int lane = lane_id();
    const int b = row_ptr[r], e = row_ptr[r + 1];
    const int64_t base = (r / rps) * nb;
    int out = FILL ? off_row_ptr[r] : 0;
    for (int i0 = b; i0 < e; i0 += kWave) {
        const int i = i0 + lane;
        const int c = i < e ? col_idx[i] : 0;
        const bool keep = i < e && !flag[base + (c >> shift)];
        const uint64_t m = __ballot(keep);
        if (FILL && keep) {
            const int o = out + __popcll(m & ((1ull << lane) - 1ull));
            off_col[o] = c;
            off_val[o] = edge_val[i];
        }
        out += __popcll(m);
    }
    if (!FILL && lane == 0) row_cnt[r] = out;
}

// pull_locality: occupied (row, bucket) pairs, one wave per row; columns sorted within rows
__global__ void locality_kernel(const int32_t *__restrict__ row_ptr,
                                const int32_t *__restrict__ col_idx, int64_t num_rows, int shift,
                                unsigned long long *__restrict__ pairs) {
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    if (r >= num_rows) return;
    const int lane = lane_id();
    const int b = row_ptr[r], e = row_ptr[r + 1];
    unsigned n = 0;
    for (int i = b + lane; i < e; i += kWave)
        n += (i == b || (col_idx[i] >> shift) != (col_idx[i - 1] >> shift)) ? 1u : 0u;
    for (int o = kWave / 2; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if (lane == 0 && n) atomicAdd(pairs, (unsigned long long)n);
}

// ent_out = ent with each weight divided by its source row's row_div; tile i of the run list
// is tile_ids[i] (or i), its entries [tile_ent[i], tile_ent[i + 1])
__global__ void scale_ent_kernel(const uint2 *__restrict__ ent, const int32_t *__restrict__ tile_ids,
                                 const int32_t *__restrict__ tile_ent, int64_t n_runs, int nb,
                                 int rps, const float *__restrict__ row_div,
                                 uint2 *__restrict__ ent_out) {
    for (int64_t i = blockIdx.x; i < n_runs; i += gridDim.x) {
        const int64_t t = tile_ids ? tile_ids[i] : i;
        const int64_t row0 = (t / nb) * rps;
        const int b = tile_ent[i], e = tile_ent[i + 1];
        for (int x = b + (int)threadIdx.x; x < e; x += blockDim.x) {
            const uint2 v = ent[x];
            const float w = __uint_as_float(v.y) / row_div[row0 + (v.x & 0xffffu)];
            ent_out[x] = make_uint2(v.x, __float_as_uint(w));
        }
    }
}

size_t scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t *)nullptr,
                                           (int32_t *)nullptr, (int)std::max<int64_t>(n, 1));
    return bytes;
}

struct HybridWs {
    int32_t *flag, *pos, *cnt_d, *off, *bcnt, *row_cnt;
    int64_t *totals;
    void *tmp;
    size_t tmp_bytes;
};

size_t hybrid_ws_layout(int64_t num_rows, int64_t n_tiles, int64_t nb, char *base, HybridWs *w) {
    const size_t nt4 = al256((size_t)(n_tiles + 1) * 4);
    const size_t nb4 = al256((size_t)(nb + 1) * 4);
    const size_t nr4 = al256((size_t)(num_rows + 1) * 4);
    const size_t tmp = al256(std::max(scan_temp_bytes(n_tiles + 1),
                                      std::max(scan_temp_bytes(nb + 1), scan_temp_bytes(num_rows + 1))));
    size_t o = 0;
    if (w) {
        w->flag = reinterpret_cast<int32_t *>(base + o);
        w->pos = reinterpret_cast<int32_t *>(base + o + nt4);
        w->cnt_d = reinterpret_cast<int32_t *>(base + o + 2 * nt4);
        w->off = reinterpret_cast<int32_t *>(base + o + 3 * nt4);
    }
    o += 4 * nt4;
    if (w) w->bcnt = reinterpret_cast<int32_t *>(base + o);
    o += nb4;
    if (w) w->row_cnt = reinterpret_cast<int32_t *>(base + o);
    o += nr4;
    if (w) w->totals = reinterpret_cast<int64_t *>(base + o);
    o += 256;
    if (w) {
        w->tmp = base + o;
        w->tmp_bytes = tmp;
    }
    return o + tmp;
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" size_t maxk_hybrid_plan_workspace_size(int64_t num_rows, int64_t num_cols,
                                                  int64_t num_e, int32_t bucket_shift,
                                                  int32_t slices) {
    (void)num_e;
    if (num_rows < 0 || num_cols < 0 || slices <= 0 || bucket_shift < 4 || bucket_shift > 15)
        return 0;
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    return hybrid_ws_layout(num_rows, (int64_t)slices * nb, nb, nullptr, nullptr);
}

extern "C" int maxk_hybrid_plan(const int32_t *row_ptr, const int32_t *col_idx,
                                const float *edge_val, const int32_t *tile_ptr,
                                const uint32_t *ent, int64_t num_rows, int64_t num_cols,
                                int64_t num_e, int32_t bucket_shift, int32_t slices,
                                float density, int32_t *tile_list, int32_t *tile_ent,
                                int32_t *bucket_ptr, int32_t *bucket_tiles, uint32_t *ent_pull,
                                int32_t *off_row_ptr, int32_t *off_col, float *off_val,
                                int64_t *counts, void *workspace, size_t workspace_bytes,
                                void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(bucket_shift >= 4 && bucket_shift <= 15, "bucket_shift must be in [4,15]");
    MAXK_REQUIRE(density >= 0.f, "density must be >= 0");
    MAXK_REQUIRE(counts, "counts must not be NULL");
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    MAXK_REQUIRE(slices >= 1 && slices * nb < (1LL << 31), "slices %d out of range", slices);
    const int64_t rps64 = num_rows > 0 ? (num_rows + slices - 1) / slices : 1;
    MAXK_REQUIRE(rps64 <= 65536, "%d slices leave %lld rows per slice (max 65536)", slices,
                 (long long)rps64);
    const int64_t nt = slices * nb;
    MAXK_REQUIRE(tile_ptr && tile_list && tile_ent && bucket_ptr && bucket_tiles && off_row_ptr,
                 "plan pointers must not be NULL");
    MAXK_REQUIRE(num_e == 0 || (row_ptr && col_idx && edge_val && ent && ent_pull && off_col &&
                                off_val),
                 "CSR / entry pointers must not be NULL");
    const size_t need = maxk_hybrid_plan_workspace_size(num_rows, num_cols, num_e, bucket_shift,
                                                        slices);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu bytes, got %zu",
                 need, workspace_bytes);
    hipStream_t s = as_stream(stream);
    HybridWs w;
    hybrid_ws_layout(num_rows, nt, nb, reinterpret_cast<char *>(workspace), &w);
    const int rps = (int)rps64;
    if (nt > 0) {
        const dim3 gt((unsigned)ceil_div(nt, kBlock));
        hipLaunchKernelGGL(hybrid_flag_kernel, gt, dim3(kBlock), 0, s, tile_ptr, nt, (int)nb,
                           num_rows, rps, density, w.flag, w.cnt_d);
        MAXK_LAUNCHED("hybrid_flag_kernel");
        size_t tb = w.tmp_bytes;
        MAXK_HIP(hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.flag, w.pos, (int)nt, s));
        tb = w.tmp_bytes;
        MAXK_HIP(hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.cnt_d, w.off, (int)nt, s));
        hipLaunchKernelGGL(hybrid_list_kernel, gt, dim3(kBlock), 0, s, w.flag, w.pos, w.off,
                           w.cnt_d, nt, tile_list, tile_ent, w.totals);
        MAXK_LAUNCHED("hybrid_list_kernel");
        const dim3 gb((unsigned)ceil_div(nb, kBlock));
        hipLaunchKernelGGL(hybrid_bucket_count_kernel, gb, dim3(kBlock), 0, s, w.flag, (int)nb,
                           (int)slices, w.bcnt);
        MAXK_LAUNCHED("hybrid_bucket_count_kernel");
        MAXK_HIP(hipMemsetAsync(w.bcnt + nb, 0, 4, s));
        tb = w.tmp_bytes;
        MAXK_HIP(hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.bcnt, bucket_ptr, (int)(nb + 1), s));
        hipLaunchKernelGGL(hybrid_bucket_fill_kernel, gb, dim3(kBlock), 0, s, w.flag, w.pos,
                           bucket_ptr, (int)nb, (int)slices, bucket_tiles);
        MAXK_LAUNCHED("hybrid_bucket_fill_kernel");
        if (num_e > 0) {
            const int64_t grid = std::min<int64_t>(nt, 65536);
            hipLaunchKernelGGL(hybrid_copy_ent_kernel, dim3((unsigned)grid), dim3(kBlock), 0, s,
                               tile_ptr, w.flag, w.off, nt, reinterpret_cast<const uint2 *>(ent),
                               reinterpret_cast<uint2 *>(ent_pull));
            MAXK_LAUNCHED("hybrid_copy_ent_kernel");
        }
    } else {
        MAXK_HIP(hipMemsetAsync(tile_ent, 0, 4, s));
        MAXK_HIP(hipMemsetAsync(bucket_ptr, 0, (size_t)(nb + 1) * 4, s));
        MAXK_HIP(hipMemsetAsync(w.totals, 0, 16, s));
    }
    // the edges off the pulled tiles, as a CSR
    if (num_rows > 0) {
        const dim3 gr((unsigned)ceil_div(num_rows * kWave, kBlock));
        if (num_e > 0 && nt > 0) {
            hipLaunchKernelGGL(hybrid_off_kernel<false>, gr, dim3(kBlock), 0, s, row_ptr, col_idx,
                               edge_val, w.flag, num_rows, (int)nb, rps, (int)bucket_shift,
                               w.row_cnt, nullptr, nullptr, nullptr);
            MAXK_LAUNCHED("hybrid_off_kernel<0>");
        } else {
            MAXK_HIP(hipMemsetAsync(w.row_cnt, 0, (size_t)num_rows * 4, s));
        }
        MAXK_HIP(hipMemsetAsync(w.row_cnt + num_rows, 0, 4, s));
        size_t tb = w.tmp_bytes;
        MAXK_HIP(hipcub::DeviceScan::ExclusiveSum(w.tmp, tb, w.row_cnt, off_row_ptr,
                                                  (int)(num_rows + 1), s));
        if (num_e > 0 && nt > 0) {
            hipLaunchKernelGGL(hybrid_off_kernel<true>, gr, dim3(kBlock), 0, s, row_ptr, col_idx,
                               edge_val, w.flag, num_rows, (int)nb, rps, (int)bucket_shift,
                               nullptr, off_row_ptr, off_col, off_val);
            MAXK_LAUNCHED("hybrid_off_kernel<1>");
        }
    } else {
        MAXK_HIP(hipMemsetAsync(off_row_ptr, 0, 4, s));
    }
    int64_t host[2] = {0, 0};
    int32_t n_off = 0;
    MAXK_HIP(hipMemcpyAsync(host, w.totals, 16, hipMemcpyDeviceToHost, s));
    MAXK_HIP(hipMemcpyAsync(&n_off, off_row_ptr + num_rows, 4, hipMemcpyDeviceToHost, s));
    MAXK_HIP(hipStreamSynchronize(s));
    counts[0] = host[0];
    counts[1] = host[1];
    counts[2] = n_off;
    return MAXK_OK;
}

extern "C" int maxk_pull_locality(const int32_t *row_ptr, const int32_t *col_idx,
                                  int64_t num_rows, int64_t num_e, int32_t bucket_shift,
                                  double *locality, void *workspace, size_t workspace_bytes,
                                  void *stream) {
    clear_error();
    MAXK_REQUIRE(locality, "locality must not be NULL");
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31) && num_e >= 0 && num_e < (1LL << 31),
                 "num_rows / num_e out of range");
    MAXK_REQUIRE(bucket_shift >= 0 && bucket_shift <= 16, "bucket_shift must be in [0,16]");
    *locality = 0.0;
    if (num_e == 0 || num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && col_idx, "CSR pointers must not be NULL");
    MAXK_REQUIRE(workspace && workspace_bytes >= 8, "workspace too small: need 8 bytes");
    hipStream_t s = as_stream(stream);
    auto *pairs = reinterpret_cast<unsigned long long *>(workspace);
    MAXK_HIP(hipMemsetAsync(pairs, 0, 8, s));
    hipLaunchKernelGGL(locality_kernel, dim3((unsigned)ceil_div(num_rows * kWave, kBlock)),
                       dim3(kBlock), 0, s, row_ptr, col_idx, num_rows, (int)bucket_shift, pairs);
    MAXK_LAUNCHED("locality_kernel");
    unsigned long long n = 0;
    MAXK_HIP(hipMemcpyAsync(&n, pairs, 8, hipMemcpyDeviceToHost, s));
    MAXK_HIP(hipStreamSynchronize(s));
    *locality = (double)num_e / (double)(n ? n : 1);
    return MAXK_OK;
}

extern "C" int maxk_pull_entries_scale(const uint32_t *ent, const int32_t *tile_ids,
                                       const int32_t *tile_ent, int64_t n_runs,
                                       int64_t num_rows, int64_t num_cols, int32_t bucket_shift,
                                       int32_t slices, const float *row_div, uint32_t *ent_out,
                                       void *stream) {
    clear_error();
    MAXK_REQUIRE(n_runs >= 0 && num_rows >= 0 && num_cols >= 0, "sizes out of range");
    MAXK_REQUIRE(bucket_shift >= 4 && bucket_shift <= 15, "bucket_shift must be in [4,15]");
    MAXK_REQUIRE(slices >= 1, "slices must be >= 1");
    if (n_runs == 0 || num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(ent && tile_ent && row_div && ent_out, "pointers must not be NULL");
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    const int rps = (int)((num_rows + slices - 1) / slices);
    hipLaunchKernelGGL(scale_ent_kernel, dim3((unsigned)std::min<int64_t>(n_runs, 65536)),
                       dim3(kBlock), 0, as_stream(stream), reinterpret_cast<const uint2 *>(ent),
                       tile_ids, tile_ent, n_runs, (int)nb, rps, row_div,
                       reinterpret_cast<uint2 *>(ent_out));
    MAXK_LAUNCHED("scale_ent_kernel");
    return MAXK_OK;
}

// The "auto" backward rule (the Python binding's _bwd_mode defers to it).
extern "C" int maxk_backward_mode_auto(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                       int32_t dim_origin, int32_t dim_k, double pull_locality) {
    const int k = dim_k;
    if (k > 0 && num_cols > 0 && dim_origin > 0 && dense_route(dim_origin, k)) return MAXK_BWD_DENSE;
    if (k <= 0 || num_cols <= 0 || (dim_origin > 0 && dim_origin % 4 != 0) || !(k % 4 == 0 || k <= 64))
        return MAXK_BWD_CSC;
    const int shift = maxk_bucket_shift(k);
    const int64_t rows = num_rows > 0 ? num_rows : num_cols;
    // at least ~1/2 edge per (source row, bucket of 2^shift columns), or a G small enough to
    // stay cache-resident (64 MiB) however sparse the graph
    const bool dense = (double)num_e * (double)(1LL << shift) >= (double)rows * (double)num_cols / 2;
    const bool small = dim_origin > 0 && (double)rows * dim_origin * 4 <= (double)(64 << 20);
    // a small, narrow G (D <= MAXK_DENSE_PICK_DMAX, cache-resident) of a sparse graph (the
    // pull's tiles share no source rows) at D / 4 <= k < D / 2: the
    // dense backward's selected-column form (pick_rows_kernel) -- Flickr-sized (configs[0]),
    // k = 16: 0.0561 against 0.0587-0.0588 ms for the pull; at k = 8 the pull stays (0.049
    // against 0.051-0.053; profiles/r05/tune/dense_pick/)
    if (small && !dense && dim_origin <= MAXK_DENSE_PICK_DMAX && 4 * k >= dim_origin && k % 4 == 0 &&
        dim_origin % 4 == 0 && dense_pick(dim_origin, k))
        return MAXK_BWD_DENSE;
    if ((dense || small) && rows <= 256LL * 65536) return MAXK_BWD_PULL;
    if (k % 4 == 0 && rows <= 256LL * 65536 && num_e > 0 && pull_locality >= MAXK_HYBRID_LOCALITY)
        return MAXK_BWD_HYBRID;
    // window-sorted contribution rows where a window holds runs of >= 2 rows per bucket
    // (ogbn-products-sized: k = 4 / 8 1.76 / 2.91 ms against csc 3.52 / 3.87 with the selector
    // stream; at k = 16 the runs are ~1 row and csc wins, 5.07 vs 5.88)
    if (k % 4 == 0 && k <= MAXK_BSORT_KMAX && num_e > 0 &&
        (double)maxk_bsort_window(k) * (double)(1LL << shift) >= 2.0 * (double)num_cols)
        return MAXK_BWD_BSORT;
    return MAXK_BWD_CSC;
}

// ---- the whole hybrid backward --------------------------------------------------------------
extern "C" size_t maxk_sspmm_backward_hybrid_workspace_size(int64_t num_rows, int64_t num_cols,
                                                            int64_t n_off_e, int32_t dim_origin,
                                                            int32_t dim_k, int64_t n_tiles) {
    const size_t a = al256(maxk_sspmm_backward_csc_workspace_size(num_rows, num_cols, n_off_e,
                                                                  dim_origin, dim_k, 0));
    const size_t b = maxk_sspmm_backward_pull_tiles_workspace_size(num_rows, num_cols, dim_origin,
                                                                   dim_k, (int32_t)n_tiles);
    return a + b;
}

extern "C" int maxk_sspmm_backward_hybrid(
    const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
    const int32_t *tile_list, const int32_t *tile_ent, int32_t n_tiles, const int32_t *bucket_ptr,
    const int32_t *bucket_tiles, const uint32_t *ent_pull, int64_t n_pull_e, int32_t bucket_shift,
    int32_t slices, const int32_t *off_row_ptr, const int32_t *off_col, const float *off_val,
    int64_t n_off_e, const int32_t *off_col_ptr, const int32_t *off_csc_eid, int32_t flags,
    float *grad_cbsr, int64_t num_rows, int64_t num_cols, int32_t dim_origin, int32_t dim_k,
    void *workspace, size_t workspace_bytes, void *stream, void *side_stream, void *ev_fork,
    void *ev_join) {
    clear_error();
    const size_t need = maxk_sspmm_backward_hybrid_workspace_size(num_rows, num_cols, n_off_e,
                                                                  dim_origin, dim_k, n_tiles);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu bytes, got %zu",
                 need, workspace_bytes);
    MAXK_REQUIRE(!side_stream || (ev_fork && ev_join), "a side stream needs ev_fork and ev_join");
    const size_t a = al256(maxk_sspmm_backward_csc_workspace_size(num_rows, num_cols, n_off_e,
                                                                  dim_origin, dim_k, 0));
    char *ws_csc = reinterpret_cast<char *>(workspace);
    char *ws_pull = ws_csc + a;
    const size_t pull_bytes = workspace_bytes - a;
    hipStream_t s = as_stream(stream);
    const bool overlap = side_stream && n_off_e > 0 && n_tiles > 0;
    // entries pre-divided by their rows' row_div (maxk_pull_entries_scale): the tiles gather
    // G itself, only the csc part divides
    const float *tile_div = (flags & MAXK_HYBRID_PRESCALED) ? nullptr : row_div;
    auto tiles = [&](int acc, void *st) {
        return maxk_sspmm_backward_pull_tiles(grad_out, tile_div, cbsr_idx, tile_list, tile_ent,
                                              n_tiles, bucket_ptr, bucket_tiles, ent_pull,
                                              bucket_shift, slices, acc, grad_cbsr, num_rows,
                                              num_cols, n_pull_e, dim_origin, dim_k, ws_pull,
                                              pull_bytes, st);
    };
    if (overlap) {  // the tile kernels on the side stream beside the csc, joined at the reduce
        MAXK_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_fork), s));
        MAXK_HIP(hipStreamWaitEvent(as_stream(side_stream), reinterpret_cast<hipEvent_t>(ev_fork), 0));
        if (int rc = tiles(MAXK_PULL_NO_REDUCE, side_stream)) return rc;
        MAXK_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_join), as_stream(side_stream)));
    }
    if (n_off_e > 0) {
        if (int rc = maxk_sspmm_backward_csc(off_row_ptr, off_col, off_val, grad_out, row_div,
                                             cbsr_idx, off_col_ptr, off_csc_eid, grad_cbsr,
                                             num_rows, num_cols, n_off_e, dim_origin, dim_k, 0,
                                             ws_csc, a, stream))
            return rc;
    } else {
        if (int rc = zero_words(grad_cbsr, num_cols * dim_k, s)) return rc;
    }
    if (overlap) {
        MAXK_HIP(hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(ev_join), 0));
        return tiles(MAXK_PULL_REDUCE_ONLY | 1, stream);
    }
    return tiles(1, stream);
}
