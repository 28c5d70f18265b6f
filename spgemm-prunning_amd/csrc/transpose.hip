// Transpose plan for the atomic-free backward: for the CSR of A, the CSC column
// pointer and, for every CSC slot t, the CSR edge id it holds (stable: edges
// into the same column keep their CSR order).  Built once per graph on the GPU with
// a stable LSD radix sort of (column, edge id) -- the MI355X replacement for
// the CSC side files of generate_meta_csc.py:14-93 / load_warp4_metadata_csc.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.h"

namespace maxk {
namespace {

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

__global__ void iota_kernel(int32_t *__restrict__ a, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}

// col_ptr from the sorted column keys: col_ptr[c] = first slot with key >= c.
__global__ void col_ptr_kernel(const int32_t *__restrict__ sorted_cols, int64_t num_e,
                               int num_cols, int32_t *__restrict__ col_ptr) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > num_e) return;
    int cur = t < num_e ? sorted_cols[t] : num_cols;
    int prev = t == 0 ? -1 : sorted_cols[t - 1];
    cur = cur > num_cols ? num_cols : cur;  // out-of-range columns: never write past col_ptr
    prev = prev > num_cols ? num_cols : prev;
    for (int c = prev + 1; c <= cur; ++c) col_ptr[c] = (int32_t)t;
}

int key_bits(int64_t num_cols) {
    int b = 1;
    while ((1LL << b) < num_cols + 1) ++b;
    return b;
}

size_t sort_temp_bytes(int64_t num_e, int64_t num_cols) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (int)num_e, 0,
                                             key_bits(num_cols));
    return bytes;
}

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" size_t maxk_transpose_plan_workspace_size(int64_t num_cols, int64_t num_e) {
    if (num_cols < 0 || num_e <= 0) return 0;
    return 2 * al256((size_t)num_e * 4) + al256(sort_temp_bytes(num_e, num_cols));
}

extern "C" int maxk_transpose_plan(const int32_t *col_idx, int64_t num_cols, int64_t num_e,
                                   int32_t *col_ptr, int32_t *csc_eid, void *workspace,
                                   size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(col_ptr != nullptr, "col_ptr must not be NULL");
    hipStream_t s = as_stream(stream);
    if (num_e == 0) {
        MAXK_HIP(hipMemsetAsync(col_ptr, 0, (size_t)(num_cols + 1) * 4, s));
        return MAXK_OK;
    }
    MAXK_REQUIRE(col_idx && csc_eid, "col_idx/csc_eid must not be NULL");
    const size_t need = maxk_transpose_plan_workspace_size(num_cols, num_e);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu", need);
    char *ws = reinterpret_cast<char *>(workspace);
    const size_t a = al256((size_t)num_e * 4);
    int32_t *ids = reinterpret_cast<int32_t *>(ws);
    int32_t *keys_out = reinterpret_cast<int32_t *>(ws + a);
    void *tmp = ws + 2 * a;
    size_t tmp_bytes = workspace_bytes - 2 * a;
    const dim3 g((unsigned)ceil_div(num_e, kBlock));
    hipLaunchKernelGGL(iota_kernel, g, dim3(kBlock), 0, s, ids, num_e);
    MAXK_LAUNCHED("iota_kernel");
    MAXK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, col_idx, keys_out, ids, csc_eid,
                                                (int)num_e, 0, key_bits(num_cols), s));
    hipLaunchKernelGGL(col_ptr_kernel, dim3((unsigned)ceil_div(num_e + 1, kBlock)), dim3(kBlock),
                       0, s, keys_out, num_e, (int)num_cols, col_ptr);
    MAXK_LAUNCHED("col_ptr_kernel");
    return MAXK_OK;
}

// ---- bucket plan (phase 2 of the bucketed backward) ------------------------------------
// Destinations are cut into buckets of 2^shift consecutive columns.  bucket_eid lists,
// bucket by bucket, the CSR edge ids whose column lies in the bucket, in CSR order (a
// stable radix sort on the column bits >= shift); bucket_dst holds each entry's column
// inside its bucket.  Neighbouring entries of one source row are neighbouring T rows, so
// the phase-2 reads of a bucket share cache lines.
namespace maxk {
namespace {

__global__ void bucket_ptr_kernel(const int32_t *__restrict__ sorted_cols, int64_t num_e,
                                  int shift, int n_buckets, int32_t *__restrict__ bucket_ptr,
                                  uint16_t *__restrict__ bucket_dst) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > num_e) return;
    const int c = t < num_e ? sorted_cols[t] : 0;
    if (t < num_e) bucket_dst[t] = (uint16_t)(c & ((1 << shift) - 1));
    int cur = t < num_e ? (c >> shift) : n_buckets;
    int prev = t == 0 ? -1 : (sorted_cols[t - 1] >> shift);
    cur = cur > n_buckets ? n_buckets : cur;
    prev = prev > n_buckets ? n_buckets : prev;
    for (int b = prev + 1; b <= cur; ++b) bucket_ptr[b] = (int32_t)t;
}

}  // namespace
}  // namespace maxk

extern "C" int maxk_bucket_shift(int32_t dim_k) {
    if (dim_k <= 0) return -1;
    int s = 0;
    while (((2LL << s) * (dim_k + 1)) <= maxk::kBucketAccDoubles) ++s;
    return s;
}

extern "C" int64_t maxk_bucket_count(int64_t num_cols, int32_t bucket_shift) {
    if (num_cols < 0 || bucket_shift < 0 || bucket_shift > 16) return -1;
    return (num_cols + (1LL << bucket_shift) - 1) >> bucket_shift;
}

// The bucket plan (internal since r06: only the window-sorted bsort plan builds one; the
// "bucket" backward mode it served is gone).
static size_t bucket_plan_workspace_size(int64_t num_cols, int64_t num_e) {
    if (num_cols < 0 || num_e <= 0) return 0;
    return 2 * al256((size_t)num_e * 4) + al256(sort_temp_bytes(num_e, num_cols));
}

static int bucket_plan(const int32_t *col_idx, int64_t num_cols, int64_t num_e,
                       int32_t bucket_shift, int32_t *bucket_ptr, int32_t *bucket_eid,
                       uint16_t *bucket_dst, void *workspace, size_t workspace_bytes,
                       void *stream) {
    clear_error();
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(bucket_shift >= 0 && bucket_shift <= 16, "bucket_shift must be in [0,16]");
    MAXK_REQUIRE(bucket_ptr != nullptr, "bucket_ptr must not be NULL");
    hipStream_t s = as_stream(stream);
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    if (num_e == 0) {
        MAXK_HIP(hipMemsetAsync(bucket_ptr, 0, (size_t)(nb + 1) * 4, s));
        return MAXK_OK;
    }
    MAXK_REQUIRE(col_idx && bucket_eid && bucket_dst, "col_idx/bucket_eid/bucket_dst must not be NULL");
    const size_t need = bucket_plan_workspace_size(num_cols, num_e);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu", need);
    char *ws = reinterpret_cast<char *>(workspace);
    const size_t a = al256((size_t)num_e * 4);
    int32_t *ids = reinterpret_cast<int32_t *>(ws);
    int32_t *keys_out = reinterpret_cast<int32_t *>(ws + a);
    void *tmp = ws + 2 * a;
    size_t tmp_bytes = workspace_bytes - 2 * a;
    hipLaunchKernelGGL(iota_kernel, dim3((unsigned)ceil_div(num_e, kBlock)), dim3(kBlock), 0, s,
                       ids, num_e);
    MAXK_LAUNCHED("iota_kernel");
    const int kb = key_bits(num_cols);
    if (bucket_shift < kb) {
        MAXK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, col_idx, keys_out, ids,
                                                    bucket_eid, (int)num_e, bucket_shift, kb, s));
    } else {  // a single bucket: CSR order as it is
        MAXK_HIP(hipMemcpyAsync(keys_out, col_idx, (size_t)num_e * 4, hipMemcpyDeviceToDevice, s));
        MAXK_HIP(hipMemcpyAsync(bucket_eid, ids, (size_t)num_e * 4, hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL(bucket_ptr_kernel, dim3((unsigned)ceil_div(num_e + 1, kBlock)),
                       dim3(kBlock), 0, s, keys_out, num_e, (int)bucket_shift, (int)nb, bucket_ptr,
                       bucket_dst);
    MAXK_LAUNCHED("bucket_ptr_kernel");
    return MAXK_OK;
}

// ---- window-sorted plan (maxk_sspmm_backward_bsort) ---------------------------------------
// The bucket plan, with each entry's CSR edge id replaced by the T row phase 1 stores that
// edge's contribution in, plus win_src.  Windows are W = maxk_bsort_window(k) consecutive CSR
// edges; a stable radix sort of (window, bucket, edge id) gives every window's edges in
// bucket order, and since windows sort in order, the sorted position p of edge e IS its T
// row: win_src[p] = e - window_start(p), pos[e] = p, bucket_pos[i] = pos[bucket_eid[i]].
namespace maxk {
namespace {

__global__ void bsort_key_kernel(const int32_t *__restrict__ col_idx, int64_t num_e, int W,
                                 int nb, int shift, int32_t *__restrict__ keys,
                                 int32_t *__restrict__ ids) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= num_e) return;
    int b = col_idx[e] >> shift;
    b = b < 0 ? 0 : (b >= nb ? nb - 1 : b);  // out-of-range columns stay inside their window
    keys[e] = (int32_t)((e / W) * nb + b);
    ids[e] = (int32_t)e;
}

__global__ void bsort_pos_kernel(const int32_t *__restrict__ perm, int64_t num_e, int W,
                                 uint16_t *__restrict__ win_src, int32_t *__restrict__ pos) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= num_e) return;
    const int e = perm[p];
    win_src[p] = (uint16_t)(e - p / W * W);
    pos[e] = (int32_t)p;
}

__global__ void bsort_map_kernel(const int32_t *__restrict__ pos, int64_t num_e,
                                 int32_t *__restrict__ bucket_pos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < num_e) bucket_pos[i] = pos[bucket_pos[i]];
}

// Source row of every CSR edge (the COO row array): the last r with row_ptr[r] <= e.
__global__ void bsort_rows_kernel(const int32_t *__restrict__ row_ptr, int num_rows,
                                  int64_t num_e, int32_t *__restrict__ edge_row) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= num_e) return;
    int lo = 0, hi = num_rows - 1;
    while (lo < hi) {
        const int mid = (int)(((int64_t)lo + hi + 1) >> 1);
        if (row_ptr[mid] <= e) lo = mid; else hi = mid - 1;
    }
    edge_row[e] = lo;
}

size_t bsort_sort_bytes(int64_t num_e) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (int)num_e, 0, 31);
    return bytes;
}

}  // namespace
}  // namespace maxk

extern "C" size_t maxk_bsort_plan_workspace_size(int64_t num_cols, int64_t num_e) {
    if (num_cols < 0 || num_e <= 0) return 0;
    const size_t a = al256((size_t)num_e * 4);
    const size_t bucket = bucket_plan_workspace_size(num_cols, num_e);
    const size_t own = 4 * a + al256(bsort_sort_bytes(num_e));
    return own > bucket ? own : bucket;
}

extern "C" int maxk_bsort_plan(const int32_t *row_ptr, const int32_t *col_idx, int64_t num_rows,
                               int64_t num_cols, int64_t num_e, int32_t dim_k,
                               int32_t bucket_shift, int32_t *bucket_ptr, int32_t *bucket_pos,
                               uint16_t *bucket_dst, uint16_t *win_src, int32_t *edge_row,
                               void *workspace, size_t workspace_bytes, void *stream) {
    clear_error();
    const int W = maxk_bsort_window(dim_k);
    MAXK_REQUIRE(W > 0, "window-sorted plan needs dim_k %% 4 == 0 in [4, 256], got %d", dim_k);
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(bucket_shift >= 0 && bucket_shift <= 16, "bucket_shift must be in [0,16]");
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    const int64_t nwin = ceil_div(num_e, W);
    MAXK_REQUIRE(nwin * (nb > 0 ? nb : 1) < (1LL << 31),
                 "%lld windows x %lld buckets exceed the 31-bit sort key", (long long)nwin,
                 (long long)nb);
    // the bucket plan, its edge ids landing in bucket_pos (num_e == 0: bucket_ptr zeroed)
    if (int rc = bucket_plan(col_idx, num_cols, num_e, bucket_shift, bucket_ptr, bucket_pos,
                                  bucket_dst, workspace, workspace_bytes, stream))
        return rc;
    if (num_e == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && win_src && edge_row, "row_ptr/win_src/edge_row must not be NULL");
    MAXK_REQUIRE(num_rows > 0, "edges present but num_rows == 0");
    const size_t need = maxk_bsort_plan_workspace_size(num_cols, num_e);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu", need);
    hipStream_t s = as_stream(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    const size_t a = al256((size_t)num_e * 4);
    int32_t *keys = reinterpret_cast<int32_t *>(ws);
    int32_t *ids = reinterpret_cast<int32_t *>(ws + a);
    int32_t *keys_out = reinterpret_cast<int32_t *>(ws + 2 * a);
    int32_t *perm = reinterpret_cast<int32_t *>(ws + 3 * a);
    void *tmp = ws + 4 * a;
    size_t tmp_bytes = workspace_bytes - 4 * a;
    const dim3 g((unsigned)ceil_div(num_e, kBlock));
    const int nbi = (int)(nb > 0 ? nb : 1);
    hipLaunchKernelGGL(bsort_key_kernel, g, dim3(kBlock), 0, s, col_idx, num_e, W, nbi,
                       (int)bucket_shift, keys, ids);
    MAXK_LAUNCHED("bsort_key_kernel");
    MAXK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_out, ids, perm,
                                                (int)num_e, 0, key_bits(nwin * nbi), s));
    int32_t *pos = keys;  // the keys are consumed by the sort
    hipLaunchKernelGGL(bsort_pos_kernel, g, dim3(kBlock), 0, s, perm, num_e, W, win_src, pos);
    MAXK_LAUNCHED("bsort_pos_kernel");
    hipLaunchKernelGGL(bsort_map_kernel, g, dim3(kBlock), 0, s, pos, num_e, bucket_pos);
    MAXK_LAUNCHED("bsort_map_kernel");
    hipLaunchKernelGGL(bsort_rows_kernel, g, dim3(kBlock), 0, s, row_ptr, (int)num_rows, num_e,
                       edge_row);
    MAXK_LAUNCHED("bsort_rows_kernel");
    return MAXK_OK;
}

// ---- pull plan (the tiled pull backward, maxk_sspmm_backward_pull) -----------------------
// Tiles t = s * n_buckets + j: rows cut into `slices` equal slices s, columns into buckets j
// of 2^shift.  A stable radix sort of (t, edge id) lists every tile's edges in CSR order;
// ent_row / ent_w / ent_dst are their source row, weight and column inside the bucket.
// The weights are copied: a plan built from one `edge_val` serves that array only.
namespace maxk {
namespace {

constexpr int64_t kPullSliceBytes = 7LL << 19;  // 3.5 MiB of G' rows per slice

// one wave per row: key and source row of each of its edges
__global__ void pull_key_kernel(const int32_t *__restrict__ row_ptr,
                                const int32_t *__restrict__ col_idx, int num_rows,
                                int rows_per_slice, int n_buckets, int shift,
                                int32_t *__restrict__ keys, int32_t *__restrict__ row_of) {
    const int r = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave);
    if (r >= num_rows) return;
    const int lane = lane_id();
    const int b = row_ptr[r], e = row_ptr[r + 1];
    const int base = (r / rows_per_slice) * n_buckets;
    for (int i = b + lane; i < e; i += kWave) {
        keys[i] = base + (col_idx[i] >> shift);
        row_of[i] = r;
    }
}

__global__ void pull_gather_kernel(const int32_t *__restrict__ eid,
                                   const int32_t *__restrict__ row_of,
                                   const int32_t *__restrict__ col_idx,
                                   const float *__restrict__ edge_val, int64_t num_e, int shift,
                                   int rows_per_slice, uint2 *__restrict__ ent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= num_e) return;
    const int e = eid[i];
    const int r = row_of[e];
    const uint32_t in_slice = (uint32_t)(r % rows_per_slice);
    const uint32_t dst = (uint32_t)(col_idx[e] & ((1 << shift) - 1));
    ent[i] = make_uint2(in_slice | (dst << 16), __float_as_uint(edge_val[e]));
}

// tile_ptr[t] = first slot with key >= t
__global__ void tile_ptr_kernel(const int32_t *__restrict__ sorted_keys, int64_t num_e,
                                int n_tiles, int32_t *__restrict__ tile_ptr) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > num_e) return;
    int cur = t < num_e ? sorted_keys[t] : n_tiles;
    int prev = t == 0 ? -1 : sorted_keys[t - 1];
    cur = cur > n_tiles ? n_tiles : cur;  // out-of-range columns: never write past tile_ptr
    prev = prev > n_tiles ? n_tiles : prev;
    for (int x = prev + 1; x <= cur; ++x) tile_ptr[x] = (int32_t)t;
}

size_t pull_sort_temp_bytes(int64_t num_e, int64_t n_tiles) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (const int32_t *)nullptr,
                                             (int32_t *)nullptr, (int)num_e, 0,
                                             key_bits(n_tiles));
    return bytes;
}

}  // namespace
}  // namespace maxk

// The widest bucket that up to MAXK_PULL_H parts reach (pull_q_kernel, k % (4H) == 0) while
// a part keeps at least MAXK_PULL_MIN_KP slots (k < 32; MAXK_PULL_MIN_KP_WIDE from k = 32):
// the accumulator holds k/H slots per destination, so H parts give a bucket H times the
// destinations and a source row meets H times fewer buckets, for H reads of the entries.
// Measured (Reddit / proteins, whole backward, profiles/r02/tune/pull_parts_r02.txt):
// k=16 8 slots 2.43 / 1.23 ms against 16 slots 2.52 / 1.29; k=32 16 slots 3.56 / 1.88 against
// 8 slots 3.50 / 2.15; k=64 16 slots 5.71 / 3.25 against 32 slots 6.15 / 3.62 and 8 slots
// 6.15 / 4.07.  A part count that does not widen the bucket is not used.  At least 4: the
// backward copies a bucket's selector rows 16 B at a time (16 | 2^shift * k).
extern "C" int maxk_pull_shift(int32_t dim_k) {
    if (dim_k <= 0) return -1;
    int s = maxk_bucket_shift(dim_k);
    const int kp_min = dim_k >= 32 ? MAXK_PULL_MIN_KP_WIDE : MAXK_PULL_MIN_KP;
    for (int H = 2; MAXK_PULL_Q && H <= MAXK_PULL_H && dim_k % (4 * H) == 0 &&
                    dim_k / H >= kp_min;
         H *= 2) {
        // the widest bucket whose kp-slot rows (unpadded, maxk::pull_ks) and selectors fit
        const int kp = dim_k / H;
        int sh = 0;
        while (sh < 15 && (((size_t)kp * 8 + kp) << (sh + 1)) <= maxk::kPullLdsBytes) ++sh;
        s = std::max(s, sh);
    }
    const int p = s - MAXK_PULL_SHIFT_DELTA;
    return p < 4 ? 4 : (p > 15 ? 15 : p);
}

// Parts per tile the pull backward uses at width k (the largest H of maxk_pull_shift's rule:
// k % (4H) == 0 and k/H slots at least MAXK_PULL_MIN_KP, or _WIDE from k = 32).
static int pull_parts_of(int32_t dim_k) {
    int H = 1;
    const int kp_min = dim_k >= 32 ? MAXK_PULL_MIN_KP_WIDE : MAXK_PULL_MIN_KP;
    while (MAXK_PULL_Q && 2 * H <= MAXK_PULL_H && dim_k % (8 * H) == 0 && dim_k / (2 * H) >= kp_min)
        H *= 2;
    return H;
}


// ~3.5 MiB of G rows per slice and part: a part gathers only its share of a row's columns
// (its rank range of the sorted selectors), so an XCD's L2 holds H times the rows of G for
// it.  The S tile partials (S x num_cols x k floats, written and read once) fall as the
// slices grow.  Reddit (whole backward, profiles/r02/tune/pull_slices_r02.txt): k = 16
// (2 parts) best at S = 30-34 (2.23 ms against 2.42 at S = 66), k = 8 (1 part) flat over
// 40-66, k = 32 (2 parts) at 33.  Past 3 parts the gain stops: k = 64 (4 parts) runs 5.32 ms
// at S = 20-22 against 5.74 at 17 (profiles/r02/tune/pull_slices_k64.txt), so the factor is
// capped at 3 (proteins k = 64 is flat over S = 8-12).
// r03 (profiles/r03/tune/pull_slices.txt, two repeats each): the narrower a part's share of
// a row's columns, the more rows a slice may hold -- k = 8 (one 8-slot part) best at
// S = 44 (5.3 MiB; 1.400 ms against 1.418 at S = 66), k = 16 (two 8-slot parts) at S = 28
// (4.1 MiB per part; 2.120 against 2.145 at S = 33), k = 32 (two 16-slot parts) still at 33.
extern "C" int maxk_pull_slices(int64_t num_rows, int64_t num_cols, int32_t dim_origin,
                                int32_t dim_k) {
    if (num_rows <= 0 || dim_origin <= 0) return 1;
    if (num_cols <= 0) num_cols = num_rows;
    const int parts = dim_k % 4 == 0 ? pull_parts_of(dim_k) : 1;
    const int64_t part_bytes = dim_k <= 8    ? maxk::kPullSliceBytes * 3 / 2
                               : dim_k <= 16 ? maxk::kPullSliceBytes * 33 / 28
                                             : maxk::kPullSliceBytes;
    const int64_t per = part_bytes * (parts < 3 ? parts : 3);
    int64_t s = (num_rows * dim_origin * 4 + per - 1) / per;
    const int64_t lo = (num_rows + 65535) / 65536;  // rows within a slice fit 16 bits
    s = s < lo ? lo : s;
    // A small graph's pull is a few rounds of workgroups, one per CU (a part's slot table
    // fills the LDS), so a nearly empty last round costs a whole round: of the slice counts
    // in [ceil(s/2), s], take the largest with the fewest rounds when s makes at most 5
    // (buckets counted over num_cols, rounds over the device's CUs: ADVICE r04).  Flickr-sized (89k rows, D = 64; 220 / 264 / 704 / 1056
    // workgroups at k = 8 / 16 / 32 / 64): k = 16 S = 3 -> 2, 0.054 -> 0.046 ms; k = 32 4 -> 2,
    // 0.069 -> 0.064; k = 64 3 -> 2, 0.111 -> 0.100; k = 8 keeps 5 (0.037)
    // (profiles/r04/tune/flickr_pull_slices.txt).  Reddit- and proteins-sized graphs make
    // 1.6k-15k workgroups and keep the rule above.
    if (dim_k % 4 == 0 && MAXK_PULL_Q) {
        const int shift = maxk_pull_shift(dim_k);
        const int64_t wg = maxk_bucket_count(num_cols, shift) * parts;  // per slice
        const int64_t cus = device_cus();
        auto rounds = [&](int64_t n) { return (n * wg + cus - 1) / cus; };
        if (shift > 0 && wg > 0 && rounds(s) <= 5) {
            int64_t best = s;
            for (int64_t c = s - 1; c >= (s + 1) / 2 && c >= lo; --c)
                if (rounds(c) < rounds(best)) best = c;
            s = best;
        }
    }
    return (int)(s < 1 ? 1 : (s > 256 ? 256 : s));
}

extern "C" size_t maxk_pull_plan_workspace_size(int64_t num_rows, int64_t num_cols,
                                                int64_t num_e, int32_t bucket_shift,
                                                int32_t slices) {
    if (num_rows < 0 || num_cols < 0 || num_e <= 0 || slices <= 0) return 0;
    const int64_t nt = slices * maxk_bucket_count(num_cols, bucket_shift);
    return 5 * al256((size_t)num_e * 4) + al256(pull_sort_temp_bytes(num_e, nt));
}

extern "C" int maxk_pull_plan(const int32_t *row_ptr, const int32_t *col_idx,
                              const float *edge_val, int64_t num_rows, int64_t num_cols,
                              int64_t num_e, int32_t bucket_shift, int32_t slices,
                              int32_t *tile_ptr, uint32_t *ent, void *workspace,
                              size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_cols >= 0 && num_cols < (1LL << 31), "num_cols out of range");
    MAXK_REQUIRE(num_e >= 0 && num_e < (1LL << 31), "num_e out of range");
    MAXK_REQUIRE(bucket_shift >= 4 && bucket_shift <= 15, "bucket_shift must be in [4,15]");
    const int64_t nb = maxk_bucket_count(num_cols, bucket_shift);
    MAXK_REQUIRE(slices >= 1 && slices * nb < (1LL << 31), "slices %d out of range", slices);
    const int64_t rps64 = (num_rows + slices - 1) / slices;
    MAXK_REQUIRE(rps64 <= 65536, "%d slices leave %lld rows per slice (max 65536)", slices,
                 (long long)rps64);
    MAXK_REQUIRE(tile_ptr != nullptr, "tile_ptr must not be NULL");
    hipStream_t s = as_stream(stream);
    const int64_t nt = slices * nb;
    if (num_e == 0 || num_rows == 0) {
        MAXK_HIP(hipMemsetAsync(tile_ptr, 0, (size_t)(nt + 1) * 4, s));
        return MAXK_OK;
    }
    MAXK_REQUIRE(row_ptr && col_idx && edge_val && ent, "CSR/plan pointers must not be NULL");
    const size_t need = maxk_pull_plan_workspace_size(num_rows, num_cols, num_e, bucket_shift, slices);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu", need);
    char *ws = reinterpret_cast<char *>(workspace);
    const size_t a = al256((size_t)num_e * 4);
    int32_t *keys = reinterpret_cast<int32_t *>(ws);
    int32_t *keys_out = reinterpret_cast<int32_t *>(ws + a);
    int32_t *ids = reinterpret_cast<int32_t *>(ws + 2 * a);
    int32_t *eid = reinterpret_cast<int32_t *>(ws + 3 * a);
    int32_t *row_of = reinterpret_cast<int32_t *>(ws + 4 * a);
    void *tmp = ws + 5 * a;
    size_t tmp_bytes = workspace_bytes - 5 * a;
    const int rps = (int)rps64;
    hipLaunchKernelGGL(pull_key_kernel, dim3((unsigned)ceil_div(num_rows * kWave, kBlock)),
                       dim3(kBlock), 0, s, row_ptr, col_idx, (int)num_rows, rps, (int)nb,
                       (int)bucket_shift, keys, row_of);
    MAXK_LAUNCHED("pull_key_kernel");
    hipLaunchKernelGGL(iota_kernel, dim3((unsigned)ceil_div(num_e, kBlock)), dim3(kBlock), 0, s,
                       ids, num_e);
    MAXK_LAUNCHED("iota_kernel");
    MAXK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_out, ids, eid,
                                                (int)num_e, 0, key_bits(nt), s));
    hipLaunchKernelGGL(pull_gather_kernel, dim3((unsigned)ceil_div(num_e, kBlock)), dim3(kBlock),
                       0, s, eid, row_of, col_idx, edge_val, num_e, (int)bucket_shift, rps,
                       reinterpret_cast<uint2 *>(ent));
    MAXK_LAUNCHED("pull_gather_kernel");
    hipLaunchKernelGGL(tile_ptr_kernel, dim3((unsigned)ceil_div(num_e + 1, kBlock)), dim3(kBlock),
                       0, s, keys_out, num_e, (int)nt, tile_ptr);
    MAXK_LAUNCHED("tile_ptr_kernel");
    return MAXK_OK;
}
