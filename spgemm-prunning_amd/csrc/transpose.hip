// Transpose plan for the atomic-free backward: for the CSR of A, the CSC column
// pointer and, for every CSC slot t, the CSR edge id it holds (stable: edges
// into the same column keep their CSR order).  Built once per graph on the GPU with
// a stable LSD radix sort of (column, edge id) -- the MI355X replacement for
// the CSC side files of generate_meta_csc.py:14-93 / load_warp4_metadata_csc.
#include <hipcub/hipcub.hpp>

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

extern "C" size_t maxk_bucket_plan_workspace_size(int64_t num_cols, int64_t num_e) {
    if (num_cols < 0 || num_e <= 0) return 0;
    return 2 * al256((size_t)num_e * 4) + al256(sort_temp_bytes(num_e, num_cols));
}

extern "C" int maxk_bucket_plan(const int32_t *col_idx, int64_t num_cols, int64_t num_e,
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
    const size_t need = maxk_bucket_plan_workspace_size(num_cols, num_e);
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
