// warp4 schedule on the GPU: builder (drop-in for kernels/generate_meta.py:30-48
// and generate_meta_csc.py:14-93, which are O(V) Python loops) and the inverse
// map warp4 -> CSR row_ptr used when a caller drives the kernels through the
// reference's spmm_maxk_forward(warp4, ...) signature.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace maxk {
namespace {

__global__ void warp4_count_kernel(const int32_t *__restrict__ row_ptr, int num_rows, int nz,
                                   int32_t *__restrict__ counts,
                                   unsigned long long *__restrict__ total) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    int c = 0;
    if (r < num_rows) {
        const int deg = row_ptr[r + 1] - row_ptr[r];
        c = (deg + nz - 1) / nz;
        if (counts) counts[r] = c;
    }
    if (total) {
        // wave reduction, then one atomic per wave
        int s = c;
        for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
        if (lane_id() == 0 && s) atomicAdd(total, (unsigned long long)s);
    }
}

__global__ void warp4_fill_kernel(const int32_t *__restrict__ row_ptr,
                                  const int32_t *__restrict__ offsets, int num_rows, int nz,
                                  int32_t *__restrict__ warp4, int64_t num_entries) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= num_rows) return;
    int loc = row_ptr[r];
    const int end = row_ptr[r + 1];
    int64_t w = offsets[r];
    while (loc < end && w < num_entries) {
        const int len = end - loc < nz ? end - loc : nz;
        reinterpret_cast<int4 *>(warp4)[w] = make_int4(r, loc, len, 0);
        loc += len;
        ++w;
    }
}

// row_ptr from warp4 entries sorted by row: entry i starts row `row` (and every
// empty row after the previous entry's row) at `loc`; the last entry closes all
// remaining rows at loc+len.
__global__ void warp4_to_row_ptr_kernel(const int32_t *__restrict__ warp4, int64_t num_entries,
                                        int num_rows, int32_t *__restrict__ row_ptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= num_entries) return;
    const int4 cur = reinterpret_cast<const int4 *>(warp4)[i];
    const int prev_row = i == 0 ? -1 : reinterpret_cast<const int4 *>(warp4)[i - 1].x;
    if (cur.x != prev_row) {
        const int hi = cur.x < num_rows ? cur.x : num_rows;
        for (int v = prev_row + 1; v <= hi; ++v) row_ptr[v] = cur.y;
    }
    if (i == num_entries - 1) {
        for (int v = cur.x + 1; v <= num_rows; ++v) row_ptr[v] = cur.y + cur.z;
    }
}

size_t cub_scan_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
                                     n);
    return bytes;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace
}  // namespace maxk

using namespace maxk;

extern "C" int maxk_warp4_count(const int32_t *row_ptr, int64_t num_rows, int32_t warp_max_nz,
                                int64_t *num_entries, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_entries != nullptr, "num_entries must not be NULL");
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(warp_max_nz >= 1, "warp_max_nz must be >= 1");
    *num_entries = 0;
    if (num_rows == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr != nullptr, "row_ptr must not be NULL");
    hipStream_t s = as_stream(stream);
    unsigned long long *d_total = nullptr;
    MAXK_HIP(hipMalloc(&d_total, sizeof(unsigned long long)));
    unsigned long long h_total = 0;
    int rc = MAXK_OK;
    if (hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s) != hipSuccess) rc = MAXK_ERR_HIP;
    if (rc == MAXK_OK) {
        hipLaunchKernelGGL(warp4_count_kernel, dim3((unsigned)ceil_div(num_rows, kBlock)),
                           dim3(kBlock), 0, s, row_ptr, (int)num_rows, warp_max_nz, nullptr,
                           d_total);
        if (hipGetLastError() != hipSuccess) rc = MAXK_ERR_HIP;
    }
    if (rc == MAXK_OK &&
        hipMemcpyAsync(&h_total, d_total, sizeof(h_total), hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = MAXK_ERR_HIP;
    if (rc == MAXK_OK && hipStreamSynchronize(s) != hipSuccess) rc = MAXK_ERR_HIP;
    (void)hipFree(d_total);
    if (rc != MAXK_OK) {
        set_error("maxk_warp4_count: HIP failure");
        return rc;
    }
    *num_entries = (int64_t)h_total;
    return MAXK_OK;
}

extern "C" size_t maxk_warp4_build_workspace_size(int64_t num_rows) {
    if (num_rows <= 0) return 0;
    return 2 * align256((size_t)num_rows * sizeof(int32_t)) + align256(cub_scan_bytes((int)num_rows));
}

extern "C" int maxk_warp4_build(const int32_t *row_ptr, int64_t num_rows, int32_t warp_max_nz,
                                int32_t *warp4, int64_t num_entries, void *workspace,
                                size_t workspace_bytes, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(warp_max_nz >= 1, "warp_max_nz must be >= 1");
    MAXK_REQUIRE(num_entries >= 0 && num_entries < (1LL << 31), "num_entries out of range");
    if (num_rows == 0 || num_entries == 0) return MAXK_OK;
    MAXK_REQUIRE(row_ptr && warp4, "row_ptr/warp4 must not be NULL");
    const size_t need = maxk_warp4_build_workspace_size(num_rows);
    MAXK_REQUIRE(workspace && workspace_bytes >= need, "workspace too small: need %zu", need);
    char *ws = reinterpret_cast<char *>(workspace);
    int32_t *counts = reinterpret_cast<int32_t *>(ws);
    int32_t *offsets = reinterpret_cast<int32_t *>(ws + align256((size_t)num_rows * 4));
    void *tmp = ws + 2 * align256((size_t)num_rows * 4);
    size_t tmp_bytes = align256(cub_scan_bytes((int)num_rows));
    hipStream_t s = as_stream(stream);
    const dim3 grid((unsigned)ceil_div(num_rows, kBlock));
    hipLaunchKernelGGL(warp4_count_kernel, grid, dim3(kBlock), 0, s, row_ptr, (int)num_rows,
                       warp_max_nz, counts, nullptr);
    MAXK_LAUNCHED("warp4_count_kernel");
    MAXK_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, offsets, (int)num_rows, s));
    hipLaunchKernelGGL(warp4_fill_kernel, grid, dim3(kBlock), 0, s, row_ptr, offsets,
                       (int)num_rows, warp_max_nz, warp4, num_entries);
    MAXK_LAUNCHED("warp4_fill_kernel");
    return MAXK_OK;
}

extern "C" int maxk_warp4_to_row_ptr(const int32_t *warp4, int64_t num_entries, int64_t num_rows,
                                     int32_t *row_ptr, void *stream) {
    clear_error();
    MAXK_REQUIRE(num_rows >= 0 && num_rows < (1LL << 31), "num_rows out of range");
    MAXK_REQUIRE(num_entries >= 0, "num_entries must be >= 0");
    MAXK_REQUIRE(row_ptr != nullptr, "row_ptr must not be NULL");
    hipStream_t s = as_stream(stream);
    if (num_entries == 0) {
        MAXK_HIP(hipMemsetAsync(row_ptr, 0, (size_t)(num_rows + 1) * sizeof(int32_t), s));
        return MAXK_OK;
    }
    MAXK_REQUIRE(warp4 != nullptr, "warp4 must not be NULL");
    hipLaunchKernelGGL(warp4_to_row_ptr_kernel, dim3((unsigned)ceil_div(num_entries, kBlock)),
                       dim3(kBlock), 0, s, warp4, num_entries, (int)num_rows, row_ptr);
    MAXK_LAUNCHED("warp4_to_row_ptr_kernel");
    return MAXK_OK;
}
