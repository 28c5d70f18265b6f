// Dense SpMM baseline on rocSPARSE: Y = A . X, CSR fp32 x row-major fp32.
// The MI355X counterpart of the reference's cuSPARSE denominator
// (kernels/spmm_cusparse.cu:6-62: cusparseSpMM, CSR, row-major, alpha=1,
// beta=0) -- used only by the benchmark/validation helpers, never by the
// MaxK path itself.
#include <rocsparse/rocsparse.h>

#include "common.h"

struct maxk_dense_spmm_plan {
    rocsparse_handle handle = nullptr;
    rocsparse_spmat_descr A = nullptr;
    rocsparse_dnmat_descr X = nullptr;
    rocsparse_dnmat_descr Y = nullptr;
    rocsparse_spmm_alg alg = rocsparse_spmm_alg_default;
    void *buffer = nullptr;
    size_t buffer_size = 0;
};

namespace {

const rocsparse_spmm_alg kAlgs[] = {rocsparse_spmm_alg_default, rocsparse_spmm_alg_csr,
                                    rocsparse_spmm_alg_csr_row_split,
                                    rocsparse_spmm_alg_csr_merge_path,
                                    rocsparse_spmm_alg_csr_nnz_split};

void destroy(maxk_dense_spmm_plan *p) {
    if (!p) return;
    if (p->A) rocsparse_destroy_spmat_descr(p->A);
    if (p->X) rocsparse_destroy_dnmat_descr(p->X);
    if (p->Y) rocsparse_destroy_dnmat_descr(p->Y);
    if (p->handle) rocsparse_destroy_handle(p->handle);
    if (p->buffer) (void)hipFree(p->buffer);
    delete p;
}

int spmm_stage(maxk_dense_spmm_plan *p, rocsparse_spmm_stage stage, size_t *bytes, void *buf) {
    const float one = 1.f, zero = 0.f;
    const rocsparse_status st =
        rocsparse_spmm(p->handle, rocsparse_operation_none, rocsparse_operation_none, &one, p->A,
                       p->X, &zero, p->Y, rocsparse_datatype_f32_r, p->alg, stage, bytes, buf);
    if (st != rocsparse_status_success) {
        maxk::set_error("rocsparse_spmm (stage %d) failed: status %d", (int)stage, (int)st);
        return MAXK_ERR_LIBRARY;
    }
    return MAXK_OK;
}

}  // namespace

#define MAXK_SPARSE(call)                                                         \
    do {                                                                          \
        rocsparse_status st_ = (call);                                            \
        if (st_ != rocsparse_status_success) {                                    \
            maxk::set_error("%s failed: status %d", #call, (int)st_);             \
            destroy(p);                                                           \
            return MAXK_ERR_LIBRARY;                                              \
        }                                                                         \
    } while (0)

extern "C" int maxk_dense_spmm_plan_create(maxk_dense_spmm_plan **plan, const int32_t *row_ptr,
                                           const int32_t *col_idx, const float *edge_val,
                                           const float *x, float *y, int64_t num_rows,
                                           int64_t num_cols, int64_t num_e, int32_t dim,
                                           int32_t alg, void *stream) {
    maxk::clear_error();
    MAXK_REQUIRE(plan != nullptr, "plan must not be NULL");
    *plan = nullptr;
    MAXK_REQUIRE(num_rows > 0 && num_cols > 0 && num_e >= 0 && dim > 0, "bad shape");
    MAXK_REQUIRE(row_ptr && x && y && (num_e == 0 || (col_idx && edge_val)), "NULL pointer");
    MAXK_REQUIRE(alg >= 0 && alg < (int)(sizeof(kAlgs) / sizeof(kAlgs[0])), "bad alg %d", alg);
    auto *p = new maxk_dense_spmm_plan();
    p->alg = kAlgs[alg];
    MAXK_SPARSE(rocsparse_create_handle(&p->handle));
    MAXK_SPARSE(rocsparse_set_stream(p->handle, maxk::as_stream(stream)));
    MAXK_SPARSE(rocsparse_create_csr_descr(
        &p->A, num_rows, num_cols, num_e, const_cast<int32_t *>(row_ptr),
        const_cast<int32_t *>(col_idx), const_cast<float *>(edge_val), rocsparse_indextype_i32,
        rocsparse_indextype_i32, rocsparse_index_base_zero, rocsparse_datatype_f32_r));
    MAXK_SPARSE(rocsparse_create_dnmat_descr(&p->X, num_cols, dim, dim, const_cast<float *>(x),
                                             rocsparse_datatype_f32_r, rocsparse_order_row));
    MAXK_SPARSE(rocsparse_create_dnmat_descr(&p->Y, num_rows, dim, dim, y,
                                             rocsparse_datatype_f32_r, rocsparse_order_row));
    int rc = spmm_stage(p, rocsparse_spmm_stage_buffer_size, &p->buffer_size, nullptr);
    if (rc == MAXK_OK && p->buffer_size > 0 && hipMalloc(&p->buffer, p->buffer_size) != hipSuccess) {
        maxk::set_error("hipMalloc(%zu) for rocSPARSE buffer failed", p->buffer_size);
        rc = MAXK_ERR_HIP;
    }
    if (rc == MAXK_OK) rc = spmm_stage(p, rocsparse_spmm_stage_preprocess, &p->buffer_size, p->buffer);
    if (rc == MAXK_OK && hipStreamSynchronize(maxk::as_stream(stream)) != hipSuccess) {
        maxk::set_error("hipStreamSynchronize failed");
        rc = MAXK_ERR_HIP;
    }
    if (rc != MAXK_OK) {
        destroy(p);
        return rc;
    }
    *plan = p;
    return MAXK_OK;
}

extern "C" int maxk_dense_spmm_run(maxk_dense_spmm_plan *plan, void *stream) {
    maxk::clear_error();
    MAXK_REQUIRE(plan != nullptr, "plan must not be NULL");
    if (rocsparse_set_stream(plan->handle, maxk::as_stream(stream)) != rocsparse_status_success) {
        maxk::set_error("rocsparse_set_stream failed");
        return MAXK_ERR_LIBRARY;
    }
    return spmm_stage(plan, rocsparse_spmm_stage_compute, &plan->buffer_size, plan->buffer);
}

extern "C" int maxk_dense_spmm_bind(maxk_dense_spmm_plan *plan, const float *x, float *y) {
    maxk::clear_error();
    MAXK_REQUIRE(plan != nullptr && x != nullptr && y != nullptr, "NULL plan / x / y");
    if (rocsparse_dnmat_set_values(plan->X, const_cast<float *>(x)) != rocsparse_status_success ||
        rocsparse_dnmat_set_values(plan->Y, y) != rocsparse_status_success) {
        maxk::set_error("rocsparse_dnmat_set_values failed");
        return MAXK_ERR_LIBRARY;
    }
    return MAXK_OK;
}

extern "C" int maxk_dense_spmm_plan_destroy(maxk_dense_spmm_plan *plan) {
    destroy(plan);
    return MAXK_OK;
}
