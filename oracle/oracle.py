"""CPU oracle for the MaxK-GNN aggregation hot path -- TEST INFRASTRUCTURE ONLY.

numpy front-end over ``oracle/maxk_oracle.c`` (built by ``oracle/Makefile`` into
``oracle/_build/liboracle.so``).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker or the timed CPU baseline.  The product path
(``spgemm-prunning_amd/``) never imports it.

Every function cites the reference code it restates; the C file holds the
arithmetic.  Pinned against the reference's own Python code by
``tests/golden/*.npz`` (generator: ``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def build() -> str:
    """Compile the oracle (gcc) if needed; returns the .so path."""
    src = os.path.join(_HERE, "maxk_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        L.oracle_spgemm_fwd.argtypes = [_i32p, _i32p, _f32p, _f32p, _u8p, ctypes.c_void_p,
                                        _f32p, _i64, _i32, _i32, _i64, _i64]
        L.oracle_sspmm_bwd.argtypes = [_i32p, _i32p, _f32p, _f32p, ctypes.c_void_p, _u8p,
                                       _f32p, _i64, _i64, _i32, _i32, _i64, _i64]
        L.oracle_sspmm_bwd_pull.argtypes = [_i32p, _i32p, _f32p, _f32p, ctypes.c_void_p, _u8p,
                                            _f32p, _i64, _i32, _i32, _i64, _i64]
        L.oracle_topk.argtypes = [_f32p, _f32p, _u8p, _i64, _i32, _i32]
        L.oracle_transpose.argtypes = [_i32p, _i32p, _f32p, _i64, _i64, _i32p, _i32p, _f32p]
        L.oracle_warp4.argtypes = [_i32p, _i64, _i32, ctypes.c_void_p, _i64]
        L.oracle_warp4.restype = _i64
        L.oracle_scatter_dense.argtypes = [_f32p, _u8p, _f32p, _i64, _i32, _i32]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _opt_f32(a):
    if a is None:
        return None, None
    a = _c(a, np.float32)
    return a, a.ctypes.data_as(ctypes.c_void_p)


def num_threads() -> int:
    return lib().oracle_num_threads()


def set_num_threads(n: int) -> None:
    lib().oracle_set_num_threads(int(n))


def spgemm_fwd(row_ptr, col_idx, val, cbsr_val, cbsr_idx, D, row_div=None, rows=None):
    """Forward SpGEMM, kernels/spmm_maxk.cu:66-105 (+ /in_deg, maxk_spgemm_function.py:85-86).

    Returns fp32 [V, D].  ``rows=(r0, r1)`` computes only that row range (the
    other rows are returned as zeros) -- the bounded CPU-baseline sample.
    """
    row_ptr, col_idx, val = _c(row_ptr, np.int32), _c(col_idx, np.int32), _c(val, np.float32)
    cbsr_val, cbsr_idx = _c(cbsr_val, np.float32), _c(cbsr_idx, np.uint8)
    V = row_ptr.shape[0] - 1
    k = cbsr_val.shape[1] if cbsr_val.ndim == 2 else int(cbsr_val.size // max(V, 1))
    r0, r1 = (0, V) if rows is None else rows
    out = np.zeros((V, D), dtype=np.float32)
    keep, div = _opt_f32(row_div)
    lib().oracle_spgemm_fwd(row_ptr, col_idx, val, cbsr_val, cbsr_idx, div, out, V, D, k, r0, r1)
    del keep
    return out


def sspmm_bwd(row_ptr, col_idx, val, grad, cbsr_idx, row_div=None, rows=None):
    """Backward SSpMM in the reference's push order, kernels/spmm_maxk_backward.cu:52-103
    (G / out_deg first, maxk_spgemm_function.py:154-155).  Returns fp32 [num_cols, k]
    (num_cols = rows of cbsr_idx).  ``rows=(r0, r1)`` pushes only those source rows."""
    row_ptr, col_idx, val = _c(row_ptr, np.int32), _c(col_idx, np.int32), _c(val, np.float32)
    grad, cbsr_idx = _c(grad, np.float32), _c(cbsr_idx, np.uint8)
    R, D = grad.shape
    C, k = cbsr_idx.shape
    assert row_ptr.shape[0] == R + 1
    out = np.zeros((C, k), dtype=np.float32)
    keep, div = _opt_f32(row_div)
    r0, r1 = (0, R) if rows is None else rows
    lib().oracle_sspmm_bwd(row_ptr, col_idx, val, grad, div, cbsr_idx, out, R, C, D, k, r0, r1)
    del keep
    return out


def transpose(row_ptr, col_idx, val, num_cols):
    """CSR of A -> CSR of A^T (t_ptr over columns, t_src = rows, t_val), stable in row order,
    by the C counting sort (oracle_transpose): seconds at ogbn-products size, and independent
    of the GPU-built plans it checks."""
    row_ptr, col_idx, val = _c(row_ptr, np.int32), _c(col_idx, np.int32), _c(val, np.float32)
    R = row_ptr.shape[0] - 1
    E = col_idx.shape[0]
    t_ptr = np.zeros(num_cols + 1, dtype=np.int32)
    t_src = np.zeros(E, dtype=np.int32)
    t_val = np.zeros(E, dtype=np.float32)
    lib().oracle_transpose(row_ptr, col_idx, val, R, num_cols, t_ptr, t_src, t_val)
    return t_ptr, t_src, t_val


def transpose_csr(row_ptr, col_idx, val, V=None):
    """CSR of A -> CSR of A^T (t_ptr over columns, t_src = rows), stable in row order."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    col_idx = np.asarray(col_idx, dtype=np.int64)
    V = row_ptr.shape[0] - 1 if V is None else V
    rows = np.repeat(np.arange(V, dtype=np.int64), np.diff(row_ptr))
    order = np.argsort(col_idx, kind="stable")
    t_ptr = np.zeros(V + 1, dtype=np.int64)
    np.cumsum(np.bincount(col_idx, minlength=V), out=t_ptr[1:])
    return (t_ptr.astype(np.int32), rows[order].astype(np.int32),
            np.asarray(val, dtype=np.float32)[order])


def sspmm_bwd_pull(t_ptr, t_src, t_val, grad, cbsr_idx, row_div=None, cols=None):
    """Backward via the transpose (pull), OpenMP; same sums as :func:`sspmm_bwd`.
    ``cols=(c0, c1)`` computes only those output rows (bounded baseline sample)."""
    t_ptr, t_src, t_val = _c(t_ptr, np.int32), _c(t_src, np.int32), _c(t_val, np.float32)
    grad, cbsr_idx = _c(grad, np.float32), _c(cbsr_idx, np.uint8)
    V, D = grad.shape
    k = cbsr_idx.shape[1]
    c0, c1 = (0, V) if cols is None else cols
    out = np.zeros((V, k), dtype=np.float32)
    keep, div = _opt_f32(row_div)
    lib().oracle_sspmm_bwd_pull(t_ptr, t_src, t_val, grad, div, cbsr_idx, out, V, D, k, c0, c1)
    del keep
    return out


def topk(x, k):
    """CBSR encode = torch.topk(x, k, dim=1) + .to(uint8), maxk_spgemm_function.py:51-57."""
    x = _c(x, np.float32)
    V, D = x.shape
    val = np.zeros((V, k), dtype=np.float32)
    idx = np.zeros((V, k), dtype=np.uint8)
    lib().oracle_topk(x, val, idx, V, D, k)
    return val, idx


def topk_u8_reference(x, k):
    """The reference uint8 top-k's INTENDED per-row convention (kernels/maxk_kernel.cu:23-94,
    behind cuda_topk_maxk, cuda_kernel_bindings.cpp:164-201), restated in numpy; rows of 256
    bytes.  Threshold (:35-63): 8 bisection steps over the row's own bytes, count = #(bytes >
    mid); count < k: high = mid, else low = mid; mid = (low + high) // 2.  Selection (:69-88):
    for each 32-column step (column 32 ext + lane), the bytes > mid go to slot total + (picks of
    lower lanes in the step) while that is < k; then total += lane 31's exclusive prefix
    (:84-86: lane 31 adds its own `loc`, which leaves its own pick out, so the next step's first
    pick overwrites it); stop once total >= k (:70-73).  Slots never written stay 0.

    This is NOT the CUDA kernel as built: there every warp takes its threshold from
    the block's FIRST row (:42 reads cache[laneid * 8 + j], no warp offset) with per-lane counts
    and mids (:44-48 leaves the full sum on lane 0 only), warps 1..15 read that row across a
    __syncwarp only (a data race), unfilled slots are uninitialised shared memory and the
    write-out (:91-94) is right only at k = 32.  topk_u8_reference_as_built models the defined
    part of that behaviour; the product keeps this convention.  Parity with the CUDA kernel is
    unpinned (it cannot run here); the GPU test checks the HIP kernel against this function."""
    x = np.ascontiguousarray(x, dtype=np.uint8)
    V, D = x.shape
    if D != 256:
        raise ValueError("rows of 256 bytes")
    val = np.zeros((V, k), dtype=np.uint8)
    idx = np.zeros((V, k), dtype=np.uint8)
    for r in range(V):
        row = x[r].astype(np.int64)
        low, high, mid = 0, 255, 127
        for _ in range(8):
            if int((row > mid).sum()) < k:
                high = mid
            else:
                low = mid
            mid = (low + high) // 2
        total = 0
        for ext in range(8):
            if total >= k:
                break
            chunk = row[32 * ext:32 * ext + 32]
            choose = chunk > mid
            loc = np.cumsum(choose) - choose
            for lane in range(32):
                if choose[lane] and total + loc[lane] < k:
                    val[r, total + loc[lane]] = chunk[lane]
                    idx[r, total + loc[lane]] = 32 * ext + lane
            total += int(loc[31])
    return val, idx


def topk_u8_reference_as_built(x, k=32):
    """A model of what the reference's uint8 top-k kernel (kernels/maxk_kernel.cu:23-94) computes
    as built, launched as its main() and binding launch it (16 warps of 32 lanes per block, one
    row per warp, dim_origin = 256), where that is defined: k = 32 (the block write-out at
    :91-94 copies 16 rows x 32 bytes) and N % 16 == 0 (a partial last block reads past the
    input).  Returns (val, idx, written): slots the kernel never writes hold uninitialised
    shared memory there; here they are 0 and `written` is False.

    Threshold (:35-63), per BLOCK and per LANE: lane l of every warp counts bytes 8l..8l+7 of
    the block's first row (:42, no warp offset; warps 1..15 read it after a __syncwarp only --
    modelled as if warp 0's load (:32) has landed, the one outcome that reads defined data)
    against its own mid; the shfl_down chain (:44-48) gives lane l c[l] + c[l + d], or 2 c[l]
    where l + d >= 32 (an out-of-range source returns the caller's own value), so only lane 0
    holds the full count; each lane bisects its own low / high / mid from its own sum.
    Selection (:69-88): column 32 ext + l of warp w's own row is picked when it exceeds lane
    l's mid; compaction as in topk_u8_reference (lane 31's exclusive-prefix count)."""
    x = np.ascontiguousarray(x, dtype=np.uint8)
    N, D = x.shape
    if D != 256 or k != 32 or N % 16:
        raise ValueError("the as-built kernel is defined for [16 n, 256] rows and k = 32")
    B = N // 16
    row0 = x.reshape(B, 16, 256)[:, 0, :].astype(np.int64).reshape(B, 32, 8)
    low = np.zeros((B, 32), np.int64)
    high = np.full((B, 32), 255, np.int64)
    mid = np.full((B, 32), 127, np.int64)
    for _ in range(8):
        c = (row0 > mid[:, :, None]).sum(-1)
        for d in (16, 8, 4, 2, 1):  # count += __shfl_down_sync(count, d), all lanes at once
            c = c + np.concatenate([c[:, d:], c[:, 32 - d:]], axis=1)
        less = c < k
        high = np.where(less, mid, high)
        low = np.where(less, low, mid)
        mid = (low + high) // 2
    val = np.zeros((N, k), np.uint8)
    idx = np.zeros((N, k), np.uint8)
    written = np.zeros((N, k), bool)
    for r in range(N):
        m = mid[r // 16]
        row = x[r].astype(np.int64)
        total = 0
        for ext in range(8):
            if total >= k:
                break
            chunk = row[32 * ext:32 * ext + 32]
            choose = chunk > m
            loc = np.cumsum(choose) - choose
            for lane in np.nonzero(choose & (total + loc < k))[0]:
                s = total + loc[lane]
                val[r, s], idx[r, s], written[r, s] = chunk[lane], 32 * ext + lane, True
            total += int(loc[31])
    return val, idx, written


def warp4(row_ptr, warp_max_nz=64):
    """warp4 schedule, kernels/generate_meta.py:30-48.  Returns int32 [W*4] (flat, as on disk)."""
    row_ptr = _c(row_ptr, np.int32)
    V = row_ptr.shape[0] - 1
    W = lib().oracle_warp4(row_ptr, V, warp_max_nz, None, 0)
    out = np.zeros(4 * W, dtype=np.int32)
    lib().oracle_warp4(row_ptr, V, warp_max_nz, out.ctypes.data_as(ctypes.c_void_p), W)
    return out


def scatter_dense(grad_cbsr, cbsr_idx, D):
    """zeros(V,D).scatter_(1, sel, grad_cbsr), maxk_spgemm_function.py:152,175."""
    grad_cbsr, cbsr_idx = _c(grad_cbsr, np.float32), _c(cbsr_idx, np.uint8)
    V, k = grad_cbsr.shape
    out = np.zeros((V, D), dtype=np.float32)
    lib().oracle_scatter_dense(grad_cbsr, cbsr_idx, out, V, D, k)
    return out
