"""maxk_cuda_kernels -- MI355X-native drop-in for the reference extension of the same name.

Same function names, argument names, defaults and return shapes as the
reference's pybind11 module (cuda_kernel_bindings.cpp:429-490, plus the v2
additions load_warp4_metadata_csc / validate_spmm_maxk_backward,
binding_v2.py:320-351,464-486).  Every compute call goes to hand-written HIP
kernels for gfx950 in libmaxk_hip.so through its C ABI (include/maxk_hip.h);
there is no CPU or PyTorch fallback.

Differences from the reference, all deliberate (DESIGN.md "Boundary"):
  * launches go on torch's *current* HIP stream, not the legacy default stream;
  * `dim_origin` (the dense width D) is a keyword argument defaulting to the
    reference's hard-coded 256 (cuda_kernel_bindings.cpp:70) instead of a constant;
  * the kernels consume the CSR row_ptr; `spmm_maxk_forward/backward` accept the
    reference's warp4 metadata and derive row_ptr from it on the GPU (or take
    `indptr=` directly);
  * results are exact for every k in [1, D] (the reference drops rows / reads
    stale shared memory for k < 32);
  * cuda_topk_maxk_float is an exact top-k (the reference quantises to uint8).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import warnings
import weakref
from typing import List, Optional, Tuple

import torch

from . import _capi

_capi.load()  # ImportError here <=> extension missing (callers test this, like the reference)

__all__ = [
    "spmm_maxk_forward", "spmm_maxk_backward", "cuda_topk_maxk", "cuda_topk_maxk_float",
    "topk_u8_reference",
    "records_ok",
    "cbsr_records",
    "spgemm_forward_records",
    "prepare_cbsr_format_maxk", "cusparse_spmm", "load_warp4_metadata",
    "load_warp4_metadata_csc", "generate_sparse_selector", "benchmark_spmm_maxk",
    "validate_spmm_maxk", "validate_spmm_maxk_backward", "CudaTimer",
    # MI355X additions
    "topk_cbsr", "cbsr_scatter_dense", "topk_cbsr_dense", "topk_backward", "topk_error_rows",
    "build_warp4_metadata", "warp4_to_indptr",
    "spgemm_forward", "sspmm_backward", "DenseSpMMPlan", "version", "device_count",
    "transpose_plan", "bsort_plan", "pull_plan", "edge_selector_mode", "backward_plan", "BWD_MODES",
]

FULL_DIM = 256  # the reference binding's fixed output width (cuda_kernel_bindings.cpp:70)


def _lib():
    return _capi.load()


def version() -> int:
    return _lib().maxk_version()


def device_count() -> int:
    return _lib().maxk_device_count()


def _validate_mode() -> str:
    """MAXK_VALIDATE: unset -> check each graph once (cached per tensor, like the transpose
    plan); "1" -> check every call (graph and selectors); "0" -> never check."""
    v = os.environ.get("MAXK_VALIDATE", "")
    return "once" if v == "" else ("never" if v == "0" else "always")


def _validate_default() -> bool:
    return _validate_mode() == "always"


_CHECKED: "dict" = {}


def _ver(t):
    """Version counter of a cached-on tensor.  Inference tensors have none (reading it raises):
    they get a fresh token, so a cache entry on one never hits and the plan or check is redone
    per call, which is always correct."""
    return object() if t.is_inference() else t._version


def _check_graph_once(row_ptr, col_idx, num_cols):
    """Out-of-range row_ptr / col_idx are the only inputs that can make a kernel read out of
    bounds, so each graph is validated the first time it is used; the check is cached on the
    tensors' identity and versions.  Selectors change every call and are not checked here:
    a selector >= D contributes nothing in every kernel (the forward sends it to a trash
    column, the two-phase and atomic backwards read a zeroed LDS slot, the pull backward
    gathers 0 for it), so it cannot read outside G or another row of it."""
    key = (id(row_ptr), id(col_idx))
    hit = _CHECKED.get(key)
    if hit is not None:
        rr, cr, rv, cv, nc = hit
        if rr() is row_ptr and cr() is col_idx and rv == _ver(row_ptr) and \
                cv == _ver(col_idx) and nc == num_cols:
            return
    _validate_graph(row_ptr, col_idx, num_cols, col_idx.numel())
    if key not in _CHECKED:
        weakref.finalize(col_idx, _CHECKED.pop, key, None)
    _CHECKED[key] = (weakref.ref(row_ptr), weakref.ref(col_idx), _ver(row_ptr),
                     _ver(col_idx), int(num_cols))


def _validate_call(validate, row_ptr, col_idx, num_cols, sel, D):
    if torch.cuda.is_current_stream_capturing():
        return  # a range check synchronises the host: impossible inside a hipGraph capture
    if validate if validate is not None else _validate_default():
        _validate_graph(row_ptr, col_idx, num_cols, col_idx.numel())
        _validate_selector(sel, D)
    elif validate is None and _validate_mode() == "once":
        _check_graph_once(row_ptr, col_idx, num_cols)


def _ptr(t: Optional[torch.Tensor]):
    # a plain int: ctypes converts it for the c_void_p argument (no c_void_p object per call)
    return t.data_ptr() if t is not None and t.numel() > 0 else None


def _need(t, name, dtype=None):
    if not isinstance(t, torch.Tensor):
        raise RuntimeError(f"{name} must be a tensor")
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be CUDA tensor")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"{name} must be {str(dtype).replace('torch.', '')}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _stream(dev):
    """torch's current HIP stream on `dev` as a raw pointer (int).  The raw accessor skips the
    torch.cuda.Stream object torch.cuda.current_stream() builds per call (~3 us of the ~20 us
    a small graph's call spent on the host, tools/host_profile.py)."""
    return torch._C._cuda_getCurrentRawStream(
        dev.index if dev.index is not None else torch.cuda.current_device())


_NO_SWITCH = contextlib.nullcontext()


def _on(dev):
    """torch.cuda.device(dev), or nothing when dev is already the current device (the
    context manager costs ~2.6 us per call)."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    return _NO_SWITCH if idx == torch.cuda.current_device() else torch.cuda.device(dev)


def _validate_graph(row_ptr, col_idx, num_cols, num_e):
    if row_ptr.numel() == 0:
        raise RuntimeError("row_ptr must have num_rows+1 entries")
    if int(row_ptr[0]) != 0 or int(row_ptr[-1]) != num_e:
        raise RuntimeError(f"row_ptr must start at 0 and end at num_e={num_e}")
    if row_ptr.numel() > 1 and bool((row_ptr[1:] < row_ptr[:-1]).any()):
        raise RuntimeError("row_ptr must be non-decreasing")
    if num_e and (int(col_idx.min()) < 0 or int(col_idx.max()) >= num_cols):
        raise RuntimeError(f"col_idx out of range [0, {num_cols})")


def _validate_selector(sel, D):
    if sel.numel() and int(sel.max()) >= D:
        raise RuntimeError(f"sparse_selector entries must be < dim_origin={D}")


# --------------------------------------------------------------------------- schedule
def warp4_to_indptr(warp4_metadata: torch.Tensor, num_v: int,
                    num_warps: Optional[int] = None) -> torch.Tensor:
    """CSR row_ptr [num_v+1] described by a warp4 array (first `num_warps` entries)."""
    _need(warp4_metadata, "warp4_metadata", torch.int32)
    W = warp4_metadata.numel() // 4 if num_warps is None else min(int(num_warps),
                                                                   warp4_metadata.numel() // 4)
    row_ptr = torch.empty(num_v + 1, dtype=torch.int32, device=warp4_metadata.device)
    with torch.cuda.device(warp4_metadata.device):
        _capi.check(_lib().maxk_warp4_to_row_ptr(_ptr(warp4_metadata), W, num_v, _ptr(row_ptr),
                                                 _stream(warp4_metadata.device)),
                    "maxk_warp4_to_row_ptr")
    return row_ptr


def build_warp4_metadata(indptr: torch.Tensor, warp_max_nz: int = 64) -> torch.Tensor:
    """warp4 schedule built on the GPU (kernels/generate_meta.py:30-48 semantics).
    Returns flat int32 [4W] on the device of `indptr` -- the layout of a .warp4 file."""
    _need(indptr, "indptr", torch.int32)
    dev = indptr.device
    V = indptr.numel() - 1
    with _on(dev):
        s = _stream(dev)
        n = ctypes.c_int64(0)
        _capi.check(_lib().maxk_warp4_count(_ptr(indptr), V, warp_max_nz, ctypes.byref(n), s),
                    "maxk_warp4_count")
        out = torch.empty(4 * n.value, dtype=torch.int32, device=dev)
        ws = torch.empty(max(1, _lib().maxk_warp4_build_workspace_size(V)), dtype=torch.uint8,
                         device=dev)
        _capi.check(_lib().maxk_warp4_build(_ptr(indptr), V, warp_max_nz, _ptr(out), n.value,
                                            _ptr(ws), ws.numel(), s), "maxk_warp4_build")
    return out


def _read_warp4_file(path: str, device="cuda") -> torch.Tensor:
    if not os.path.exists(path):
        raise RuntimeError(f"Cannot open warp4 file: {path}")
    import numpy as np
    data = np.fromfile(path, dtype=np.int32)
    return torch.from_numpy(data).to(device)


def load_warp4_metadata(graph_name: str, num_warps: int = 12, warp_max_nz: int = 64) -> torch.Tensor:
    """Read kernels/w{num_warps}_nz{warp_max_nz}_warp_4/<graph>.warp4 (CWD-relative) into
    an int32 CUDA tensor -- cuda_kernel_bindings.cpp:287-317."""
    path = f"kernels/w{num_warps}_nz{warp_max_nz}_warp_4/{graph_name}.warp4"
    return _read_warp4_file(path)


def load_warp4_metadata_csc(graph_name: str, num_warps: int = 12,
                            warp_max_nz: int = 64) -> torch.Tensor:
    """CSC twin, binding_v2.py:320-351 (kernels/w12_nz64_warp_4_csc/<graph>.warp4_csc)."""
    path = f"kernels/w{num_warps}_nz{warp_max_nz}_warp_4_csc/{graph_name}.warp4_csc"
    return _read_warp4_file(path)


# --------------------------------------------------------------------------- hot path
def spgemm_forward(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                   cbsr_val: torch.Tensor, cbsr_idx: torch.Tensor, dim_origin: int,
                   row_div: Optional[torch.Tensor] = None, chunk: int = 0,
                   out: Optional[torch.Tensor] = None, validate: Optional[bool] = None,
                   accumulate: bool = False, edge_sel_out: Optional[torch.Tensor] = None
                   ) -> torch.Tensor:
    """out[num_rows, D] = diag(1/row_div) . A . scatter(cbsr)  (CSR A: indptr/indices/values).
    accumulate: out += the product instead (out= required; maxk_spgemm_forward_accumulate).
    edge_sel_out (uint8 [E, k]): also store each edge's selectors, cbsr_idx[indices[e]], for
    sspmm_backward(..., edge_sel=) (maxk_spgemm_forward_sel; with accumulate,
    maxk_spgemm_forward_accumulate_sel)."""
    for t, n, dt in ((indptr, "indptr", torch.int32), (indices, "indices", torch.int32),
                     (values, "values", torch.float32), (cbsr_val, "input_data", torch.float32),
                     (cbsr_idx, "sparse_selector", torch.uint8)):
        _need(t, n, dt)
    num_rows = indptr.numel() - 1
    num_cols, k = (cbsr_val.shape[0], cbsr_val.shape[1]) if cbsr_val.dim() == 2 else (0, 0)
    if cbsr_idx.shape != cbsr_val.shape:
        raise RuntimeError("input_data and sparse_selector must have the same [V, k] shape")
    if values.numel() != indices.numel():
        raise RuntimeError("values and indices must have the same length")
    D = int(dim_origin)
    if row_div is not None:
        _need(row_div, "row_div", torch.float32)
        if row_div.numel() != num_rows:
            raise RuntimeError("row_div must have num_rows entries")
    _validate_call(validate, indptr, indices, num_cols, cbsr_idx, D)
    dev = cbsr_val.device
    if out is None:
        if accumulate:
            raise RuntimeError("accumulate=True needs out=")
        out = torch.empty(num_rows, D, dtype=torch.float32, device=dev)
    else:
        _need(out, "out", torch.float32)
        if tuple(out.shape) != (num_rows, D):
            raise RuntimeError("out must be [num_rows, dim_origin]")
    L = _lib()
    E = indices.numel()
    ws_bytes = L.maxk_spgemm_forward_workspace_size(num_rows, num_cols, E, D, k, chunk)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if edge_sel_out is not None:
        _need(edge_sel_out, "edge_sel_out", torch.uint8)
        if tuple(edge_sel_out.shape) != (E, k):
            raise RuntimeError("edge_sel_out must be [num_e, k]")
        fn = L.maxk_spgemm_forward_accumulate_sel if accumulate else L.maxk_spgemm_forward_sel
        with _on(dev):
            _capi.check(fn(
                _ptr(indptr), _ptr(indices), _ptr(values), _ptr(cbsr_val), _ptr(cbsr_idx),
                _ptr(row_div), _ptr(out), num_rows, num_cols, E, D, k, chunk, _ptr(ws),
                ws.numel(), _stream(dev), _ptr(edge_sel_out)),
                "maxk_spgemm_forward_accumulate_sel" if accumulate else "maxk_spgemm_forward_sel")
        return out
    fn = L.maxk_spgemm_forward_accumulate if accumulate else L.maxk_spgemm_forward
    with _on(dev):
        _capi.check(fn(
            _ptr(indptr), _ptr(indices), _ptr(values), _ptr(cbsr_val), _ptr(cbsr_idx),
            _ptr(row_div), _ptr(out), num_rows, num_cols, E, D, k, chunk, _ptr(ws), ws.numel(),
            _stream(dev)), "maxk_spgemm_forward_accumulate" if accumulate else "maxk_spgemm_forward")
    return out


def records_ok(num_rows: int, num_cols: int, num_e: int, dim_origin: int, k: int) -> bool:
    """Whether the forward over transport records applies (maxk_records_ok)."""
    return bool(_lib().maxk_records_ok(int(num_rows), int(num_cols), int(num_e), int(dim_origin),
                                       int(k)))


def cbsr_records(cbsr_val: torch.Tensor, cbsr_idx: torch.Tensor, dim_origin: int,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Transport records [V, 5k] uint8 of a CBSR ([k f32 | k u8] per vertex; maxk_cbsr_records):
    what a shard owner all-gathers so the receivers' forward needs no record pack."""
    _need(cbsr_val, "cbsr_val", torch.float32)
    _need(cbsr_idx, "cbsr_idx", torch.uint8)
    if cbsr_val.dim() != 2 or cbsr_idx.shape != cbsr_val.shape:
        raise RuntimeError("cbsr_val / cbsr_idx must be the same [V, k] shape")
    V, k = cbsr_val.shape
    if out is None:
        out = torch.empty(V, 5 * k, dtype=torch.uint8, device=cbsr_val.device)
    elif out.dtype != torch.uint8 or tuple(out.shape) != (V, 5 * k) or not out.is_contiguous():
        raise RuntimeError("out must be a contiguous uint8 [V, 5k] tensor")
    with _on(cbsr_val.device):
        _capi.check(_lib().maxk_cbsr_records(_ptr(cbsr_val), _ptr(cbsr_idx), _ptr(out), V,
                                             int(dim_origin), k, _stream(cbsr_val.device)),
                    "maxk_cbsr_records")
    return out


def spgemm_forward_records(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                           rec: torch.Tensor, k: int, dim_origin: int,
                           row_div: Optional[torch.Tensor] = None, chunk: int = 0,
                           out: Optional[torch.Tensor] = None,
                           accumulate: bool = False,
                           validate: Optional[bool] = None) -> torch.Tensor:
    """spgemm_forward over transport records (cbsr_records of every column, e.g. all-gathered
    by a sharded forward): the same sums, no record pack.  The same input checks as
    spgemm_forward: dtypes, contiguity, shapes of out / row_div / values, and the
    graph's range check (once per graph by default, every call with validate=True)."""
    _need(indptr, "indptr", torch.int32)
    _need(indices, "indices", torch.int32)
    _need(values, "values", torch.float32)
    _need(rec, "rec", torch.uint8)
    k = int(k)
    if k <= 0 or rec.dim() != 2 or rec.shape[1] != 5 * k:
        raise RuntimeError("rec must be [num_cols, 5k]")
    if values.numel() != indices.numel():
        raise RuntimeError("values and indices must have the same length")
    num_rows, num_cols, E, D = indptr.numel() - 1, rec.shape[0], indices.numel(), int(dim_origin)
    dev = rec.device
    if row_div is not None:
        _need(row_div, "row_div", torch.float32)
        if row_div.numel() != num_rows:
            raise RuntimeError("row_div must have num_rows entries")
    # the selectors are the records' last k bytes: a strided view, read only by the selector
    # range check (validate=True); the graph check is what bounds the kernel's record reads
    _validate_call(validate, indptr, indices, num_cols, rec[:, 4 * k:], D)
    if out is None:
        if accumulate:
            raise RuntimeError("accumulate=True needs out=")
        out = torch.empty(num_rows, D, dtype=torch.float32, device=dev)
    else:
        _need(out, "out", torch.float32)
        if tuple(out.shape) != (num_rows, D):
            raise RuntimeError("out must be [num_rows, dim_origin]")
    L = _lib()
    ws_bytes = L.maxk_spgemm_forward_workspace_size(num_rows, num_cols, E, D, k, chunk)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    with _on(dev):
        _capi.check(L.maxk_spgemm_forward_records(
            _ptr(indptr), _ptr(indices), _ptr(values), _ptr(rec), _ptr(row_div), _ptr(out),
            num_rows, num_cols, E, D, k, chunk, _ptr(ws), ws.numel(), _stream(dev),
            1 if accumulate else 0), "maxk_spgemm_forward_records")
    return out


_PLAN_CACHE: "dict" = {}


def transpose_plan(indices: torch.Tensor, num_cols: int, cache: bool = True):
    """(col_ptr int32 [num_cols+1], csc_eid int32 [E]) of the CSR column indices: the CSC
    pointer and, per CSC slot, the CSR edge id it holds.  Built once per graph on the GPU
    (stable radix sort); cached per `indices` tensor object (and its version counter)."""
    _need(indices, "indices", torch.int32)
    key = id(indices)
    hit = _PLAN_CACHE.get(key)
    if cache and hit is not None:
        ref, nc, ver, plan = hit
        if ref() is indices and nc == num_cols and ver == _ver(indices):
            return plan
    dev = indices.device
    E = indices.numel()
    col_ptr = torch.empty(num_cols + 1, dtype=torch.int32, device=dev)
    csc_eid = torch.empty(max(E, 1), dtype=torch.int32, device=dev)[:E]
    L = _lib()
    ws = torch.empty(max(1, L.maxk_transpose_plan_workspace_size(num_cols, E)), dtype=torch.uint8,
                     device=dev)
    with _on(dev):
        _capi.check(L.maxk_transpose_plan(_ptr(indices), num_cols, E, _ptr(col_ptr),
                                          _ptr(csc_eid), _ptr(ws), ws.numel(), _stream(dev)),
                    "maxk_transpose_plan")
    plan = (col_ptr, csc_eid)
    if cache:
        if key not in _PLAN_CACHE:
            weakref.finalize(indices, _PLAN_CACHE.pop, key, None)
        _PLAN_CACHE[key] = (weakref.ref(indices), int(num_cols), _ver(indices), plan)
    return plan


_DENSE_CACHE: "dict" = {}


def dense_plan(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, num_cols: int,
               cache: bool = True):
    """(col_ptr int32 [num_cols+1], t_src int32 [E], t_w float [E]) of the dense backward: the
    graph's transpose (transpose_plan) with, per CSC slot, the CSR row of its edge and its
    weight (maxk_dense_plan).  Cached per (indptr, indices, values) tensor objects and their
    version counters."""
    for t, n, dt in ((indptr, "indptr", torch.int32), (indices, "indices", torch.int32),
                     (values, "values", torch.float32)):
        _need(t, n, dt)
    key = (id(indptr), id(indices), id(values))
    hit = _DENSE_CACHE.get(key)
    if cache and hit is not None:
        rp, ri, rv, nc, pv, vi, vv, plan = hit
        if (rp() is indptr and ri() is indices and rv() is values and nc == num_cols
                and pv == _ver(indptr) and vi == _ver(indices) and vv == _ver(values)):
            return plan
    col_ptr, csc_eid = transpose_plan(indices, num_cols, cache=False)
    dev = indices.device
    E = indices.numel()
    t_src = torch.empty(max(E, 1), dtype=torch.int32, device=dev)[:E]
    t_w = torch.empty(max(E, 1), dtype=torch.float32, device=dev)[:E]
    with _on(dev):
        _capi.check(_lib().maxk_dense_plan(_ptr(indptr), _ptr(values), _ptr(csc_eid),
                                           indptr.numel() - 1, E, _ptr(t_src), _ptr(t_w),
                                           _stream(dev)), "maxk_dense_plan")
    plan = (col_ptr, t_src, t_w)
    if cache:
        if key not in _DENSE_CACHE:
            for t in (indptr, indices, values):
                weakref.finalize(t, _DENSE_CACHE.pop, key, None)
        _DENSE_CACHE[key] = (weakref.ref(indptr), weakref.ref(indices), weakref.ref(values),
                             int(num_cols), _ver(indptr), _ver(indices), _ver(values), plan)
    return plan


_BSORT_CACHE: "dict" = {}


def bsort_plan(indptr: torch.Tensor, indices: torch.Tensor, num_cols: int, k: int,
               cache: bool = True):
    """(bucket_ptr int32 [nb+1], bucket_pos int32 [E], bucket_dst uint16 [E], win_src uint16
    [E], edge_row int32 [E], shift) of a CSR graph for the window-sorted backward at width k
    (maxk_bsort_plan): the bucket plan of maxk_bucket_shift(k) with each entry's T row in
    place of its edge id, per T row the edge (within its window of maxk_bsort_window(k) CSR
    edges) phase 1 stores there, and the source row of every edge.  Built once per graph and k on the GPU; cached per
    (indptr, indices) tensor objects (and their version counters)."""
    _need(indptr, "indptr", torch.int32)
    _need(indices, "indices", torch.int32)
    L = _lib()
    if int(L.maxk_bsort_window(int(k))) <= 0:
        raise RuntimeError(f"bsort_plan: k must be a multiple of 4 in [4, 256], got {k}")
    shift = int(L.maxk_bucket_shift(int(k)))
    key = (id(indptr), id(indices), int(k))
    hit = _BSORT_CACHE.get(key)
    if cache and hit is not None:
        rp, ri, nc, pv, vi, plan = hit
        if (rp() is indptr and ri() is indices and nc == num_cols and pv == _ver(indptr)
                and vi == _ver(indices)):
            return plan
    dev = indices.device
    E = indices.numel()
    num_rows = indptr.numel() - 1
    nb = int(L.maxk_bucket_count(num_cols, shift))
    bptr = torch.empty(nb + 1, dtype=torch.int32, device=dev)
    bpos = torch.empty(max(E, 1), dtype=torch.int32, device=dev)[:E]
    bdst = torch.empty(max(E, 1), dtype=torch.uint16, device=dev)[:E]
    wsrc = torch.empty(max(E, 1), dtype=torch.uint16, device=dev)[:E]
    wrow = torch.empty(max(E, 1), dtype=torch.int32, device=dev)[:E]
    ws = torch.empty(max(1, L.maxk_bsort_plan_workspace_size(num_cols, E)), dtype=torch.uint8,
                     device=dev)
    with _on(dev):
        _capi.check(L.maxk_bsort_plan(_ptr(indptr), _ptr(indices), num_rows, num_cols, E, int(k),
                                      shift, _ptr(bptr), _ptr(bpos), _ptr(bdst), _ptr(wsrc),
                                      _ptr(wrow), _ptr(ws), ws.numel(), _stream(dev)),
                    "maxk_bsort_plan")
    plan = (bptr, bpos, bdst, wsrc, wrow, shift)
    if cache:
        if key not in _BSORT_CACHE:
            for t in (indptr, indices):
                weakref.finalize(t, _BSORT_CACHE.pop, key, None)
        _BSORT_CACHE[key] = (weakref.ref(indptr), weakref.ref(indices), int(num_cols),
                             _ver(indptr), _ver(indices), plan)
    return plan


_PULL_CACHE: dict = {}


def pull_plan(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, num_cols: int,
              k: int, dim: int = 256, slices: Optional[int] = None, cache: bool = True,
              shift: Optional[int] = None):
    """(tile_ptr int32 [S*nb+1], ent int32 [E, 2], shift, S) of a CSR graph and its edge
    values for the pull backward at width k: rows cut into S slices (default
    maxk_pull_slices: ~3.5 MiB of G rows per slice and rank part, at most 3 parts), columns into
    buckets of 2^shift; per tile
    (slice, bucket) the edges in CSR order, each {row in its slice | column in its bucket
    << 16, weight bits}.  Built on the GPU (one stable radix sort); cached per
    (indptr, indices, values) tensor objects and their version counters -- indptr assigns
    the edges to rows and slices, and the weights are copied into the plan, so a plan serves
    the graph and values it was built from.  `shift` overrides the bucket shift
    (maxk_pull_shift(k) by default; any shift the C ABI accepts for k)."""
    for t, n, dt in ((indptr, "indptr", torch.int32), (indices, "indices", torch.int32),
                     (values, "values", torch.float32)):
        _need(t, n, dt)
    L = _lib()
    num_rows = indptr.numel() - 1
    shift = int(L.maxk_pull_shift(int(k))) if shift is None else int(shift)
    if shift < 0:
        raise RuntimeError(f"pull_plan: invalid k {k}")
    if slices:
        S = int(slices)
    else:  # sized by the CU count of the device that holds the graph
        with _on(indices.device):
            S = int(L.maxk_pull_slices(num_rows, int(num_cols), int(dim), int(k)))
    key = (id(indptr), id(indices), id(values), shift, S)
    hit = _PULL_CACHE.get(key)
    if cache and hit is not None:
        rp, ri, rv, nc, pv, vi, vv, plan = hit
        if (rp() is indptr and ri() is indices and rv() is values and nc == num_cols
                and pv == _ver(indptr) and vi == _ver(indices)
                and vv == _ver(values)):
            return plan
    dev = indices.device
    E = indices.numel()
    nb = int(L.maxk_bucket_count(num_cols, shift))
    tptr = torch.empty(S * nb + 1, dtype=torch.int32, device=dev)
    ent = torch.empty(max(E, 1), 2, dtype=torch.int32, device=dev)[:E]
    ws = torch.empty(max(1, L.maxk_pull_plan_workspace_size(num_rows, num_cols, E, shift, S)),
                     dtype=torch.uint8, device=dev)
    with _on(dev):
        _capi.check(L.maxk_pull_plan(_ptr(indptr), _ptr(indices), _ptr(values), num_rows,
                                     num_cols, E, shift, S, _ptr(tptr), _ptr(ent), _ptr(ws),
                                     ws.numel(), _stream(dev)), "maxk_pull_plan")
    plan = (tptr, ent, shift, S)
    if cache:
        if key not in _PULL_CACHE:
            for t in (indptr, indices, values):
                weakref.finalize(t, _PULL_CACHE.pop, key, None)
        _PULL_CACHE[key] = (weakref.ref(indptr), weakref.ref(indices), weakref.ref(values),
                            int(num_cols), _ver(indptr), _ver(indices), _ver(values),
                            plan)
    return plan


_HYBRID_CACHE: "dict" = {}
MAXK_PULL_NO_REDUCE, MAXK_PULL_REDUCE_ONLY = 2, 4  # include/maxk_hip.h
MAXK_HYBRID_PRESCALED = 1
# maxk_backward_mode_auto's codes (include/maxk_hip.h MAXK_BWD_*)
_MODE_OF_CODE = {0: "pull", 1: "csc", 3: "hybrid", 4: "atomic", 5: "bsort", 6: "dense"}
_SIDE: "dict" = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """One extra HIP stream per device (the hybrid backward's tile kernels)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _SIDE:
        _SIDE[i] = torch.cuda.Stream(device=i)
    return _SIDE[i]
# a tile pulls when it holds at least this many entries per row of its slice
HYBRID_DENSITY = 0.5  # MAXK_HYBRID_DENSITY in include/maxk_hip.h
# mode "auto" picks "hybrid" on a sparse graph whose pull_locality reaches this (products-
# sized, k=32: 1.02 (random labels) csc 8.2 vs hybrid 8.4 ms; 1.9: 8.1 vs 6.4; 6.9: 7.4 vs 4.7)
HYBRID_LOCALITY = 1.5  # MAXK_HYBRID_LOCALITY


def hybrid_plan(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                num_cols: int, k: int, dim: int = 256, density: Optional[float] = None,
                cache: bool = True):
    """Plan of the "hybrid" backward (maxk_hybrid_plan, C ABI): the pull over the dense tiles
    of the graph's pull plan (at least `density` entries per row of the tile's slice), the
    two-phase csc over the other edges.  A community-ordered graph keeps most edges in the
    tiles near the diagonal, which pull well, while a pull over every tile would write one
    [num_cols, k] partial per row slice.  Returns (tile_list, tile_ent, bucket_ptr,
    bucket_tiles, ent, shift, S, (off_indptr, off_indices, off_values, off_transpose_plan));
    cached like pull_plan.  k % 4 == 0.  `density` defaults to MAXK_HYBRID_DENSITY or
    HYBRID_DENSITY."""
    if density is None:
        density = float(os.environ.get("MAXK_HYBRID_DENSITY", HYBRID_DENSITY))
    if k % 4:
        raise RuntimeError(f"hybrid backward needs k % 4 == 0, got k={k}")
    key = (id(indptr), id(indices), id(values), int(k), int(dim), float(density))
    hit = _HYBRID_CACHE.get(key)
    if cache and hit is not None:
        rp, ri, rv, nc, pv, vi, vv, plan = hit
        if (rp() is indptr and ri() is indices and rv() is values and nc == num_cols
                and pv == _ver(indptr) and vi == _ver(indices)
                and vv == _ver(values)):
            return plan
    tptr, ent, shift, S = pull_plan(indptr, indices, values, num_cols, k, dim, cache=False)
    dev = indices.device
    L = _lib()
    num_rows = indptr.numel() - 1
    E = indices.numel()
    nb = int(L.maxk_bucket_count(num_cols, shift))
    nt = S * nb
    i32 = dict(dtype=torch.int32, device=dev)
    tile_list = torch.empty(max(nt, 1), **i32)
    tile_ent = torch.empty(nt + 1, **i32)
    bucket_ptr = torch.empty(nb + 1, **i32)
    bucket_tiles = torch.empty(max(nt, 1), **i32)
    ent_d = torch.empty(max(E, 1), 2, **i32)
    off_ip = torch.empty(num_rows + 1, **i32)
    off_ix = torch.empty(max(E, 1), **i32)
    off_val = torch.empty(max(E, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(1, L.maxk_hybrid_plan_workspace_size(num_rows, num_cols, E, shift, S)),
                     dtype=torch.uint8, device=dev)
    counts = (ctypes.c_int64 * 3)()
    with _on(dev):
        _capi.check(L.maxk_hybrid_plan(
            _ptr(indptr), _ptr(indices), _ptr(values), _ptr(tptr), _ptr(ent), num_rows, num_cols,
            E, shift, S, float(density), _ptr(tile_list), _ptr(tile_ent), _ptr(bucket_ptr),
            _ptr(bucket_tiles), _ptr(ent_d), _ptr(off_ip), _ptr(off_ix), _ptr(off_val), counts,
            _ptr(ws), ws.numel(), _stream(dev)), "maxk_hybrid_plan")
    n_t, n_p, n_o = (int(c) for c in counts)
    del tptr, ent, ws
    # the slices are views of their worst-case buffers; copies keep the plan compact
    tile_list, bucket_tiles = tile_list[:n_t].clone(), bucket_tiles[:n_t].clone()
    tile_ent = tile_ent[:n_t + 1].clone()
    ent_d = ent_d[:n_p].clone()
    off_ix, off_val = off_ix[:n_o].clone(), off_val[:n_o].clone()
    off = (off_ip, off_ix, off_val, transpose_plan(off_ix, num_cols, cache=False))
    plan = (tile_list, tile_ent, bucket_ptr, bucket_tiles, ent_d, shift, S, off)
    if cache:
        if key not in _HYBRID_CACHE:
            for t in (indptr, indices, values):
                weakref.finalize(t, _HYBRID_CACHE.pop, key, None)
        _HYBRID_CACHE[key] = (weakref.ref(indptr), weakref.ref(indices), weakref.ref(values),
                              int(num_cols), _ver(indptr), _ver(indices), _ver(values),
                              plan)
    return plan


BWD_MODES = ("auto", "pull", "csc", "atomic", "hybrid", "bsort", "dense")
BSORT_KMAX = 8  # MAXK_BSORT_KMAX: the auto rule's bsort limit
_BSORT_WARNED: set = set()  # (id(indptr), k) already warned about


_LOCALITY: "dict" = {}


_SCALED: "dict" = {}


def _scaled_entries(ent: torch.Tensor, tiles: Optional[torch.Tensor], tile_ent: torch.Tensor,
                    num_rows: int, num_cols: int, shift: int, S: int,
                    row_div: torch.Tensor) -> Optional[torch.Tensor]:
    """The pull entries with each weight divided by its source row's row_div
    (maxk_pull_entries_scale), so the tile kernels gather G itself instead of a G / row_div
    copy (gprime_kernel: a read and a write of all of G per call; ogbn-products 2 x 2.5 GB).
    `tiles[i]` (None: i) is the tile of the entries' i-th run [tile_ent[i], tile_ent[i+1]).
    Cached per entry tensor for one (row_div object, version): the degrees a layer divides by
    are the same tensor every call (maxk_layers.CSRGraph).  None when it would have to be built
    inside a stream capture."""
    key = id(ent)
    hit = _SCALED.get(key)
    if hit is not None:
        re, rd, ver, sc = hit
        if re() is ent and rd() is row_div and ver == _ver(row_div):
            return sc
    if ent.is_cuda and torch.cuda.is_current_stream_capturing():
        # a hipGraph capture records kernels without running them: a copy built here would
        # be cached before it holds anything, so the caller keeps the G / row_div route
        return None
    sc = torch.empty_like(ent)
    dev = ent.device
    n_runs = tile_ent.numel() - 1
    with _on(dev):
        _capi.check(_lib().maxk_pull_entries_scale(
            _ptr(ent), _ptr(tiles), _ptr(tile_ent), n_runs, num_rows, num_cols, shift, S,
            _ptr(row_div), _ptr(sc), _stream(dev)), "maxk_pull_entries_scale")
    if key not in _SCALED:
        weakref.finalize(ent, _SCALED.pop, key, None)
    _SCALED[key] = (weakref.ref(ent), weakref.ref(row_div), _ver(row_div), sc)
    return sc


def _prescale() -> bool:
    """MAXK_PULL_PRESCALE=0 keeps the per-call G / row_div copy instead of scaled entries."""
    return os.environ.get("MAXK_PULL_PRESCALE", "1") != "0"


def pull_locality(indptr: torch.Tensor, indices: torch.Tensor, shift: int) -> float:
    """Edges per occupied (source row, bucket of 2^shift columns) pair (maxk_pull_locality):
    how many entries of a pull tile share a source row's G lines.  A randomly labelled graph
    with `a` edges per (row, bucket) on average has a / (1 - e^-a) (ogbn-products-sized:
    ~1.0); a graph whose vertex order groups its communities (maxk_graph.locality_order) has
    many more, whatever the average.  One pass over the edges (columns sorted within rows,
    else an under-estimate), cached per (indptr, indices, shift) and their versions.  Reported
    by bench.py (extra.pull_locality); on sparse graphs it steers mode "auto" to "hybrid"."""
    key = (id(indptr), id(indices), int(shift))
    hit = _LOCALITY.get(key)
    if hit is not None:
        rp, ri, pv, iv, val = hit
        if rp() is indptr and ri() is indices and pv == _ver(indptr) and \
                iv == _ver(indices):
            return val
    _need(indptr, "indptr", torch.int32)
    _need(indices, "indices", torch.int32)
    dev = indices.device
    out = ctypes.c_double(0.0)
    ws = torch.empty(8, dtype=torch.uint8, device=dev)
    with _on(dev):
        _capi.check(_lib().maxk_pull_locality(_ptr(indptr), _ptr(indices), indptr.numel() - 1,
                                              indices.numel(), int(shift), ctypes.byref(out),
                                              _ptr(ws), ws.numel(), _stream(dev)),
                    "maxk_pull_locality")
    val = float(out.value)
    if key not in _LOCALITY:
        weakref.finalize(indices, _LOCALITY.pop, key, None)
    _LOCALITY[key] = (weakref.ref(indptr), weakref.ref(indices), _ver(indptr),
                      _ver(indices), val)
    return val


def _bwd_mode(mode: Optional[str], k: int = 4, num_e: int = 0, num_cols: int = 0,
              num_rows: Optional[int] = None, dim: Optional[int] = None,
              graph: Optional[tuple] = None) -> str:
    """Resolve the backward mode.  "auto" (default; MAXK_BWD_MODE overrides) is the C ABI's
    rule, maxk_backward_mode_auto: "dense" at k >= dim / 2 (dim % 4 == 0, dim <= 128, k % 4 ==
    0: Flickr-shaped D = 64 at k = 32 / 64, where a CBSR row is as wide as the dense row);
    else "pull" where it measured faster than "csc" -- k % 4 == 0
    or k <= 64, dim % 4 == 0 when dim is given, and at least ~1/2 edge per (source row,
    bucket of 2^maxk_bucket_shift(k) columns) on average (Reddit k=16: 2.2, k=64: 0.54;
    ogbn-proteins k=64: 1.2; ogbn-products: 0.02), or a gradient G of at most 64 MiB (Flickr:
    23 MB, 0.05 vs 0.13 ms), which stays cache-resident however sparse the graph (at most
    256 x 65536 rows; past that the rules below apply).  On a sparse graph the whole pull loses
    even with locality (its per-slice partials, [num_cols, k] per row slice: a community-
    ordered ogbn-products-sized graph 46 ms against 8 ms csc), but where
    `graph` = (indptr, indices) is given and its pull_locality reaches HYBRID_LOCALITY (k % 4
    == 0, dim % 4 == 0) "hybrid" pulls the dense tiles and runs csc over the rest (that graph:
    4.7 against 7.4 ms); otherwise "bsort" at k % 4 == 0, k <= 8 when a window of
    maxk_bsort_window(k) edges holds >= 2 rows per destination bucket on average (ogbn-
    products k = 8: 2.9 against 3.9 ms for csc, both with the selector stream), else "csc".
    "pull", "bsort" and "hybrid" sum in fp64 LDS accumulators: two runs
    agree except in rare fp32 rounding ties; MAXK_BWD_MODE=csc forces the bitwise-
    deterministic form everywhere."""
    mode = mode or os.environ.get("MAXK_BWD_MODE", "auto")
    if mode not in BWD_MODES:
        raise RuntimeError(f"backward mode must be one of {BWD_MODES}, got {mode!r}")
    if mode == "auto":
        L = _lib()
        rows = num_rows if num_rows else num_cols
        D = -1 if dim is None else int(dim)
        code = int(L.maxk_backward_mode_auto(rows, num_cols, num_e, D, int(k), -1.0))
        if (code in (1, 5) and graph is not None and k % 4 == 0 and num_e > 0
                and rows <= 256 * 65536):  # csc / bsort unless the locality asks for hybrid
            loc = pull_locality(graph[0], graph[1], int(L.maxk_pull_shift(int(k))))
            code = int(L.maxk_backward_mode_auto(rows, num_cols, num_e, D, int(k), loc))
        mode = _MODE_OF_CODE[code]
    if mode == "bsort" and k % 4 != 0:
        raise RuntimeError(f"backward mode '{mode}' needs k % 4 == 0, got k={k}")
    if mode == "pull" and k % 4 != 0 and k > 64:
        raise RuntimeError(f"backward mode 'pull' needs k % 4 == 0 or k <= 64, got k={k}")
    if mode == "pull" and dim is not None and dim % 4 != 0:
        raise RuntimeError(f"backward mode 'pull' needs dim_origin % 4 == 0, got {dim}")
    if mode == "dense" and (k % 4 != 0 or (dim is not None and dim % 4 != 0)):
        raise RuntimeError(f"backward mode 'dense' needs k % 4 == 0 and dim_origin % 4 == 0, "
                           f"got k={k}, dim={dim}")
    if mode == "hybrid" and (k % 4 != 0 or (dim is not None and dim % 4 != 0)):
        raise RuntimeError(f"backward mode 'hybrid' needs k % 4 == 0 and dim_origin % 4 == 0, "
                           f"got k={k}, dim={dim}")
    return mode


def backward_plan(indices: torch.Tensor, num_cols: int, k: int, mode: Optional[str] = None,
                  num_rows: Optional[int] = None, indptr: Optional[torch.Tensor] = None,
                  values: Optional[torch.Tensor] = None, dim: Optional[int] = None):
    """The per-graph plan sspmm_backward needs for `mode` at width k (None for "atomic");
    num_rows (default num_cols) and dim only steer mode "auto".  Mode "pull" also needs
    the graph's indptr and edge values."""
    mode = _bwd_mode(mode, k, indices.numel(), num_cols, num_rows, dim,
                     None if indptr is None else (indptr, indices))
    if mode in ("pull", "hybrid"):
        if indptr is None or values is None:
            raise RuntimeError(f"backward_plan: mode '{mode}' needs indptr= and values=")
        if mode == "hybrid":
            return hybrid_plan(indptr, indices, values, num_cols, k, dim or 256)
        return pull_plan(indptr, indices, values, num_cols, k, dim or 256)
    if mode == "dense":
        if indptr is None or values is None:
            raise RuntimeError("backward_plan: mode 'dense' needs indptr= and values=")
        return dense_plan(indptr, indices, values, num_cols)
    if mode == "bsort":
        if indptr is None:
            raise RuntimeError("backward_plan: mode 'bsort' needs indptr=")
        return bsort_plan(indptr, indices, num_cols, k)
    if mode == "csc":
        return transpose_plan(indices, num_cols)
    return None


def sspmm_backward(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                   grad_output: torch.Tensor, cbsr_idx: torch.Tensor,
                   row_div: Optional[torch.Tensor] = None, chunk: int = 0,
                   out: Optional[torch.Tensor] = None, validate: Optional[bool] = None,
                   mode: Optional[str] = None, plan=None,
                   edge_sel: Optional[torch.Tensor] = None) -> torch.Tensor:
    """grad_cbsr[num_cols, k] = (A^T diag(1/row_div) G)[c, cbsr_idx[c, l]].

    edge_sel (uint8 [E, k], k % 4 == 0; modes "csc" and "bsort", ignored by the others): the
    selectors per edge (edge_selectors(), or the forward's by-product), read in CSR order
    instead of gathered.

    mode "auto" (default; MAXK_BWD_MODE overrides): "pull", "hybrid" or "csc", see _bwd_mode.
    mode "pull": per tile (row slice, destination bucket), the k values of every edge
    gathered from G and summed in fp64 LDS accumulators, no contribution rows (with a
    row_div the plan's weights are pre-divided, once per divisor: _scaled_entries);
    uses the graph's pull plan (built once per (indptr, indices, values) and cached, or
    `plan=` from pull_plan()); fp64 tile sums, so two runs agree except in rare rounding
    ties (use "csc" for bitwise repeatability).
    mode "csc": two-phase, atomic-free and bitwise deterministic, using the graph's
    transpose plan (built once and cached, or `plan=` from transpose_plan()).
    mode "bsort" (k % 4 == 0): two-phase, phase 1 writing each window of maxk_bsort_window(k)
    CSR edges' rows ordered by destination bucket (staged in LDS), phase 2 summing each
    bucket's rows of a window as one run in fp64 LDS accumulators -- for large sparse graphs
    at small k, where a csc phase 2 pays a whole random line per 32-B row (bsort_plan()).
    mode "atomic": one global fp32 atomic per (edge, l); no preprocessing.
    mode "dense" (k % 4 == 0, dim % 4 == 0; "auto" picks it at k >= dim / 2, dim <= 128,
    maxk_dense_route): Y = A^T diag(1/row_div) G over dense G rows along the graph's transpose
    with source rows (dense_plan), then the k selected columns of each row of Y; bitwise
    repeatable.
    mode "hybrid" (k % 4 == 0; "auto" picks it on sparse graphs with locality): the pull
    over the dense tiles of the pull plan, on a second stream, beside csc over the other
    edges (hybrid_plan), for large graphs whose vertex order groups their communities."""
    for t, n, dt in ((indptr, "indptr", torch.int32), (indices, "indices", torch.int32),
                     (values, "values", torch.float32), (grad_output, "grad_output", torch.float32),
                     (cbsr_idx, "sparse_selector", torch.uint8)):
        _need(t, n, dt)
    num_rows = indptr.numel() - 1
    if grad_output.dim() != 2 or grad_output.shape[0] != num_rows:
        raise RuntimeError("grad_output must be [num_rows, dim_origin]")
    D = grad_output.shape[1]
    num_cols, k = cbsr_idx.shape
    if row_div is not None:
        _need(row_div, "row_div", torch.float32)
        if row_div.numel() != num_rows:
            raise RuntimeError("row_div must have num_rows entries")
    _validate_call(validate, indptr, indices, num_cols, cbsr_idx, D)
    dev = grad_output.device
    if out is None:
        out = torch.empty(num_cols, k, dtype=torch.float32, device=dev)
    else:
        _need(out, "out", torch.float32)
        if tuple(out.shape) != (num_cols, k):
            raise RuntimeError("out must be [num_cols, k]")
    L = _lib()
    E = indices.numel()
    asked = mode or os.environ.get("MAXK_BWD_MODE", "auto")
    mode = _bwd_mode(mode, k, E, num_cols, num_rows, D, (indptr, indices))
    if mode == "dense":
        aligned = (grad_output.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
                   and cbsr_idx.data_ptr() % 4 == 0)
        if not aligned and asked == "auto":
            mode, plan = "pull", None  # the dense kernels' vector loads need aligned rows
    if mode == "dense":
        col_ptr, t_src, t_w = (plan if plan is not None
                               else dense_plan(indptr, indices, values, num_cols))
        ws_bytes = L.maxk_sspmm_backward_dense_workspace_size(num_rows, num_cols, E, D, k, chunk)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        with _on(dev):
            _capi.check(L.maxk_sspmm_backward_dense(
                _ptr(col_ptr), _ptr(t_src), _ptr(t_w), _ptr(grad_output), _ptr(row_div),
                _ptr(cbsr_idx), _ptr(out), num_rows, num_cols, E, D, k, chunk, _ptr(ws),
                ws.numel(), _stream(dev)), "maxk_sspmm_backward_dense")
        return out
    if mode == "hybrid":
        tl, te, bp, bt, ent, shift, S, off = (plan if plan is not None else
                                             hybrid_plan(indptr, indices, values, num_cols, k, D))
        oip, oix, oval, (ocp, oeid) = off
        n_t = tl.numel()
        flags = 0
        if row_div is not None and n_t > 0 and _prescale():
            sc = _scaled_entries(ent, tl, te, num_rows, num_cols, shift, S, row_div)
            if sc is not None:
                ent, flags = sc, MAXK_HYBRID_PRESCALED
        ws_bytes = L.maxk_sspmm_backward_hybrid_workspace_size(num_rows, num_cols, oix.numel(),
                                                               D, k, n_t)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        with _on(dev):
            overlap = (oix.numel() > 0 and n_t > 0
                       and os.environ.get("MAXK_HYBRID_STREAMS", "1") != "0")
            if not overlap:  # everything on the caller's stream, in one C-ABI call
                _capi.check(L.maxk_sspmm_backward_hybrid(
                    _ptr(grad_output), _ptr(row_div), _ptr(cbsr_idx), _ptr(tl), _ptr(te), n_t,
                    _ptr(bp), _ptr(bt), _ptr(ent), ent.shape[0], shift, S, _ptr(oip), _ptr(oix),
                    _ptr(oval), oix.numel(), _ptr(ocp), _ptr(oeid), flags, _ptr(out), num_rows,
                    num_cols, D, k, _ptr(ws), ws.numel(), _stream(dev), None, None, None),
                    "maxk_sspmm_backward_hybrid")
                return out
            # the same sequence with the tile kernels on a side stream beside the csc, forked
            # and joined by torch (fresh events each call: one pair re-recorded by eager calls
            # broke the join of a graph captured with it, test_hipgraph_capture_*[hybrid])
            a = L.maxk_sspmm_backward_csc_workspace_size(num_rows, num_cols, oix.numel(), D, k, 0)
            a = (a + 255) // 256 * 256
            ws_csc, ws_pull = ws[:a], ws[a:]
            tile_div = None if flags & MAXK_HYBRID_PRESCALED else row_div

            def tiles(acc, stream):
                _capi.check(L.maxk_sspmm_backward_pull_tiles(
                    _ptr(grad_output), _ptr(tile_div), _ptr(cbsr_idx), _ptr(tl), _ptr(te), n_t,
                    _ptr(bp), _ptr(bt), _ptr(ent), shift, S, acc, _ptr(out), num_rows, num_cols,
                    ent.shape[0], D, k, _ptr(ws_pull), ws_pull.numel(), stream),
                    "maxk_sspmm_backward_pull_tiles")
            main = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(main)
            tiles(MAXK_PULL_NO_REDUCE, ctypes.c_void_p(side.cuda_stream))
            _capi.check(L.maxk_sspmm_backward_csc(
                _ptr(oip), _ptr(oix), _ptr(oval), _ptr(grad_output), _ptr(row_div),
                _ptr(cbsr_idx), _ptr(ocp), _ptr(oeid), _ptr(out), num_rows, num_cols, oix.numel(),
                D, k, 0, _ptr(ws_csc), ws_csc.numel(), _stream(dev)), "maxk_sspmm_backward_csc")
            main.wait_stream(side)
            tiles(MAXK_PULL_REDUCE_ONLY | 1, _stream(dev))
        # the side stream is joined to the caller's stream before the call returns, so what
        # it read (ws included) is free for reuse in that stream's order
        return out
    if mode == "pull":
        tptr, ent, shift, S = (plan if plan is not None else
                               pull_plan(indptr, indices, values, num_cols, k, D))
        if row_div is not None and E > 0 and _prescale():
            sc = _scaled_entries(ent, None, tptr, num_rows, num_cols, shift, S, row_div)
            if sc is not None:
                ent, row_div = sc, None
        ws_bytes = L.maxk_sspmm_backward_pull_workspace_size(num_rows, num_cols, D, k, S)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        with _on(dev):
            _capi.check(L.maxk_sspmm_backward_pull(
                _ptr(grad_output), _ptr(row_div), _ptr(cbsr_idx), _ptr(tptr), _ptr(ent), shift,
                S, _ptr(out), num_rows, num_cols, E, D, k, _ptr(ws), ws.numel(), _stream(dev)),
                "maxk_sspmm_backward_pull")
        return out
    if mode == "bsort":
        if k > BSORT_KMAX and (id(indptr), k) not in _BSORT_WARNED:
            _BSORT_WARNED.add((id(indptr), k))
            warnings.warn(f"backward mode 'bsort' at k={k} > {BSORT_KMAX} (MAXK_BSORT_KMAX): a "
                          f"window of {int(L.maxk_bsort_window(k))} edges holds few rows per "
                          "destination bucket; correct, but csc is faster", stacklevel=2)
        bptr, bpos, bdst, wsrc, wrow, shift = (plan if plan is not None
                                               else bsort_plan(indptr, indices, num_cols, k))
        if edge_sel is not None:
            _need(edge_sel, "edge_sel", torch.uint8)
            if tuple(edge_sel.shape) != (E, k):
                raise RuntimeError("edge_sel must be [num_e, k]")
        ws_bytes = L.maxk_sspmm_backward_bsort_workspace_size(num_rows, num_cols, E, D, k)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        with _on(dev):
            _capi.check(L.maxk_sspmm_backward_bsort(
                _ptr(indptr), _ptr(indices), _ptr(values), _ptr(grad_output), _ptr(row_div),
                _ptr(cbsr_idx), _ptr(edge_sel), _ptr(bptr), _ptr(bpos), _ptr(bdst), _ptr(wsrc),
                _ptr(wrow), shift, _ptr(out), num_rows, num_cols, E, D, k, _ptr(ws), ws.numel(),
                _stream(dev)), "maxk_sspmm_backward_bsort")
        return out
    if mode == "atomic":
        ws_bytes = L.maxk_sspmm_backward_workspace_size(num_rows, num_cols, E, D, k, chunk)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        with _on(dev):
            _capi.check(L.maxk_sspmm_backward(
                _ptr(indptr), _ptr(indices), _ptr(values), _ptr(grad_output), _ptr(row_div),
                _ptr(cbsr_idx), _ptr(out), num_rows, num_cols, E, D, k, chunk, _ptr(ws),
                ws.numel(), _stream(dev)), "maxk_sspmm_backward")
        return out
    col_ptr, csc_eid = plan if plan is not None else transpose_plan(indices, num_cols)
    ws_bytes = L.maxk_sspmm_backward_csc_workspace_size(num_rows, num_cols, E, D, k, chunk)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if edge_sel is not None:
        _need(edge_sel, "edge_sel", torch.uint8)
        if tuple(edge_sel.shape) != (E, k):
            raise RuntimeError("edge_sel must be [num_e, k]")
        with _on(dev):
            _capi.check(L.maxk_sspmm_backward_csc_sel(
                _ptr(indptr), _ptr(indices), _ptr(values), _ptr(grad_output), _ptr(row_div),
                _ptr(edge_sel), _ptr(col_ptr), _ptr(csc_eid), _ptr(out), num_rows, num_cols, E,
                D, k, chunk, _ptr(ws), ws.numel(), _stream(dev)), "maxk_sspmm_backward_csc_sel")
        return out
    with _on(dev):
        _capi.check(L.maxk_sspmm_backward_csc(
            _ptr(indptr), _ptr(indices), _ptr(values), _ptr(grad_output), _ptr(row_div),
            _ptr(cbsr_idx), _ptr(col_ptr), _ptr(csc_eid), _ptr(out), num_rows, num_cols, E, D,
            k, chunk, _ptr(ws), ws.numel(), _stream(dev)), "maxk_sspmm_backward_csc")
    return out


EDGE_SEL_KMAX = 16


def edge_selectors_wanted(k: int) -> bool:
    """The rule for the per-edge selector stream given a csc / bsort backward: k % 4 == 0 and
    k <= EDGE_SEL_KMAX by default (MAXK_EDGE_SEL=auto); MAXK_EDGE_SEL=0 never, =1 at every
    k % 4 == 0.  Measured on the ogbn-products-sized graph: the forward that
    writes the stream takes +0.68 / +0.80 / +0.79 ms at k = 8 / 16 / 32, the csc backward that
    reads it -1.16 / -1.08 / -0.93 ms.  At k = 32 that nets +1 % on the bench step and -1.5 % on
    the 3-layer training epoch (r04, one box, alternating runs: 13.46 -> 13.31 ms, 100.1 ->
    101.6 ms; profiles/r04/tune/es32/), for num_e * k bytes (4 GB) held per layer from the
    forward to the backward, so the default stops at 16; none at 64 (+2.15 / -1.33 ms)."""
    mode = os.environ.get("MAXK_EDGE_SEL", "auto")
    if k % 4 or mode == "0":
        return False
    return mode == "1" or k <= EDGE_SEL_KMAX


def edge_selector_mode(indptr: torch.Tensor, indices: torch.Tensor, k: int, num_cols: int,
                       dim: Optional[int] = None) -> Optional[str]:
    """The backward mode a forward should write the per-edge selector stream for
    (spgemm_forward(edge_sel_out=) -> sspmm_backward(edge_sel=, mode=)), or None: the backward
    resolves to "csc" or "bsort" (large sparse graphs without locality, where phase 1
    otherwise gathers a 128-B line of the selector table per edge) and
    edge_selectors_wanted(k).  The stream holds num_e * k bytes until the backward."""
    if indices.numel() == 0 or not edge_selectors_wanted(k):
        return None
    mode = _bwd_mode(None, k, indices.numel(), num_cols, indptr.numel() - 1, dim,
                     (indptr, indices))
    return mode if mode in ("csc", "bsort") else None


def use_edge_selectors(indptr: torch.Tensor, indices: torch.Tensor, k: int, num_cols: int,
                       dim: Optional[int] = None) -> bool:
    """Whether a forward should write the per-edge selector stream (edge_selector_mode)."""
    return edge_selector_mode(indptr, indices, k, num_cols, dim) is not None


def edge_selectors(indices: torch.Tensor, cbsr_idx: torch.Tensor,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [E, k]: edge e's destination selectors, cbsr_idx[indices[e]] (any k, any
    alignment), for sspmm_backward(..., edge_sel=) (maxk_edge_selectors)."""
    _need(indices, "indices", torch.int32)
    _need(cbsr_idx, "sparse_selector", torch.uint8)
    E, k = indices.numel(), cbsr_idx.shape[1]
    if out is None:
        out = torch.empty(E, k, dtype=torch.uint8, device=indices.device)
    with torch.cuda.device(indices.device):
        _capi.check(_lib().maxk_edge_selectors(_ptr(indices), _ptr(cbsr_idx), E, k, _ptr(out),
                                               _stream(indices.device)), "maxk_edge_selectors")
    return out


def spmm_maxk_forward(warp4_metadata: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                      input_data: torch.Tensor, sparse_selector: torch.Tensor, num_warps: int,
                      dim_sparse: int, *, dim_origin: int = FULL_DIM,
                      indptr: Optional[torch.Tensor] = None,
                      row_div: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MaxK forward SpGEMM (cuda_kernel_bindings.cpp:42-104): returns f32 [V, dim_origin]."""
    _need(input_data, "input_data", torch.float32)
    if input_data.dim() != 2 or input_data.shape[1] != dim_sparse:
        raise RuntimeError("input_data must be [V, dim_sparse]")
    if indptr is None:
        indptr = warp4_to_indptr(warp4_metadata, input_data.shape[0], num_warps)
    return spgemm_forward(indptr, indices, values, input_data, sparse_selector, dim_origin,
                          row_div=row_div)


def spmm_maxk_backward(warp4_metadata: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                       grad_output: torch.Tensor, sparse_selector: torch.Tensor, num_warps: int,
                       dim_sparse: int, *, indptr: Optional[torch.Tensor] = None,
                       row_div: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MaxK backward SSpMM (cuda_kernel_bindings.cpp:106-161): returns f32 [V, dim_sparse]."""
    _need(grad_output, "grad_output", torch.float32)
    _need(sparse_selector, "sparse_selector", torch.uint8)
    if sparse_selector.dim() != 2 or sparse_selector.shape[1] != dim_sparse:
        raise RuntimeError("sparse_selector must be [V, dim_sparse]")
    if indptr is None:
        indptr = warp4_to_indptr(warp4_metadata, grad_output.shape[0], num_warps)
    return sspmm_backward(indptr, indices, values, grad_output, sparse_selector, row_div=row_div)


# --------------------------------------------------------------------------- CBSR encode
def topk_cbsr(x: torch.Tensor, k: int, with_int32: bool = False):
    """(values, uint8 indices[, int32 indices]) = torch.topk(x, k, dim=1) on the GPU kernel."""
    if x.dim() != 2:
        raise RuntimeError("Input must be 2D tensor")
    if not x.is_cuda:
        raise RuntimeError("Input must be on CUDA")
    if x.stride(1) != 1:
        x = x.contiguous()
    V, D = x.shape
    if not (0 < k <= D):
        raise RuntimeError("Invalid k value")
    dev = x.device
    val = torch.empty(V, k, dtype=x.dtype, device=dev)
    idx = torch.empty(V, k, dtype=torch.uint8, device=dev)
    idx32 = torch.empty(V, k, dtype=torch.int32, device=dev) if with_int32 else None
    L = _lib()
    if x.dtype == torch.float32:
        fn, name = L.maxk_topk_cbsr, "maxk_topk_cbsr"
    elif x.dtype == torch.uint8:
        fn, name = L.maxk_topk_cbsr_u8, "maxk_topk_cbsr_u8"
    else:
        raise RuntimeError("Input must be float32 or uint8")
    check = _checks_topk_rows(dev)
    with _on(dev):
        _capi.check(fn(_ptr(x), x.stride(0), _ptr(val), _ptr(idx), _ptr(idx32), V, D, k,
                       _stream(dev)), name)
    if check:
        _check_topk_rows(dev, name)
    return (val, idx, idx32) if with_int32 else (val, idx)


def topk_error_rows(device=None, reset: bool = True) -> int:
    """Rows whose top-k search took other than k winners on `device` since the last reset
    (maxk_topk_error_rows; read in order on torch's current stream, which it synchronises).
    Always 0 unless the kernel has a bug: the kernels count such a row and keep its writes
    inside its own k winner slots."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    n = ctypes.c_int64(0)
    with _on(dev):
        _capi.check(_lib().maxk_topk_error_rows(ctypes.byref(n), 1 if reset else 0,
                                                _stream(dev)), "maxk_topk_error_rows")
    return int(n.value)


def _checks_topk_rows(dev) -> bool:
    """MAXK_VALIDATE=1 outside a capture: zero the device's bad-row count before the launch
    (a count left by an earlier unvalidated call is not this launch's), so the
    read after it (_check_topk_rows) sees this launch's rows only.  Both run on the current
    stream, in order with the launch."""
    if not _validate_default() or torch.cuda.is_current_stream_capturing():
        return False
    topk_error_rows(dev, reset=True)
    return True


def _check_topk_rows(dev, name):
    """Raise if the launch just made left a row with other than k winners."""
    bad = topk_error_rows(dev)
    if bad:
        raise RuntimeError(f"{name}: {bad} rows took other than k winners (kernel bug)")


def topk_u8_reference(input: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """The reference uint8 top-k's intended per-row convention (maxk_topk_u8_reference; rows of
    256 bytes): (values u8 [N,k], indices u8 [N,k]) -- the row's bytes above its own 8-step
    bisection threshold in ascending column order, the lane-31 overwrite and zero-filled slots
    included.  Not the CUDA kernel as built, which thresholds every row on its block's first
    row per lane, with a shared-memory race and uninitialised slots (kernels/maxk_kernel.cu:42,
    :44-48, :91-94; oracle.topk_u8_reference_as_built models it, and it agrees with this on
    0.2 % of uniform rows): parity with the CUDA kernel is unpinned."""
    _need(input, "input", torch.uint8)
    if input.dim() != 2 or input.shape[1] != 256:
        raise RuntimeError("the reference's uint8 top-k takes [N, 256] rows")
    if not 0 < k <= 256:
        raise RuntimeError("Invalid k value")
    N = input.shape[0]
    val = torch.empty(N, k, dtype=torch.uint8, device=input.device)
    idx = torch.empty(N, k, dtype=torch.uint8, device=input.device)
    with _on(input.device):
        _capi.check(_lib().maxk_topk_u8_reference(_ptr(input), _ptr(val), _ptr(idx), N, 256, int(k),
                                                  _stream(input.device)), "maxk_topk_u8_reference")
    return val, idx


def cuda_topk_maxk(input: torch.Tensor, k: int,
                   reference_compat: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """uint8 top-k (cuda_kernel_bindings.cpp:164-201): (values u8 [N,k], indices u8 [N,k]).
    Exact torch.topk order by default; reference_compat=True takes the reference kernel's
    intended convention (topk_u8_reference: per-row threshold bisection, ascending columns,
    rows of 256) -- not its as-built output, which is racy; parity with it unpinned."""
    if input.dtype != torch.uint8:
        raise RuntimeError("Input must be uint8 tensor")
    if reference_compat:
        return topk_u8_reference(input, k)
    return topk_cbsr(input, k)


def cuda_topk_maxk_float(input: torch.Tensor, k: int,
                         reference_compat: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """(values, int32 indices) (cuda_kernel_bindings.cpp:203-238), exact (no uint8 quantisation)
    by default.  reference_compat=True follows the reference binding: float input quantised to
    clamp(round(x * 255), 0, 255) as uint8, the reference kernel's intended top-k convention on
    that (topk_u8_reference; parity with the as-built CUDA kernel unpinned), values returned as
    float / 255; uint8 input passes through."""
    if not reference_compat:
        val, _, idx32 = topk_cbsr(input, k, with_int32=True)
        return val, idx32
    if input.dtype == torch.float32:
        q = torch.clamp((input * 255.0).round(), 0, 255).to(torch.uint8)
        v8, i8 = topk_u8_reference(q.contiguous(), k)
        # byte / 255 correctly rounded (the device divide may be off by an ulp): a 256-entry
        # table divided on the host
        table = (torch.arange(256, dtype=torch.float32) / 255.0).to(input.device)
        return table[v8.long()], i8.to(torch.int32)
    if input.dtype == torch.uint8:
        v8, i8 = topk_u8_reference(input, k)
        return v8, i8.to(torch.int32)
    raise RuntimeError("Input must be float32 or uint8")


def prepare_cbsr_format_maxk(features: torch.Tensor, maxk: int):
    """(sparse_data, sparse_indices) (cuda_kernel_bindings.cpp:240-251)."""
    return cuda_topk_maxk_float(features, maxk)


def cbsr_scatter_dense(cbsr_val: torch.Tensor, cbsr_idx: torch.Tensor, dim_origin: int,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """zeros(V, D).scatter_(1, idx, val) in one HIP pass (maxk_spgemm_function.py:152,175)."""
    _need(cbsr_val, "cbsr_val", torch.float32)
    _need(cbsr_idx, "cbsr_idx", torch.uint8)
    V, k = cbsr_val.shape
    dev = cbsr_val.device
    if out is None:
        out = torch.empty(V, dim_origin, dtype=torch.float32, device=dev)
    with _on(dev):
        _capi.check(_lib().maxk_cbsr_scatter_dense(_ptr(cbsr_val), _ptr(cbsr_idx), _ptr(out), V,
                                                   dim_origin, k, _stream(dev)),
                    "maxk_cbsr_scatter_dense")
    return out


def topk_cbsr_dense(x: torch.Tensor, k: int):
    """Fused MaxK forward: (dense masked x, values, uint8 indices) from one HIP kernel --
    torch.topk + zeros_like + scatter_ of model_integrated_v3.py:28-38 in a single pass."""
    if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32):
        raise RuntimeError("x must be a float32 CUDA tensor")
    if x.dim() != 2:
        raise RuntimeError("Input must be 2D tensor")
    if x.stride(1) != 1:
        x = x.contiguous()
    V, D = x.shape
    if not (0 < k <= D):
        raise RuntimeError("Invalid k value")
    dev = x.device
    val = torch.empty(V, k, dtype=torch.float32, device=dev)
    idx = torch.empty(V, k, dtype=torch.uint8, device=dev)
    dense = torch.empty(V, D, dtype=torch.float32, device=dev)
    check = _checks_topk_rows(dev)
    with _on(dev):
        _capi.check(_lib().maxk_topk_cbsr_dense(_ptr(x), x.stride(0), _ptr(val), _ptr(idx),
                                                _ptr(dense), V, D, k, _stream(dev)),
                    "maxk_topk_cbsr_dense")
    if check:
        _check_topk_rows(dev, "maxk_topk_cbsr_dense")
    return dense, val, idx


def topk_backward(grad_val: Optional[torch.Tensor], grad_dense: Optional[torch.Tensor],
                  cbsr_idx: torch.Tensor, dim_origin: int,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused MaxK backward: grad_x = scatter(grad_val + grad_dense[sel]) over the selected
    columns, zero elsewhere, in one HIP pass (OPTMaxK.backward, model_integrated_v3.py:39-43,
    with the topk_values gradient it drops; maxk_spgemm_function.py:152,175)."""
    _need(cbsr_idx, "cbsr_idx", torch.uint8)
    V, k = cbsr_idx.shape
    dev = cbsr_idx.device
    if grad_val is not None:
        _need(grad_val, "grad_val", torch.float32)
        if tuple(grad_val.shape) != (V, k):
            raise RuntimeError("grad_val must be [V, k]")
    if grad_dense is not None:
        _need(grad_dense, "grad_dense", torch.float32)
        if tuple(grad_dense.shape) != (V, dim_origin):
            raise RuntimeError("grad_dense must be [V, dim_origin]")
    if out is None:
        out = torch.empty(V, dim_origin, dtype=torch.float32, device=dev)
    else:
        _need(out, "out", torch.float32)
        if tuple(out.shape) != (V, dim_origin):
            raise RuntimeError("out must be [V, dim_origin]")
    with _on(dev):
        _capi.check(_lib().maxk_topk_backward(_ptr(grad_val), _ptr(grad_dense), _ptr(cbsr_idx),
                                              _ptr(out), V, dim_origin, k, _stream(dev)),
                    "maxk_topk_backward")
    return out


def generate_sparse_selector(num_v: int, dim_origin: int, dim_sparse: int) -> torch.Tensor:
    """k distinct random columns per row, seed 123 (cuda_kernel_bindings.cpp:320-340).
    Same distribution as the reference's per-row randperm; not the same random stream."""
    gen = torch.Generator(device="cuda").manual_seed(123)
    keys = torch.rand(num_v, dim_origin, generator=gen, device="cuda")
    return topk_cbsr(keys, dim_sparse)[1]


# --------------------------------------------------------------------------- baseline
class DenseSpMMPlan:
    """rocSPARSE Y = A . X (the reference's cuSPARSE denominator, kernels/spmm_cusparse.cu:6-62).
    Buffers are bound at construction; run() launches on the current stream."""

    def __init__(self, indptr, indices, values, x, y=None, alg: int = 0):
        for t, n, dt in ((indptr, "indptr", torch.int32), (indices, "indices", torch.int32),
                         (values, "values", torch.float32), (x, "input_features", torch.float32)):
            _need(t, n, dt)
        self.num_rows = indptr.numel() - 1
        self.x = x
        self.y = y if y is not None else torch.empty(self.num_rows, x.shape[1],
                                                     dtype=torch.float32, device=x.device)
        self._keep = (indptr, indices, values)
        self.device = x.device
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _capi.check(_lib().maxk_dense_spmm_plan_create(
                ctypes.byref(h), _ptr(indptr), _ptr(indices), _ptr(values), _ptr(x),
                _ptr(self.y), self.num_rows, x.shape[0], indices.numel(), x.shape[1], alg,
                _stream(self.device)), "maxk_dense_spmm_plan_create")
        self._h = h

    def run(self, x: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None
            ) -> torch.Tensor:
        """Y = A . X on the current stream; `x` / `y` rebind the dense operands (same shapes)."""
        if x is not None or y is not None:
            x = self.x if x is None else x
            y = self.y if y is None else y
            _need(x, "x", torch.float32)
            _need(y, "y", torch.float32)
            if tuple(x.shape) != tuple(self.x.shape) or tuple(y.shape) != tuple(self.y.shape):
                raise RuntimeError("rebound x / y must keep the plan's shapes")
            _capi.check(_lib().maxk_dense_spmm_bind(self._h, _ptr(x), _ptr(y)),
                        "maxk_dense_spmm_bind")
            self.x, self.y = x, y
        with torch.cuda.device(self.device):
            _capi.check(_lib().maxk_dense_spmm_run(self._h, _stream(self.device)),
                        "maxk_dense_spmm_run")
        return self.y

    def close(self):
        if getattr(self, "_h", None):
            _lib().maxk_dense_spmm_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cusparse_spmm(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor,
                  input_features: torch.Tensor, timing: bool = False) -> torch.Tensor:
    """Dense SpMM reference (cuda_kernel_bindings.cpp:253-284), here on rocSPARSE."""
    plan = DenseSpMMPlan(indptr, indices, values, input_features)
    try:
        runs = 10 if timing else 1  # the reference's `timing` only repeats the call
        for _ in range(runs):
            plan.run()
        return plan.y
    finally:
        plan.close()


# --------------------------------------------------------------------------- harness helpers
class CudaTimer:
    """Event timer (cuda_kernel_bindings.cpp:343-369) on the current stream; stop() -> ms."""

    def __init__(self):
        self._a = torch.cuda.Event(enable_timing=True)
        self._b = torch.cuda.Event(enable_timing=True)

    def start(self):
        self._a.record()

    def stop(self) -> float:
        self._b.record()
        self._b.synchronize()
        return self._a.elapsed_time(self._b)


def benchmark_spmm_maxk(warp4_metadata, indices, values, input_data, sparse_selector,
                        num_warps: int, dim_sparse: int, num_runs: int = 4) -> List[float]:
    """num_runs warmup + num_runs timed forward calls (cuda_kernel_bindings.cpp:372-402)."""
    indptr = warp4_to_indptr(warp4_metadata, input_data.shape[0], num_warps)
    for _ in range(num_runs):
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse, indptr=indptr)
    torch.cuda.synchronize()
    times, timer = [], CudaTimer()
    for _ in range(num_runs):
        timer.start()
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse, indptr=indptr)
        times.append(timer.stop())
    return times


def validate_spmm_maxk(warp4_metadata, indices, values, input_data, sparse_selector,
                       reference_output, num_warps: int, dim_sparse: int,
                       tolerance: float = 0.001) -> bool:
    """mean |out - reference| < tolerance (cuda_kernel_bindings.cpp:405-427)."""
    out = spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector,
                            num_warps, dim_sparse, dim_origin=reference_output.shape[1])
    diff = (out - reference_output).abs()
    print(f"Validation - Max diff: {diff.max().item()}, Avg diff: {diff.mean().item()}")
    return diff.mean().item() < tolerance


def validate_spmm_maxk_backward(warp4_metadata_csc, indices_csc, values_csc, grad_output,
                                sparse_selector, reference_grad_input, num_warps_csc: int,
                                dim_sparse: int, tolerance: float = 0.001) -> bool:
    """mean |grad - reference| < tolerance (binding_v2.py:464-486).  The arrays are the CSR of
    the forward graph: the kernel forms the A^T product itself."""
    g = spmm_maxk_backward(warp4_metadata_csc, indices_csc, values_csc, grad_output,
                           sparse_selector, num_warps_csc, dim_sparse)
    diff = (g - reference_grad_input).abs()
    print(f"Backward Validation - Max diff: {diff.max().item()}, Avg diff: {diff.mean().item()}")
    return diff.mean().item() < tolerance
