"""ctypes binding of libmaxk_hip.so (the C ABI declared in include/maxk_hip.h).

This is the Python equivalent of the reference's pybind11 layer
(cuda_kernel_bindings.cpp:429-490): it only marshals torch tensors into plain
pointers + sizes and passes torch's current HIP stream.  No compute happens in
Python, and there is no fallback: if the library or a GPU is missing, calls
raise.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "MAXK_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libmaxk_hip.so"))

MAXK_OK = 0
ERRORS = {-1: "invalid argument", -2: "HIP error", -3: "no HIP device", -4: "rocSPARSE error"}

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t

# name -> (restype, argtypes); every symbol of include/maxk_hip.h
SIGNATURES = {
    "maxk_version": (ctypes.c_int, []),
    "maxk_last_error": (ctypes.c_char_p, []),
    "maxk_device_count": (ctypes.c_int, []),
    "maxk_source_digest": (ctypes.c_char_p, []),
    "maxk_build_config": (ctypes.c_char_p, []),
    "maxk_spgemm_forward_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32, _i32]),
    "maxk_spgemm_forward": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                           _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_spgemm_forward_sel": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                           _i32, _i32, _i32, _p, _sz, _p, _p]),
    "maxk_spgemm_forward_accumulate": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                           _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_spgemm_forward_accumulate_sel": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64,
                                                          _i64, _i32, _i32, _i32, _p, _sz, _p,
                                                          _p]),
    "maxk_records_ok": (ctypes.c_int, [_i64, _i64, _i64, _i32, _i32]),
    "maxk_cbsr_records": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_spgemm_forward_records": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i32,
                                                   _i32, _i32, _p, _sz, _p, _i32]),
    "maxk_sspmm_backward_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32, _i32]),
    "maxk_sspmm_backward": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                           _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_sspmm_backward_csc_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32, _i32]),
    "maxk_sspmm_backward_csc": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64,
                                               _i64, _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_sspmm_backward_csc_sel": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64,
                                               _i64, _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_edge_selectors": (ctypes.c_int, [_p, _p, _i64, _i32, _p, _p]),
    "maxk_edge_selectors_blocks": (_i64, [_i64]),
    "maxk_transpose_plan_workspace_size": (_sz, [_i64, _i64]),
    "maxk_transpose_plan": (ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _sz, _p]),
    "maxk_dense_route": (ctypes.c_int, [_i32, _i32]),
    "maxk_dense_plan": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _p, _p]),
    "maxk_sspmm_backward_dense_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32, _i32]),
    "maxk_sspmm_backward_dense": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                                 _i32, _i32, _i32, _p, _sz, _p]),
    "maxk_bucket_shift": (ctypes.c_int, [_i32]),
    "maxk_bucket_count": (_i64, [_i64, _i32]),
    "maxk_bsort_window": (_i32, [_i32]),
    "maxk_bsort_plan_workspace_size": (_sz, [_i64, _i64]),
    "maxk_bsort_plan": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _i32, _i32, _p, _p, _p, _p, _p,
                                       _p, _sz, _p]),
    "maxk_sspmm_backward_bsort_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32]),
    "maxk_sspmm_backward_bsort": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                                 _i32,
                                                 _p, _i64, _i64, _i64, _i32, _i32, _p, _sz, _p]),
    "maxk_sspmm_backward_pull_workspace_size": (_sz, [_i64, _i64, _i32, _i32, _i32]),
    "maxk_sspmm_backward_pull": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _i32, _p, _i64, _i64,
                                                _i64, _i32, _i32, _p, _sz, _p]),
    "maxk_sspmm_backward_pull_tiles_workspace_size": (_sz, [_i64, _i64, _i32, _i32, _i32]),
    "maxk_sspmm_backward_pull_tiles": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _p, _p, _p, _i32,
                                                      _i32, _i32, _p, _i64, _i64, _i64, _i32,
                                                      _i32, _p, _sz, _p]),
    "maxk_pull_shift": (ctypes.c_int, [_i32]),
    "maxk_pull_slices": (ctypes.c_int, [_i64, _i64, _i32, _i32]),
    "maxk_pull_plan_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32]),
    "maxk_pull_plan": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _i32, _i32, _p, _p, _p, _sz,
                                      _p]),
    "maxk_backward_mode_auto": (ctypes.c_int, [_i64, _i64, _i64, _i32, _i32, ctypes.c_double]),
    "maxk_pull_locality": (ctypes.c_int, [_p, _p, _i64, _i64, _i32,
                                          ctypes.POINTER(ctypes.c_double), _p, _sz, _p]),
    "maxk_hybrid_plan_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32]),
    "maxk_hybrid_plan": (ctypes.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i32, _i32,
                                        ctypes.c_float, _p, _p, _p, _p, _p, _p, _p, _p,
                                        ctypes.POINTER(_i64), _p, _sz, _p]),
    "maxk_pull_entries_scale": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _i32, _i32, _p, _p,
                                               _p]),
    "maxk_sspmm_backward_hybrid_workspace_size": (_sz, [_i64, _i64, _i64, _i32, _i32, _i64]),
    "maxk_sspmm_backward_hybrid": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _p, _p, _p, _i64,
                                                  _i32, _i32, _p, _p, _p, _i64, _p, _p, _i32, _p,
                                                  _i64, _i64, _i32, _i32, _p, _sz, _p, _p, _p,
                                                  _p]),
    "maxk_topk_cbsr": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_topk_cbsr_u8": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_topk_u8_reference": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_topk_error_rows": (ctypes.c_int, [_p, _i32, _p]),
    "maxk_cbsr_scatter_dense": (ctypes.c_int, [_p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_topk_cbsr_dense": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_topk_backward": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i32, _i32, _p]),
    "maxk_warp4_count": (ctypes.c_int, [_p, _i64, _i32, ctypes.POINTER(_i64), _p]),
    "maxk_warp4_build_workspace_size": (_sz, [_i64]),
    "maxk_warp4_build": (ctypes.c_int, [_p, _i64, _i32, _p, _i64, _p, _sz, _p]),
    "maxk_warp4_to_row_ptr": (ctypes.c_int, [_p, _i64, _i64, _p, _p]),
    "maxk_dense_spmm_plan_create": (ctypes.c_int, [ctypes.POINTER(_p), _p, _p, _p, _p, _p,
                                                   _i64, _i64, _i64, _i32, _i32, _p]),
    "maxk_dense_spmm_run": (ctypes.c_int, [_p, _p]),
    "maxk_dense_spmm_bind": (ctypes.c_int, [_p, _p, _p]),
    "maxk_dense_spmm_plan_destroy": (ctypes.c_int, [_p]),
}

_lib = None
_load_error = None


def load():
    """Load libmaxk_hip.so once; raises ImportError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise ImportError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libmaxk_hip.so not found at {LIB_PATH}; build it with "
                       f"`make -C spgemm-prunning_amd` (hipcc, gfx950)")
        raise ImportError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as exc:
        _load_error = f"cannot load {LIB_PATH}: {exc}"
        raise ImportError(_load_error) from exc
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != MAXK_OK:
        msg = _lib.maxk_last_error().decode(errors="replace") if _lib is not None else ""
        raise RuntimeError(f"{what} failed ({ERRORS.get(rc, rc)}): {msg}")
