#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE's own code.

Run here (the container with /root/reference mounted), not on the GPU box:

    python tests/golden/make_golden.py

What runs from the reference (imported read-only from /root/reference, CPU only):
  * maxk_spgemm_function.MaxKSpGEMMFunction.forward -- with the kernels absent it
    takes its pure-PyTorch path (maxk_spgemm_function.py:96-128): torch.topk ->
    scatter -> torch.sparse.mm -> / in_degrees.  Called through a plain context
    object so autograd records those torch ops; .backward(G) then yields the
    true gradient of the reference forward w.r.t. the dense input (the
    reference's own backward, :132-184, raises ValueError -- SURVEY.md 3.2).
  * generate_meta_csc.generate_warp4_metadata (generate_meta_csc.py:14-93) for
    the warp4 schedule of every fixture graph.
The prebuilt maxk_cuda_kernels*.so that ships in the reference is never loaded:
sys.modules is primed so that `import maxk_cuda_kernels` raises ImportError.

asym_outdeg_d256_k16 additionally pins the v1 backward's divisor on a graph whose in- and
out-degrees differ: `grad_cbsr_refrule` is the gradient the reference's
hand-written backward intends -- grad_output / out_degrees through the A^T product, no
in-degree division (maxk_spgemm_function.py:154-175) -- obtained by autograd through the
reference forward called without in_degrees and fed G / out_degrees; `grad_cbsr_ref` stays the
exact adjoint of the normalised forward.

Fixtures hold data only: inputs (CSR, edge weights, features, degrees, upstream
grad) and the reference's outputs.  Inputs are continuous random values, so
torch.topk has no ties and index vectors are well defined.
"""
from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


class _Ctx:
    """Stand-in for the autograd ctx so forward() runs as plain torch ops."""

    def save_for_backward(self, *tensors):
        self.saved_tensors = tensors


def _import_reference():
    sys.modules["maxk_cuda_kernels"] = None  # never load the shipped CUDA binary
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import maxk_spgemm_function as ref_fn  # noqa: E402
        import generate_meta_csc as ref_meta  # noqa: E402
    assert ref_fn.MAXK_KERNELS_AVAILABLE is False
    return ref_fn, ref_meta


def make_graph(rng, V, avg_deg, symmetric, self_loops, hub_rows=(), empty_rows=0):
    """Random CSR (sorted, deduplicated).  hub_rows: list of (row, degree)."""
    m = int(V * avg_deg / (2 if symmetric else 1))
    src = rng.integers(0, V, m)
    dst = rng.integers(0, V, m)
    if symmetric:
        src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
    for r, d in hub_rows:
        nb = rng.choice(V, size=min(d, V), replace=False)
        src = np.concatenate([src, np.full(nb.size, r)])
        dst = np.concatenate([dst, nb])
        if symmetric:
            src, dst = np.concatenate([src, nb]), np.concatenate([dst, np.full(nb.size, r)])
    if self_loops:
        src = np.concatenate([src, np.arange(V)])
        dst = np.concatenate([dst, np.arange(V)])
    if empty_rows:
        drop = rng.choice(V, size=empty_rows, replace=False)
        keep = ~np.isin(src, drop)
        if symmetric:
            keep &= ~np.isin(dst, drop)
        src, dst = src[keep], dst[keep]
    key = np.unique(src.astype(np.int64) * V + dst)
    src, dst = key // V, key % V
    row_ptr = np.zeros(V + 1, dtype=np.int64)
    np.cumsum(np.bincount(src, minlength=V), out=row_ptr[1:])
    return row_ptr.astype(np.int32), dst.astype(np.int32)


CASES = [
    # name,          V,    avg, sym,   loops, hubs,                      empty, D,   k
    ("sym_d64_k16",   300,  10,  True,  True,  (),                        0,     64,  16),
    ("sym_d256_k8",   500,  24,  True,  True,  ((7, 300),),               0,     256, 8),
    ("sym_d256_k16",  700,  40,  True,  True,  ((3, 650), (11, 130)),     0,     256, 16),
    ("asym_d256_k32", 600,  20,  False, False, ((5, 560), (17, 100)),     25,    256, 32),
    ("asym_d256_k64", 400,  30,  False, True,  ((9, 390),),               10,    256, 64),
    ("flickr_d64_k16", 1500, 11, True,  True,  ((0, 500),),               0,     64,  16),
    ("odd_d100_k10",  257,  9,   False, False, ((1, 200),),               7,     100, 10),
    ("tiny_d64_k4",   40,   3,   True,  False, (),                        5,     64,  4),
    ("asym_outdeg_d256_k16", 500, 16, False, True, ((2, 450), (33, 120)),   12,    256, 16),
]
OUTDEG = {"asym_outdeg_d256_k16"}


def gen_case(ref_fn, ref_meta, name, V, avg, sym, loops, hubs, empty, D, k, seed):  # noqa: C901
    rng = np.random.default_rng(seed)
    row_ptr, col_idx = make_graph(rng, V, avg, sym, loops, hubs, empty)
    E = col_idx.size
    val = rng.random(E, dtype=np.float32)
    x = rng.standard_normal((V, D), dtype=np.float32)
    g = rng.standard_normal((V, D), dtype=np.float32)
    deg = np.maximum(np.diff(row_ptr), 1).astype(np.float32)

    t_indptr = torch.from_numpy(row_ptr.copy())
    t_idx = torch.from_numpy(col_idx.copy())
    t_val = torch.from_numpy(val.copy())
    t_x = torch.from_numpy(x.copy()).requires_grad_(True)
    t_deg = torch.from_numpy(deg.copy())
    with contextlib.redirect_stdout(io.StringIO()):
        y = ref_fn.MaxKSpGEMMFunction.forward(
            _Ctx(), t_idx, t_val, t_x, k, None, 0, t_indptr, t_deg, None, None, None)
    y.backward(torch.from_numpy(g.copy()))
    topv, topi = torch.topk(torch.from_numpy(x.copy()), k, dim=1)  # maxk_spgemm_function.py:53
    with contextlib.redirect_stdout(io.StringIO()):
        w4 = ref_meta.generate_warp4_metadata(col_idx, row_ptr, V, E, "CSR")
    sel = topi.numpy().astype(np.uint8)
    grad_x = t_x.grad.numpy()
    grad_cbsr = np.take_along_axis(grad_x, sel.astype(np.int64), axis=1)
    # the reference gradient is zero off the top-k positions, so the dense
    # gradient is fully described by grad_cbsr_ref + topk_idx (not stored twice)
    off = grad_x.copy()
    np.put_along_axis(off, sel.astype(np.int64), 0.0, axis=1)
    assert not off.any()
    out = dict(
        row_ptr=row_ptr, col_idx=col_idx, val=val, x=x, g=g, deg=deg,
        k=np.int32(k), D=np.int32(D),
        y_ref=y.detach().numpy(),
        topk_val=topv.numpy(), topk_idx=sel,
        grad_cbsr_ref=grad_cbsr,
        warp4_ref=np.asarray(w4, dtype=np.int32),
    )
    if name in OUTDEG:
        out_deg = np.maximum(np.bincount(col_idx, minlength=V), 1).astype(np.float32)
        assert not np.array_equal(out_deg, deg)
        t_x2 = torch.from_numpy(x.copy()).requires_grad_(True)
        with contextlib.redirect_stdout(io.StringIO()):
            y2 = ref_fn.MaxKSpGEMMFunction.forward(
                _Ctx(), t_idx, t_val, t_x2, k, None, 0, t_indptr, None, None, None, None)
        y2.backward(torch.from_numpy(g.copy()) / torch.from_numpy(out_deg).unsqueeze(-1))
        out["out_deg"] = out_deg
        out["grad_cbsr_refrule"] = np.take_along_axis(t_x2.grad.numpy(), sel.astype(np.int64),
                                                      axis=1)
    return out


def main(only=None):
    torch.manual_seed(0)
    ref_fn, ref_meta = _import_reference()
    for i, case in enumerate(CASES):
        name = case[0]
        if only and name not in only:
            continue
        data = gen_case(ref_fn, ref_meta, *case, seed=1000 + i)
        path = os.path.join(OUT, f"{name}.npz")
        np.savez_compressed(path, **data)
        print(f"{name}: V={data['row_ptr'].size - 1} E={data['col_idx'].size} "
              f"D={int(data['D'])} k={int(data['k'])} W={data['warp4_ref'].size // 4} -> {path}")


if __name__ == "__main__":
    main(set(sys.argv[1:]))  # optional case names: regenerate only those
