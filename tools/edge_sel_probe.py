"""Probe, not product: the csc backward with per-edge selectors (maxk_sspmm_backward_csc_sel)
against the selector-table form on a synthetic preset graph; checks they agree and times
phase 1 + 2 per call (HIP events), plus the gather that builds the stream.
    python tools/edge_sel_probe.py [--graph products] [--k 8 16 32]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="products")
ap.add_argument("--k", type=int, nargs="*", default=[8, 16, 32])
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E, D = row_ptr.numel() - 1, col.numel(), P["D"]
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, generator=g, device=dev)
X = torch.rand(V, D, generator=g, device=dev)
G = torch.rand(V, D, generator=g, device=dev)
plan = mk.transpose_plan(col, V)


def t(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters


for k in a.k:
    cv, ci = mk.topk_cbsr(X, k)
    out = torch.empty(V, k, device=dev)
    es = mk.edge_selectors(col, ci)
    ref = mk.sspmm_backward(row_ptr, col, val, G, ci, mode="csc", plan=plan).clone()
    got = mk.sspmm_backward(row_ptr, col, val, G, ci, mode="csc", plan=plan, out=out, edge_sel=es)
    same = torch.equal(got, ref)
    tc = t(lambda: mk.sspmm_backward(row_ptr, col, val, G, ci, mode="csc", plan=plan, out=out,
                                     validate=False))
    ts = t(lambda: mk.sspmm_backward(row_ptr, col, val, G, ci, mode="csc", plan=plan, out=out,
                                     validate=False, edge_sel=es))
    tg = t(lambda: mk.edge_selectors(col, ci, out=es))
    y = torch.empty(V, D, device=dev)
    es2 = torch.zeros_like(es)
    y_ref = mk.spgemm_forward(row_ptr, col, val, cv, ci, D).clone()
    mk.spgemm_forward(row_ptr, col, val, cv, ci, D, out=y, edge_sel_out=es2)
    emit_ok = torch.equal(es2, es) and bool(((y - y_ref).abs() <= 1e-5 * y_ref.abs().clamp(min=1)).all())
    tf = t(lambda: mk.spgemm_forward(row_ptr, col, val, cv, ci, D, out=y, validate=False))
    tfs = t(lambda: mk.spgemm_forward(row_ptr, col, val, cv, ci, D, out=y, validate=False,
                                      edge_sel_out=es2))
    print(f"{a.graph} k={k}: csc {tc:.3f} ms, csc + edge selectors {ts:.3f} ms (bitwise equal: "
          f"{same}); building the stream by a gather {tg:.3f} ms; forward {tf:.3f} ms, forward "
          f"emitting the stream {tfs:.3f} ms (stream and output equal: {emit_ok}); step "
          f"{tf + tc:.3f} -> {tfs + ts:.3f} ms", flush=True)
    del es, es2, out, y
