"""Probe, not product: the window-sorted backward (mode "bsort") against csc on a
synthetic preset graph, with and without the per-edge selector stream; checks bsort against
csc and times each whole call (HIP events).  Run under rocprofv3 --kernel-trace --stats for
the phase split.
    python tools/bsort_probe.py [--graph products] [--k 4 8 16]"""
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
ap.add_argument("--k", type=int, nargs="*", default=[4, 8, 16])
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
div = torch.clamp(torch.diff(row_ptr).float(), min=1)
tplan = mk.transpose_plan(col, V)


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
    bplan = mk.bsort_plan(row_ptr, col, V, k)
    ref = mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=div, mode="csc", plan=tplan).clone()
    got = mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=div, mode="bsort", plan=bplan,
                            edge_sel=es).clone()
    err = ((got - ref).abs() / ref.abs().clamp(min=1)).max().item()
    r = {}
    for name, mode, plan, sel in (("csc", "csc", tplan, None), ("csc+stream", "csc", tplan, es),
                                  ("bsort", "bsort", bplan, None),
                                  ("bsort+stream", "bsort", bplan, es)):
        r[name] = t(lambda: mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=div, mode=mode,
                                              plan=plan, out=out, validate=False, edge_sel=sel))
    print(f"{a.graph} k={k} (W={mk._lib().maxk_bsort_window(k)}): "
          + ", ".join(f"{n} {v:.3f} ms" for n, v in r.items())
          + f"; bsort+stream vs csc max rel err {err:.2e}", flush=True)
    del es, bplan, out
