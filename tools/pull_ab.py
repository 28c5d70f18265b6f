"""Probe, not product: the pull backward (no contribution rows) against the two-phase bucket
backward on a synthetic graph preset, for several row-slice counts.  Checks they agree with
the bucket result and prints per-call times (HIP events, `iters` calls after 3 warmups).
    python tools/pull_ab.py [--graph reddit] [--k 16] [--slices 32 64 128]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="reddit")
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--slices", type=int, nargs="*", default=[0, 32, 128])
ap.add_argument("--csc", action="store_true", help="also time the csc two-phase form")
ap.add_argument("--dim", type=int, default=None, help="feature width (default: the preset's)")
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.make_graph(P["V"], P["E"], P["alpha"], P["i0"], 1, dev)
V, E, D, k = row_ptr.numel() - 1, col.numel(), a.dim or P["D"], a.k
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, device=dev, generator=g)
x = torch.rand(V, D, device=dev, generator=g)
G = torch.rand(V, D, device=dev, generator=g)
div = torch.clamp(torch.diff(row_ptr).float(), min=1.0)
cv, ci = mk.topk_cbsr(x, k)


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


ref_mode = "csc"  # the reference form the pull is checked against
bplan = mk.transpose_plan(col, V)
out = torch.empty(V, k, device=dev)


def run(mode, plan):
    return mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=div, mode=mode, plan=plan,
                             out=out, validate=False)


ref = run(ref_mode, bplan).clone()
print(f"{a.graph} k={k} V={V} E={E}: {ref_mode} (two-phase) {t(lambda: run(ref_mode, bplan)):.3f} ms")
if a.csc and ref_mode != "csc":
    cplan = mk.transpose_plan(col, V)
    print(f"csc (two-phase) {t(lambda: run('csc', cplan)):.3f} ms")
    del cplan
for S in a.slices:
    plan = mk.pull_plan(row_ptr, col, val, V, k, D, slices=S or None, cache=False)
    got = run("pull", plan)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"pull S={plan[3]:4d}: {t(lambda: run('pull', plan)):.3f} ms  max rel err vs {ref_mode} "
          f"{err:.3e}")
