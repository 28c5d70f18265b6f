"""Probe, not product: how often the fp64-LDS-atomic backward modes differ between runs.

pull / hybrid / bsort / bucket add fp32 products into fp64 LDS accumulators in whatever order
the atomics land, then round once to fp32; two runs can differ only where the fp64 sums
differ in their last bits AND that difference crosses an fp32 rounding boundary.  This runs the
backward R times on one input and counts the elements (and runs) that are not bitwise equal to
the first run.
    python tools/repeat_probe.py [--graph reddit] [--k 16] [--mode pull] [--runs 50]"""
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
ap.add_argument("--k", type=int, default=None)
ap.add_argument("--mode", default="pull")
ap.add_argument("--runs", type=int, default=50)
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
k, D = a.k or P["k"], P["D"]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E = row_ptr.numel() - 1, col.numel()
g = torch.Generator(device=dev).manual_seed(7)
val = torch.rand(E, generator=g, device=dev)
G = torch.randn(V, D, generator=g, device=dev)  # signed: cancellation makes ties likelier
_, ci = mk.topk_cbsr(torch.randn(V, D, generator=g, device=dev), k)
deg = torch.diff(row_ptr).float().clamp(min=1)
plan = mk.backward_plan(col, V, k, a.mode, indptr=row_ptr, values=val, dim=D)
ref = mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=deg, mode=a.mode, plan=plan,
                        validate=False)
bad_runs, bad_elems, max_ulp = 0, 0, 0
out = torch.empty_like(ref)
for _ in range(a.runs):
    mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=deg, mode=a.mode, plan=plan, out=out,
                      validate=False)
    diff = out.view(torch.int32) != ref.view(torch.int32)
    n = int(diff.sum())
    if n:
        bad_runs += 1
        bad_elems += n
        ulp = (out.view(torch.int32)[diff] - ref.view(torch.int32)[diff]).abs().max()
        max_ulp = max(max_ulp, int(ulp))
print(f"{a.graph} V={V} E={E} D={D} k={k} mode {a.mode}: {a.runs} runs against the first, "
      f"{bad_runs} runs differ, {bad_elems} elements of {ref.numel() * a.runs} in all, "
      f"largest difference {max_ulp} ulp")
