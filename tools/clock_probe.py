"""Probe, not product: the ogbn-products-sized csc backward (k = 32) in a timed loop of about
`--seconds`, for sampling the box's clocks beside it (tools/session.sh step `spread`: rocm-smi
from the shell every second while this runs) -- r06, VERDICT r05 item 3: which phase moves
between boxes, and with which clock.  Prints the per-call backward time of every second of the
loop (HIP events) so the shell's clock samples line up with it.
    python tools/clock_probe.py [--seconds 12] [--k 32]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=12.0)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--graph", default="products")
a = ap.parse_args()
dev = torch.device("cuda")
P = maxk_graph.PRESETS[a.graph]
D, k = P["D"], a.k
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E = row_ptr.numel() - 1, col.numel()
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, generator=g, device=dev)
X = torch.rand(V, D, generator=g, device=dev)
G = torch.rand(V, D, generator=g, device=dev)
cv, ci = mk.topk_cbsr(X, k)
mode = mk._bwd_mode(None, k, E, V, V, D, (row_ptr, col))
plan = mk.backward_plan(col, V, k, mode, indptr=row_ptr, values=val, dim=D)
out = torch.empty(V, k, device=dev)
y = torch.empty(V, D, device=dev)


def bwd():
    mk.sspmm_backward(row_ptr, col, val, G, ci, out=out, validate=False, mode=mode, plan=plan)


def fwd():
    mk.spgemm_forward(row_ptr, col, val, cv, ci, D, out=y, validate=False)


for _ in range(5):
    fwd()
    bwd()
torch.cuda.synchronize()
print(f"[clock_probe] {a.graph} V={V} E={E} k={k} bwd {mode}: loop start {time.time():.3f}",
      flush=True)
t_end = time.time() + a.seconds
sec = 0
while time.time() < t_end:
    evs = []
    t0 = time.time()
    while time.time() - t0 < 1.0:
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        fwd()
        e[1].record()
        bwd()
        e[2].record()
        evs.append(e)
        torch.cuda.synchronize()
    f = sorted(x[0].elapsed_time(x[1]) for x in evs)
    b = sorted(x[1].elapsed_time(x[2]) for x in evs)
    print(f"[clock_probe] t={time.time():.3f} second {sec}: {len(evs)} steps, fwd median "
          f"{f[len(f) // 2]:.3f} ms, bwd median {b[len(b) // 2]:.3f} ms", flush=True)
    sec += 1
