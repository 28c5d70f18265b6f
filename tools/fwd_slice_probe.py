"""Probe, not product: how fast would the forward SpGEMM run if every XCD's record gathers hit
its own L2?  Times the forward on the Reddit-sized graph with every column folded into a
window of W vertices (col % W: W records of 128 B; W = 29k is one XCD's 4 MB L2), and the
cost of summing 8 per-XCD partial outputs [V, D] (the price of pinning a column slice to each
XCD).  python tools/fwd_slice_probe.py [--graph reddit] [--k 16]"""
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
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.make_graph(P["V"], P["E"], P["alpha"], P["i0"], 1, dev)
V, E, D, k = row_ptr.numel() - 1, col.numel(), P["D"], a.k
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, device=dev, generator=g)
x = torch.rand(V, D, device=dev, generator=g)
cv, ci = mk.topk_cbsr(x, k)
y = torch.empty(V, D, device=dev)


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


for W in (V, V // 2, V // 4, V // 8, V // 16, V // 64):
    c2 = (col % W).contiguous() if W < V else col
    ms = t(lambda: mk.spgemm_forward(row_ptr, c2, val, cv, ci, D, out=y, validate=False))
    print(f"{a.graph} k={k} forward, columns in a window of {W:7d} vertices "
          f"({W * 128 / 2**20:6.1f} MiB of records): {ms:.3f} ms", flush=True)
    del c2
# the forward as P launches over column ranges (each launch: the edges whose column lies in
# its range, a sub-CSR), so each launch's records are 1/P of the table
deg_all = torch.diff(row_ptr)
rows = torch.repeat_interleave(torch.arange(V, device=dev), deg_all.long())
for P in (2, 4):
    subs = []
    for j in range(P):
        lo, hi = V * j // P, V * (j + 1) // P
        m = (col >= lo) & (col < hi)
        cnt = torch.bincount(rows[m], minlength=V)
        rp = torch.zeros(V + 1, dtype=torch.int32, device=dev)
        rp[1:] = torch.cumsum(cnt, 0).to(torch.int32)
        subs.append((rp, col[m].contiguous(), val[m].contiguous()))
    tot = 0.0
    for j, (rp, c2, v2) in enumerate(subs):
        ms = t(lambda: mk.spgemm_forward(rp, c2, v2, cv, ci, D, out=y, validate=False))
        tot += ms
        print(f"  column part {j}/{P}: {c2.numel()} edges {ms:.3f} ms", flush=True)
    print(f"{a.graph} k={k} forward as {P} column-range launches: {tot:.3f} ms "
          f"(+ {P - 1} read-modify-writes of the output)", flush=True)
    del subs
del rows
parts = torch.rand(8, V, D, device=dev)
ms = t(lambda: torch.sum(parts, 0, out=y))
print(f"sum of 8 partials [{V}, {D}] -> [{V}, {D}]: {ms:.3f} ms "
      f"({9 * V * D * 4 / ms / 1e6:.0f} GB/s)")
ms = t(lambda: parts.fill_(1.0))
print(f"write of 8 partials: {ms:.3f} ms ({8 * V * D * 4 / ms / 1e6:.0f} GB/s)")
