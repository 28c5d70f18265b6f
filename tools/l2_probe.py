"""Probe, not product: how fast would the Reddit-sized forward walk if each XCD's record gathers
hit its own L2?  Times the forward on the synthetic graph as it is and with its columns folded
into the first 1/F of the vertices (c -> c // F: rows keep their lengths and order, the record
table shrinks F times, so at F = 8 it is ~3.7 MB, under one XCD's 4 MB L2), and the plain
streaming of a [F, V, D] fp32 partial buffer (written, then read and summed) that a
column-blocked forward would add.
    python tools/l2_probe.py [--graph reddit] [--k 16]"""
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
a = ap.parse_args()
D = maxk_graph.PRESETS[a.graph]["D"]
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E = row_ptr.numel() - 1, col.numel()
g = torch.Generator(device="cuda").manual_seed(3)
val = torch.rand(E, generator=g, device="cuda")
cv, ci = mk.topk_cbsr(torch.rand(V, D, generator=g, device="cuda"), a.k)


def timed(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(a.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


out = torch.empty(V, D, device="cuda")
for F in (1, 2, 4, 8, 16):
    c = (col // F).contiguous()
    t = timed(lambda: mk.spgemm_forward(row_ptr, c, val, cv, ci, D, out=out, validate=False))
    print(f"{a.graph} V={V} E={E} k={a.k} columns folded by {F:2d} (table {V * 128 / F / 2**20:6.1f}"
          f" MB at 128 B/record): forward {t:.3f} ms")
for F in (2, 4, 8):
    part = torch.empty(F, V, D, device="cuda")
    t_w = timed(lambda: part.fill_(1.0))
    t_r = timed(lambda: torch.sum(part, 0, out=out))
    print(f"partials F={F}: write {t_w:.3f} ms, read + sum {t_r:.3f} ms ({F * V * D * 4 / 2**20:.0f} MB)")
