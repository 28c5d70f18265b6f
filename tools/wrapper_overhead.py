"""Probe, not product: host time of the Python surfaces per call on a small graph preset, beside
the GPU time of the same calls.  Host: `n` calls enqueued back to back (no synchronisation
inside), wall time / n.  GPU: HIP events around the same n calls.  Per call with a sync
(the kernel test's recipe): median of n event pairs around one call each.
    python tools/wrapper_overhead.py [--graph flickr] [--k 16] [--n 300]"""
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
ap.add_argument("--graph", default="flickr")
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--n", type=int, default=300)
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.make_graph(P["V"], P["E"], P["alpha"], P["i0"], 1, dev)
V, E, D, k = row_ptr.numel() - 1, col.numel(), P["D"], a.k
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, device=dev, generator=g)
x = torch.rand(V, D, device=dev, generator=g)
G = torch.rand(V, D, device=dev, generator=g)
div = torch.clamp(torch.diff(row_ptr).float(), min=1.0)
cv, ci = mk.topk_cbsr(x, k)
out = torch.empty(V, D, device=dev)
gs = torch.empty(V, k, device=dev)

calls = {
    "topk_cbsr": lambda: mk.topk_cbsr(x, k),
    "spgemm_forward": lambda: mk.spgemm_forward(row_ptr, col, val, cv, ci, D, row_div=div, out=out),
    "sspmm_backward": lambda: mk.sspmm_backward(row_ptr, col, val, G, ci, row_div=div, out=gs),
}
for name, f in calls.items():
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(a.n):
        f()
    e.record()
    host = (time.perf_counter() - t0) / a.n * 1e3
    torch.cuda.synchronize()
    gpu = s.elapsed_time(e) / a.n
    ts = []
    for _ in range(a.n):
        s1, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s1.record()
        f()
        e1.record()
        e1.synchronize()
        ts.append(s1.elapsed_time(e1))
    ts.sort()
    print(f"{a.graph} k={k} {name:15s} host {host:.4f} ms/call  back-to-back GPU {gpu:.4f} "
          f"ms/call  synced per call {ts[len(ts) // 2]:.4f} ms")
