"""Probe, not product: where the host time of one binding call goes on a small graph.
cProfile over n back-to-back calls of spgemm_forward / sspmm_backward (Flickr-sized, D = 64),
then the raw C-ABI call with pre-built arguments for the floor.
    python tools/host_profile.py [--k 16] [--n 500]"""
import argparse
import cProfile
import ctypes
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--n", type=int, default=500)
a = ap.parse_args()
dev = torch.device("cuda")
rp, col = maxk_graph.synthetic_graph("flickr", device=dev)
V, E, D, k = rp.numel() - 1, col.numel(), 64, a.k
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, device=dev, generator=g)
x = torch.rand(V, D, device=dev, generator=g)
G = torch.rand(V, D, device=dev, generator=g)
cv, ci = mk.topk_cbsr(x, k)
out = torch.empty(V, D, device=dev)
gs = torch.empty(V, k, device=dev)
calls = {
    "spgemm_forward": lambda: mk.spgemm_forward(rp, col, val, cv, ci, D, out=out, validate=False),
    "sspmm_backward": lambda: mk.sspmm_backward(rp, col, val, G, ci, out=gs, validate=False),
}
for name, f in calls.items():
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.n):
        f()
    host = (time.perf_counter() - t0) / a.n * 1e6
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.n):
        f()
    pr.disable()
    torch.cuda.synchronize()
    print(f"== {name}: host {host:.1f} us/call")
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)
# the floor: the raw forward call with every argument built once
L = mk._lib()
ws_b = L.maxk_spgemm_forward_workspace_size(V, V, E, D, k, 0)
ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
args = [ctypes.c_void_p(t.data_ptr()) for t in (rp, col, val, cv, ci)] + [None] + \
    [ctypes.c_void_p(out.data_ptr()), V, V, E, D, k, 0, ctypes.c_void_p(ws.data_ptr()), ws_b,
     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)]
for _ in range(50):
    L.maxk_spgemm_forward(*args)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.n):
    L.maxk_spgemm_forward(*args)
print(f"== raw maxk_spgemm_forward: host {(time.perf_counter() - t0) / a.n * 1e6:.1f} us/call")
t0 = time.perf_counter()
for _ in range(a.n):
    torch.empty(ws_b, dtype=torch.uint8, device=dev)
print(f"== torch.empty(workspace): {(time.perf_counter() - t0) / a.n * 1e6:.1f} us/call")
t0 = time.perf_counter()
for _ in range(a.n):
    with torch.cuda.device(dev):
        pass
print(f"== with torch.cuda.device: {(time.perf_counter() - t0) / a.n * 1e6:.1f} us/call")
t0 = time.perf_counter()
for _ in range(a.n):
    torch.cuda.current_stream(dev).cuda_stream
print(f"== current_stream: {(time.perf_counter() - t0) / a.n * 1e6:.1f} us/call")
torch.cuda.synchronize()
