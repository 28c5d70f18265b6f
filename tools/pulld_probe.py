"""Probe, not product: the destination-grouped pull (maxk_exp_pulld, experimental entry of
libmaxk_hip.so) against the pull backward on a synthetic preset graph at k = 16: the pull plan's
tiles re-sorted by destination, 64 groups per tile cut at destination boundaries (plan built
here with torch), parity against mode "pull", and times (HIP events).
    python tools/pulld_probe.py [--graph reddit]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402
from maxk_cuda_kernels import _capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="reddit")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
k, NG = 16, 64
P = maxk_graph.PRESETS[a.graph]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E, D = row_ptr.numel() - 1, col.numel(), P["D"]
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, generator=g, device=dev)
X = torch.rand(V, D, generator=g, device=dev)
G = torch.rand(V, D, generator=g, device=dev)
cv, ci = mk.topk_cbsr(X, k)

tptr, ent, shift, S = mk.pull_plan(row_ptr, col, val, V, k, D)
B = 1 << shift
tiles = tptr.numel() - 1
cnt = torch.diff(tptr.long())
tile_of = torch.repeat_interleave(torch.arange(tiles, device=dev), cnt)
dst = (ent[:, 0].long() >> 16) & 0xffff
key = tile_of * 65536 + dst
perm = torch.sort(key, stable=True).indices
ent_d = ent[perm].contiguous()
key = key[perm]
seg_start = torch.nonzero(torch.cat([torch.ones(1, dtype=torch.bool, device=dev),
                                     key[1:] != key[:-1]])).flatten()
seg_start = torch.cat([seg_start, torch.tensor([E], device=dev)])
t0 = tptr[:-1].long()
tgt = t0[:, None] + (cnt[:, None] * torch.arange(NG + 1, device=dev)[None, :] + NG - 1) // NG
gi = torch.searchsorted(seg_start, tgt.flatten())
grp_e = seg_start[gi].view(tiles, NG + 1)
grp_e = torch.minimum(grp_e, tptr[1:].long()[:, None])
grp_e[:, 0] = t0
grp_e[:, NG] = tptr[1:].long()
dst_at = torch.cat([dst[perm], torch.zeros(1, dtype=torch.long, device=dev)])
grp_d = torch.where(grp_e < tptr[1:].long()[:, None], dst_at[grp_e.clamp(max=E)],
                    torch.full_like(grp_e, B))
grp_d[:, 0] = 0
grp_d[:, NG] = B
grp_e = grp_e.int().contiguous()
grp_d = grp_d.int().contiguous()
bal = torch.diff(grp_e.long(), dim=1)
print(f"{a.graph}: V={V} E={E} tiles={tiles} S={S} shift={shift}; entries per group mean "
      f"{bal.float().mean():.0f}, max per tile / mean per tile {bal.max(1).values.float().mean() / bal.float().mean():.2f}",
      flush=True)

L = _capi.load()
fn = L.maxk_exp_pulld
fn.restype = ctypes.c_int
P_ = ctypes.c_void_p
fn.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int32, ctypes.c_int32, P_, ctypes.c_int64,
               ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P_, ctypes.c_size_t, P_]
ws = torch.empty(tiles * k * B * 4 + 2 * ((V * k + 255) // 256 * 256), dtype=torch.uint8, device=dev)
out = torch.empty(V, k, device=dev)
ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def run(unroll):
    rc = fn(ptr(G), ptr(ci), ptr(grp_e), ptr(grp_d), ptr(ent_d), shift, S, ptr(out), V, V, D, k,
            unroll, ptr(ws), ws.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, L.maxk_last_error()
    return out


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


ref = mk.sspmm_backward(row_ptr, col, val, G, ci, mode="pull").clone()
for u in (4, 8):
    got = run(u).clone()
    err = ((got - ref).abs() / ref.abs().clamp(min=1)).max().item()
    print(f"  unroll {u}: max rel err vs pull {err:.2e}", flush=True)
tp = t(lambda: mk.sspmm_backward(row_ptr, col, val, G, ci, mode="pull", out=out, validate=False))
t4 = t(lambda: run(4))
t8 = t(lambda: run(8))
print(f"  pull {tp:.3f} ms; destination-grouped pull unroll 4 {t4:.3f} ms, unroll 8 {t8:.3f} ms",
      flush=True)
