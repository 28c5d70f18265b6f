"""Probe, not product: per-rank compute of the vertex-range shards at N = 2/4/8 on ONE GPU.

Builds each rank's shard exactly as maxk_dist.ShardedMaxK does in "gather" mode (no process
group is needed for that mode's setup), runs its local forward SpGEMM and backward SSpMM with
the HIP kernels on the gathered-size CBSR, and times them with HIP events.  The slowest rank
sets the step's compute time at N; with the exchange left out, T(1) / (N x max_rank T(N)) is the
compute-only ceiling of the scaling efficiency.
    python tools/shard_probe.py [--graph reddit] [--k 16] [--worlds 2 4 8]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_dist  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="reddit")
ap.add_argument("--k", type=int, default=None)
ap.add_argument("--worlds", type=int, nargs="*", default=[1, 2, 4, 8])
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--reorder", action="store_true", help="relabel by maxk_graph.locality_order")
a = ap.parse_args()
P = maxk_graph.PRESETS[a.graph]
k = a.k or P["k"]
D = P["D"]
dev = torch.device("cuda")
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
if a.reorder:
    row_ptr, col, _ = maxk_graph.permute_graph(row_ptr, col,
                                               maxk_graph.locality_order(row_ptr, col))
V, E = row_ptr.numel() - 1, col.numel()
g = torch.Generator(device=dev).manual_seed(123)
val = torch.rand(E, generator=g, device=dev)
X = torch.rand(V, D, generator=g, device=dev)
G = torch.rand(V, D, generator=g, device=dev)


def timed(f):
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


print(f"{a.graph} V={V} E={E} D={D} k={k}: per-rank compute (fwd + bwd ms), slowest rank")
base = None
for world in a.worlds:
    worst = (0.0, 0.0, 0.0, -1, None)
    for rank in range(world):
        sh = maxk_dist.ShardedMaxK(row_ptr, col, val, rank, world, device=dev, mode="gather")
        cv, ci = mk.topk_cbsr(X, k)  # the gathered CBSR: every vertex's rows, padded layout
        cv_all = torch.zeros(sh.n_cols, k, device=dev)
        ci_all = torch.zeros(sh.n_cols, k, dtype=torch.uint8, device=dev)
        b = sh.bounds
        for p in range(world):
            cv_all[p * sh.vmax:p * sh.vmax + b[p + 1] - b[p]] = cv[b[p]:b[p + 1]]
            ci_all[p * sh.vmax:p * sh.vmax + b[p + 1] - b[p]] = ci[b[p]:b[p + 1]]
        gl = G[sh.v0:sh.v1].contiguous()
        y = torch.empty(sh.n_local, D, device=dev)
        gs = torch.empty(sh.n_cols, k, device=dev)
        plan = sh.plan(k, D)
        mode = mk._bwd_mode(None, k, sh.col_idx.numel(), sh.n_cols, sh.n_local, D,
                            (sh.row_ptr, sh.col_idx))
        tf = timed(lambda: mk.spgemm_forward(sh.row_ptr, sh.col_idx, sh.values, cv_all, ci_all, D,
                                             out=y, validate=False))
        tb = timed(lambda: mk.sspmm_backward(sh.row_ptr, sh.col_idx, sh.values, gl, ci_all,
                                             out=gs, validate=False, mode=mode, plan=plan))
        if tf + tb > worst[0] + worst[1]:
            worst = (tf, tb, sh.col_idx.numel(), rank, mode)
        del sh, plan, cv_all, ci_all, gl, y, gs
    t = worst[0] + worst[1]
    base = t if world == 1 else base
    eff = f"  compute-only efficiency {base / (world * t):.2f}" if base and world > 1 else ""
    print(f"  N={world}: rank {worst[3]} fwd {worst[0]:.3f} + bwd {worst[1]:.3f} = {t:.3f} ms "
          f"({worst[2]} edges, bwd {worst[4]}){eff}", flush=True)
