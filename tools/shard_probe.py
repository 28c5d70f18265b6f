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
ap.add_argument("--pipelines", type=int, nargs="*", default=[],
                help="also time the pipelined gather mode's column parts (maxk_dist PIPELINE)")
ap.add_argument("--chunks", type=int, nargs="*", default=[],
                help="also time rank 0's forward at these item sizes (0 = the automatic one)")
ap.add_argument("--records", action="store_true",
                help="forward over transport records (maxk_cbsr_records of the rank's own rows, "
                     "timed, + maxk_spgemm_forward_records of the gathered buffer)")
ap.add_argument("--busbw", type=float, nargs="*", default=[250.0, 375.0, 500.0],
                help="RCCL all-gather / reduce-scatter bus bandwidths (GB/s) for the step model")
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
        if a.records and mk.records_ok(sh.n_local, sh.n_cols, sh.col_idx.numel(), D, k):
            rec_all = mk.cbsr_records(cv_all, ci_all, D)  # what the all-gather would deliver
            own_v, own_i = cv[sh.v0:sh.v1].contiguous(), ci[sh.v0:sh.v1].contiguous()
            t_own = timed(lambda: mk.cbsr_records(own_v, own_i, D))
            y2 = torch.empty_like(y)
            t_walk = timed(lambda: mk.spgemm_forward_records(sh.row_ptr, sh.col_idx, sh.values,
                                                             rec_all, k, D, out=y2))
            same = bool(torch.equal(y, y2))
            if rank == 0:
                print(f"  N={world} rank 0 forward: packed {tf:.3f} ms, transport records "
                      f"{t_own:.3f} (own rows) + {t_walk:.3f} (walk) = {t_own + t_walk:.3f} ms, "
                      f"bitwise equal {same}", flush=True)
            assert same, "transport-record forward differs from the packed one"
            tf = t_own + t_walk
            del rec_all, y2
        if a.chunks and rank == 0:
            line = []
            for c in a.chunks:
                tc = timed(lambda: mk.spgemm_forward(sh.row_ptr, sh.col_idx, sh.values, cv_all,
                                                     ci_all, D, out=y, validate=False, chunk=c))
                line.append(f"{c}: {tc:.3f}")
            print(f"  N={world} rank 0 forward by item size (tokens: ms): " + ", ".join(line),
                  flush=True)
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


def step_model(parts_f, parts_b, ag_bytes, rs_bytes, world, busbw):
    """Step time (ms) of one rank: the forward's all-gathers queued back to back on the
    communicator's stream, part j's product after its all-gather (j > 0 accumulating); the
    backward's part j reduce-scatter after its backward, beside the next part's backward.
    ag_bytes / rs_bytes: one part's whole collective size; a collective moves (N-1)/N of it
    per rank at the bus bandwidth."""
    P = len(parts_f)
    a = ag_bytes * (world - 1) / world / (busbw * 1e6)
    r = rs_bytes * (world - 1) / world / (busbw * 1e6)
    t_ag = t_f = 0.0  # forward: end of the last all-gather and of the last product
    for j in range(P):
        t_ag += a
        t_f = max(t_f, t_ag) + parts_f[j]
    t_b = t_rs = 0.0  # backward
    for j in range(P):
        t_b += parts_b[j]
        t_rs = max(t_rs, t_b) + r
    return t_f + max(t_b, t_rs)


if a.pipelines:
    base_t = None
    for world in [w for w in a.worlds if w > 1]:
        for Pn in a.pipelines:
            worst = None
            for rank in range(world):
                sh = maxk_dist.ShardedMaxK(row_ptr, col, val, rank, world, device=dev,
                                           mode="gather", pipeline=Pn)
                cv, ci = mk.topk_cbsr(X, k)
                b, vh, Pr = sh.bounds, (sh.vh if sh.pipeline > 1 else sh.vmax), sh.pipeline
                gl = G[sh.v0:sh.v1].contiguous()
                y = torch.empty(sh.n_local, D, device=dev)
                tf, tb = [], []
                for j in range(Pr):
                    cvj = torch.zeros(world * vh, k, device=dev)
                    cij = torch.zeros(world * vh, k, dtype=torch.uint8, device=dev)
                    for p in range(world):
                        lo, hi = b[p] + j * vh, min(b[p] + (j + 1) * vh, b[p + 1])
                        if hi > lo:
                            cvj[p * vh:p * vh + hi - lo] = cv[lo:hi]
                            cij[p * vh:p * vh + hi - lo] = ci[lo:hi]
                    rp, cj, vj = sh.parts[j] if Pr > 1 else (sh.row_ptr, sh.col_idx, sh.values)
                    nc = sh.n_cols_part if Pr > 1 else sh.n_cols
                    if a.records and Pr > 1 and mk.records_ok(sh.n_local, nc, cj.numel(), D, k):
                        # maxk_dist's transport records: the owner's part rows packed before the
                        # all-gather (timed), the gathered part walked as it lands
                        recj = mk.cbsr_records(cvj, cij, D)
                        own_v = cvj[rank * vh:(rank + 1) * vh].contiguous()
                        own_i = cij[rank * vh:(rank + 1) * vh].contiguous()
                        t_own = timed(lambda: mk.cbsr_records(own_v, own_i, D))
                        tf.append(t_own + timed(lambda: mk.spgemm_forward_records(
                            rp, cj, vj, recj, k, D, out=y, accumulate=j > 0)))
                        del recj
                    else:
                        tf.append(timed(lambda: mk.spgemm_forward(rp, cj, vj, cvj, cij, D, out=y,
                                                                  validate=False,
                                                                  accumulate=j > 0)))
                    plan = sh.plan(k, D, j if Pr > 1 else None)
                    mode = mk._bwd_mode(None, k, cj.numel(), nc, sh.n_local, D, (rp, cj))
                    gs = torch.empty(nc, k, device=dev)
                    tb.append(timed(lambda: mk.sspmm_backward(rp, cj, vj, gl, cij, out=gs,
                                                              validate=False, mode=mode,
                                                              plan=plan)))
                    del cvj, cij, gs, plan
                ag, rs = world * vh * k * 5, world * vh * k * 4
                if worst is None or sum(tf) + sum(tb) > sum(worst[0]) + sum(worst[1]):
                    worst = (tf, tb, ag, rs, rank)
                del sh, gl, y
            tf, tb, ag, rs, rk = worst
            print(f"  N={world} pipeline {Pn}: slowest rank {rk}: fwd parts "
                  f"{' + '.join(f'{x:.3f}' for x in tf)}, bwd parts "
                  f"{' + '.join(f'{x:.3f}' for x in tb)} ms; per part all-gather {ag / 1e6:.1f} MB, "
                  f"reduce-scatter {rs / 1e6:.1f} MB", flush=True)
            for bw in a.busbw:
                t = step_model(tf, tb, ag, rs, world, bw)
                sp = f", {base / t:.2f}x over N=1" if base else ""
                print(f"     busbw {bw:.0f} GB/s: step {t:.3f} ms{sp}", flush=True)
