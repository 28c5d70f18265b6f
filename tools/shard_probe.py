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
ap.add_argument("--contention", action="store_true",
                help="pipelined mode: also time each part's kernels beside a paced copy on a "
                     "second stream that moves the overlapping collective's bytes at each --busbw "
                     "with --channels workgroups (tools/paced_copy.hip; r06, VERDICT r05 item 4)")
ap.add_argument("--channels", type=int, default=32,
                help="workgroups of the collective stand-in (RCCL: one per channel)")
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


_PACED = None


def paced_lib():
    """tools/probe_lib/libpaced_copy.so (build: see tools/paced_copy.hip)."""
    global _PACED
    if _PACED is None:
        import ctypes
        _PACED = ctypes.CDLL(os.path.join(ROOT, "tools", "probe_lib", "libpaced_copy.so"))
        _PACED.paced_copy.restype = ctypes.c_int
        _PACED.paced_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_void_p]
    return _PACED


_BUF = {}


def timed_beside(f, nbytes, reduce, gbps):
    """(ms of f, ms of the paced copy) with f on the current stream and a paced copy of nbytes
    (a reduce-copy reading two buffers when `reduce`) started with it on a second stream."""
    n = max(16, nbytes // 16 * 16)
    if _BUF.get("n", 0) < n:
        _BUF.clear()
        _BUF.update(n=n, src=torch.empty(n // 4, device=dev), src2=torch.empty(n // 4, device=dev),
                    dst=torch.empty(n // 4, device=dev), side=torch.cuda.Stream())
    side, cur = _BUF["side"], torch.cuda.current_stream()
    lib = paced_lib()
    tf = tc = 0.0
    for it in range(3 + a.iters):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(cur)
        side.wait_event(e0)
        rc = lib.paced_copy(_BUF["src"].data_ptr(), _BUF["src2"].data_ptr() if reduce else None,
                            _BUF["dst"].data_ptr(), n, a.channels, gbps, side.cuda_stream)
        assert rc == 0, rc
        f()
        e1.record(cur)
        e2.record(side)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        if it >= 3:
            tf += e0.elapsed_time(e1)
            tc += e0.elapsed_time(e2)
    return tf / a.iters, tc / a.iters


def step_model_c(tf, tfc, tb, tbc, a_ms, ac_ms, r_ms, rc_ms):
    """step_model with the contention measured: forward part j < P-1 runs beside all-gather j+1
    (tfc[j]; that all-gather takes ac_ms), backward part j > 0 beside reduce-scatter j-1 (tbc[j];
    rc_ms); the first all-gather and the last reduce-scatter run alone (a_ms, r_ms)."""
    P = len(tf)
    t_ag = t_f = 0.0
    for j in range(P):
        t_ag += ac_ms if j > 0 else a_ms
        t_f = max(t_f, t_ag) + (tfc[j] if j < P - 1 else tf[j])
    t_b = t_rs = 0.0
    for j in range(P):
        t_b += tbc[j] if j > 0 else tb[j]
        t_rs = max(t_rs, t_b) + (rc_ms if j < P - 1 else r_ms)
    return t_f + max(t_b, t_rs)


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
                tf, tb, cont = [], [], {}
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
                    def bwd_j():
                        mk.sspmm_backward(rp, cj, vj, gl, cij, out=gs, validate=False, mode=mode,
                                          plan=plan)
                    tb.append(timed(bwd_j))
                    if a.contention and Pr > 1:
                        # the collective beside this part: forward -- the next part's all-gather
                        # ((N-1)/N of world * vh * 5k bytes copied); backward -- the previous
                        # part's reduce-scatter ((N-1)/N of world * vh * 4k, read twice)
                        ag_b = world * vh * k * 5 * (world - 1) // world
                        rs_b = world * vh * k * 4 * (world - 1) // world
                        rec_fwd = a.records and mk.records_ok(sh.n_local, nc, cj.numel(), D, k)
                        if rec_fwd:
                            recj = mk.cbsr_records(cvj, cij, D)
                            fwd_j = lambda: mk.spgemm_forward_records(  # noqa: E731
                                rp, cj, vj, recj, k, D, out=y, accumulate=j > 0)
                        else:
                            fwd_j = lambda: mk.spgemm_forward(  # noqa: E731
                                rp, cj, vj, cvj, cij, D, out=y, validate=False, accumulate=j > 0)
                        for bw in a.busbw:
                            cont.setdefault(bw, {"f": [], "b": [], "ag": [], "rs": []})
                            f_ms, ag_ms = timed_beside(fwd_j, ag_b, False, bw)
                            b_ms, rs_ms = timed_beside(bwd_j, rs_b, True, bw)
                            cont[bw]["f"].append(f_ms)
                            cont[bw]["b"].append(b_ms)
                            cont[bw]["ag"].append(ag_ms)
                            cont[bw]["rs"].append(rs_ms)
                        if rec_fwd:
                            del recj
                    del cvj, cij, gs, plan
                ag, rs = world * vh * k * 5, world * vh * k * 4
                if worst is None or sum(tf) + sum(tb) > sum(worst[0]) + sum(worst[1]):
                    worst = (tf, tb, ag, rs, rank, cont)
                del sh, gl, y
            tf, tb, ag, rs, rk, cont = worst
            print(f"  N={world} pipeline {Pn}: slowest rank {rk}: fwd parts "
                  f"{' + '.join(f'{x:.3f}' for x in tf)}, bwd parts "
                  f"{' + '.join(f'{x:.3f}' for x in tb)} ms; per part all-gather {ag / 1e6:.1f} MB, "
                  f"reduce-scatter {rs / 1e6:.1f} MB", flush=True)
            for bw in a.busbw:
                t = step_model(tf, tb, ag, rs, world, bw)
                sp = f", {base / t:.2f}x over N=1" if base else ""
                print(f"     busbw {bw:.0f} GB/s: step {t:.3f} ms{sp}", flush=True)
                if bw in cont:
                    c = cont[bw]
                    a_nom = ag * (world - 1) / world / (bw * 1e6)
                    r_nom = rs * (world - 1) / world / (bw * 1e6)
                    ac, rc = max(c["ag"]), max(c["rs"])
                    tc = step_model_c(tf, c["f"], tb, c["b"], a_nom, max(a_nom, ac), r_nom,
                                      max(r_nom, rc))
                    spc = f", {base / tc:.2f}x over N=1" if base else ""
                    print(f"       with contention ({a.channels} channels): fwd parts "
                          f"{' + '.join(f'{x:.3f}' for x in c['f'])} (alone "
                          f"{' + '.join(f'{x:.3f}' for x in tf)}), bwd parts "
                          f"{' + '.join(f'{x:.3f}' for x in c['b'])} (alone "
                          f"{' + '.join(f'{x:.3f}' for x in tb)}); stand-in all-gather "
                          f"{ac:.3f} ms (nominal {a_nom:.3f}), reduce-scatter {rc:.3f} ms "
                          f"(nominal {r_nom:.3f}); step {tc:.3f} ms{spc}", flush=True)
