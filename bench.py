#!/usr/bin/env python3
"""Benchmark of the MaxK-GNN aggregation hot path on MI355X.

One step = forward SpGEMM (CSR adjacency x CBSR top-k features -> dense) +
backward SSpMM (dense grad -> CBSR-shaped grad) over the whole graph, the two
kernels the reference times in kernels/main.cu:163-172.

Metric (BASELINE.json): SpGEMM+SSpMM GTEPS = 2E / (t_fwd + t_bwd) / 1e9,
whole job, inputs resident in HBM before the timed region.  Default workload:
synthetic Reddit-sized graph (V=232,965, E=114,615,891, symmetric power-law with
self loops), hidden D=256, k=16 -- BASELINE.json configs[1] at k=16.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--graph reddit] [--k 16]

N > 1, one rank per GPU: vertex-range shards balanced by nnz; per step an RCCL
all-gather of the CBSR rows before the forward and a reduce-scatter of the
CBSR-gradient partials after the backward (strong scaling: the graph is fixed).
Rank 0 prints ONE JSON line.  Launched either by torch.distributed.run
(WORLD_SIZE set: this process is one rank) or directly -- `python bench.py
--gpus N` with no WORLD_SIZE starts N ranks itself (launch_ranks: a child
torch.distributed.run on 127.0.0.1, before this process touches the GPU) and
exits with their status.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_graph  # noqa: E402

warnings.filterwarnings("ignore", message="Sparse CSR tensor support")
METRIC = "SpGEMM+SSpMM GTEPS (edges/s) & HBM-BW% on Reddit h=256 k=16; vs CPU SpMM"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# The ceilings that bind a gather kernel before HBM does (roofline.binding):
# - random lines served by the Infinity Cache: 8.6 TB/s chip-wide (MI355X_MICROARCH.md,
#   "Indexed rows: gather into LDS", 38 MB table, uniformly random rows), against the measured
#   L2 -> fabric bytes (PMC FETCH_SIZE x2 + WRITE_SIZE; they include Infinity-Cache hits);
# - the texture path's tag lookups: about one per CU-cycle (tools/ta_probe.hip),
#   256 CUs x 2.4 GHz (the part's max clock, MI355X_MICROARCH.md), against the measured
#   TCP_TOTAL_CACHE_ACCESSES per launch.
IC_GATHER_GBS = 8600.0
TAG_RATE_PER_S = 256 * 2.4e9

# kernels making up each op of one step (rocprofv3 names, maxk:: namespace)
OP_KERNELS = {
    # the record route (packed or, k in [24, 32] on sparse graphs, transport records), or
    # (k >= D / 2, D <= 128) the dense route (dense_route.hip)
    "spgemm_forward": ["spgemm_fwd_kernel", "slab_fixup_kernel<0>", "cbsr_pack4_kernel",
                       "cbsr_pack_kernel", "cbsr_records_kernel", "cbsr_dense_kernel",
                       "dense_rows_kernel"],
    "sspmm_backward_csc": ["sspmm_bwd_kernel", "csc_sum_kernel", "slab_fixup_kernel<1>"],
    # k % 4 == 0: slot-ordered selectors, quantile-slot tiles; else pull_tile_kernel; plus
    # gprime_kernel when a row_div is given (the bench passes none)
    "sspmm_backward_pull": ["pull_q_kernel", "pull_reduce_kernel", "pull_sel4_kernel",
                            "pull_sel_kernel", "pull_tile_kernel", "gprime_kernel"],
    "sspmm_backward_bsort": ["bsort_push_kernel", "bucket_sum_kernel", "bucket_fixup_kernel"],
    "sspmm_backward_atomic": ["sspmm_bwd_kernel"],
    # dense rows with the selecting store (k >= D / 2), or selected columns per lane
    "sspmm_backward_dense": ["dense_select_rows_kernel", "dense_fixup_select_kernel",
                             "pick_rows_kernel", "slab_fixup_kernel<1>"],
    # csc over the sparse tiles' edges, then the pull over the dense ones, accumulating
    "sspmm_backward_hybrid": ["sspmm_bwd_kernel", "csc_sum_kernel", "slab_fixup_kernel<1>",
                              "pull_sel4_kernel", "pull_sel_kernel", "pull_q_kernel",
                              "pull_reduce_kernel", "gprime_kernel"],
}


def traffic_files():
    """profiles/rNN/traffic.json and profiles/rNN/final/traffic.json, newest first: the latest
    round, and within a round the final build's counters before the session's earlier ones
    (the BENCH line took an earlier r04 session's figure)."""
    import glob
    import re
    paths = glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "r*", "final", "traffic.json"))

    def order(p):
        rel = os.path.relpath(p, os.path.join(ROOT, "profiles")).split(os.sep)
        m = re.match(r"r(\d+)$", rel[0])
        return (int(m.group(1)) if m else -1, rel[1] == "final")
    return sorted(paths, key=order, reverse=True)


def load_traffic_record(key, op):
    """(record, path) of `op` on workload `key` from the newest traffic file holding it
    (tools/pmc_summary.py, from separate rocprofv3 --pmc passes of this same bench command):
    "bytes" = L2 -> fabric bytes per launch (FETCH_SIZE doubled per MI355X_MICROARCH.md, HBM,
    + WRITE_SIZE), and from r05 "tag_accesses" (TCP_TOTAL_CACHE_ACCESSES)."""
    for path in traffic_files():
        with open(path) as f:
            t = json.load(f)
        if key in t and op in t[key]:
            return t[key][op], os.path.relpath(path, ROOT)
    return None, None


def load_traffic(key, op):
    rec, path = load_traffic_record(key, op)
    return (rec["bytes"], path) if rec else (None, None)


def binding_roofline(t_ms, compulsory, rec):
    """The roofline against the ceiling that binds: the launch's floor is
    the largest of (a) its compulsory bytes at the HBM peak, (b) its measured fabric bytes at the
    Infinity Cache's random-line rate, (c) its measured tag accesses at the texture path's rate;
    `frac` = floor / measured time (<= 1 whenever the floor is one).  (b) and (c) come from
    counters (load_traffic_record); without them only (a) is known and `bound` says so."""
    terms = {"hbm_compulsory": compulsory / (HBM_PEAK_GBS * 1e9) * 1e3}
    if rec and rec.get("bytes"):
        terms["fabric_lines"] = rec["bytes"] / (IC_GATHER_GBS * 1e9) * 1e3
    if rec and rec.get("tag_accesses"):
        terms["tag_rate"] = rec["tag_accesses"] / TAG_RATE_PER_S * 1e3
    bound = max(terms, key=terms.get)
    out = {"bound": bound, "floor_ms": round(terms[bound], 4),
           "frac": round(terms[bound] / t_ms, 4),
           "terms_ms": {k: round(v, 4) for k, v in terms.items()},
           "ceilings": {"hbm_compulsory": f"{HBM_PEAK_GBS:.0f} GB/s (HBM peak)",
                        "fabric_lines": f"{IC_GATHER_GBS:.0f} GB/s (Infinity-Cache random lines)",
                        "tag_rate": f"{TAG_RATE_PER_S / 1e9:.1f} G tag accesses/s "
                                    "(1 per CU-cycle, 256 CUs, 2.4 GHz)"}}
    if rec and rec.get("tag_accesses"):
        out["tag_accesses"] = rec["tag_accesses"]
        out["tag_rate_G_per_s"] = round(rec["tag_accesses"] / (t_ms * 1e-3) / 1e9, 1)
    return out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def alg_bytes(V, E, D, k, Vc=None):
    """Algorithmic bytes per launch: row_ptr, col_idx+val, per-edge CBSR
    gather (k f32 + k u8), dense read/write once; bwd adds the [V,k] gradient write."""
    Vc = V if Vc is None else Vc
    fwd = 4 * (V + 1) + 8 * E + 5 * k * E + 4 * V * D
    bwd = fwd + 4 * Vc * k
    return fwd, bwd


def compulsory_bytes(V, E, D, k, Vc=None):
    """Bytes each op must move at least once (no re-reads): row_ptr, col_idx + val, the CBSR
    once (k f32 + k u8 per vertex; the backward reads only the selectors), the dense [V, D]
    output (forward) or input G (backward) once, and the [Vc, k] gradient write."""
    Vc = V if Vc is None else Vc
    fwd = 4 * (V + 1) + 8 * E + 5 * k * Vc + 4 * V * D
    bwd = 4 * (V + 1) + 8 * E + k * Vc + 4 * V * D + 4 * Vc * k
    return fwd, bwd


# --------------------------------------------------------------------------- CPU baseline
def reference_cpu_path(row_ptr, col, val, cv, ci, G, D, deg, target_s=12.0):
    """The reference's own CPU path for one MaxK aggregation, forward + backward, restated in
    torch (maxk_spgemm_function.py:96-125 with MAXK_KERNELS_AVAILABLE False, the path its CPU
    runs take): the top-k scattered into a dense [V, D] input, a coalesced COO adjacency,
    torch.sparse.mm, / in_degrees; the backward is autograd through that forward (the
    reference's hand-written backward raises), i.e. A^T (G / deg) gathered at
    the selectors.  On every host core this process is allotted, on a leading-row sample of
    the same graph sized for ~target_s seconds; the COO build (a Python loop over rows in the
    reference) is outside the timing.  Its per-call costs (the [V, D] scatter and input
    gradient) are measured on a one-row call and charged once to the whole graph: value =
    2E / (t_call + per_edge * E), per_edge from the sized sample (the sample rate
    alone charged them to 3 % of the edges).  `sample_value` keeps the sample's own rate."""
    rp = row_ptr.cpu().long()
    c, v = col.cpu().long(), val.cpu()
    V = rp.numel() - 1
    E = int(rp[-1])
    cvn, cin, Gn, dg = cv.cpu(), ci.cpu().long(), G.cpu(), deg.cpu().float().clamp(min=1)
    nt = host_cores()
    old_nt = torch.get_num_threads()
    torch.set_num_threads(nt)

    def run(r1):
        e1 = int(rp[r1])
        rows = torch.repeat_interleave(torch.arange(r1), torch.diff(rp[:r1 + 1]))
        A = torch.sparse_coo_tensor(torch.stack([rows, c[:e1]]), v[:e1], (r1, V)).coalesce()
        tv = cvn.clone().requires_grad_(True)
        t0 = time.perf_counter()
        xs = torch.zeros(V, D).scatter(1, cin, tv)
        out = torch.sparse.mm(A, xs) / dg[:r1].unsqueeze(-1)
        t1 = time.perf_counter()
        out.backward(Gn[:r1])
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, e1

    try:
        run(1)  # warm-up (allocator, thread pool)
        # the per-call costs that do not scale with the sample (the [V, D] scatter of the
        # top-k, the dense [V, D] input gradient), from the smallest sample, one row
        fix = sorted(run(1) for _ in range(3))[1]
        t_fix, e_fix = fix[0] + fix[1], fix[2]
        r_cal = max(1, int(np.searchsorted(rp.numpy(), E // 400)))
        tf0, tb0, e0 = run(r_cal)
        per_edge = max(1e-12, (tf0 + tb0 - t_fix) / max(1, e0 - e_fix))
        r1 = int(np.searchsorted(rp.numpy(), min(E, int(target_s / per_edge))))
        r1 = max(1, min(r1, V))
        tf, tb, es = run(r1)
    finally:
        torch.set_num_threads(old_nt)
    # a line t = fixed + slope * edges through the one-row sample and the sized one charges the
    # per-call costs once to the whole graph instead of once per sample
    t1 = tf + tb
    slope = max(0.0, (t1 - t_fix) / max(1, es - e_fix))
    t_full = t_fix + slope * (E - e_fix)
    return {"value": round(2 * E / t_full / 1e9, 6), "unit": "GTEPS", "cores": nt,
            "kind": "port",
            "sample": (f"reference CPU path (maxk_spgemm_function.py:96-125 + autograd backward: "
                       f"scatter, coalesced-COO torch.sparse.mm, /deg), {nt} threads, rows "
                       f"[0,{r1}) of the same graph = {es} of {E} edges ({100.0 * es / E:.1f}%); "
                       f"fwd {tf:.2f}s, bwd {tb:.2f}s; whole graph {t_full:.1f}s = "
                       f"{t_fix:.3f}s per call (a one-row call, {e_fix} edges) + "
                       f"{slope * 1e9:.2f}ns per edge"),
            "sample_value": round(2 * es / t1 / 1e9, 6)}


def cpu_baseline(row_ptr, col, val, cv, ci, G, D, target_s=12.0, deg=None):
    """The reference's CPU path (reference_cpu_path, the headline value), and beside it the
    oracle (the port of the reference kernels' semantics, 1 thread) on a row sample sized
    for ~target_s seconds of CPU work; returns the cpu_baseline JSON object."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.set_num_threads(1)
    rp = row_ptr.cpu().numpy()
    c, v = col.cpu().numpy(), val.cpu().numpy()
    cvn, cin, Gn = cv.cpu().numpy(), ci.cpu().numpy(), G.cpu().numpy()
    E = int(rp[-1])

    def run(r1):
        t0 = time.perf_counter()
        O.spgemm_fwd(rp, c, v, cvn, cin, D, rows=(0, r1))
        t1 = time.perf_counter()
        O.sspmm_bwd(rp, c, v, Gn, cin, rows=(0, r1))
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1

    # calibrate on ~1% of the edges, then size the sample
    r_cal = int(np.searchsorted(rp, E // 100))
    tf, tb = run(r_cal)
    per_edge = (tf + tb) / max(1, int(rp[r_cal]))
    e_s = min(E, int(target_s / per_edge))
    r1 = int(np.searchsorted(rp, e_s))
    r1 = max(1, min(r1, len(rp) - 1))
    tf, tb = run(r1)
    es = int(rp[r1])
    out = reference_cpu_path(row_ptr, col, val, cv, ci, G, D,
                             torch.diff(row_ptr) if deg is None else deg, target_s)
    out["oracle"] = {
        "value": round(2 * es / (tf + tb) / 1e9, 6), "unit": "GTEPS", "cores": 1, "kind": "port",
        "sample": (f"oracle/maxk_oracle.c fwd SpGEMM + bwd SSpMM (push), 1 thread, rows [0,{r1}) "
                   f"of the same graph = {es} of {E} edges ({100.0 * es / E:.1f}%); "
                   f"fwd {tf:.2f}s, bwd {tb:.2f}s"),
    }
    # the same port on every core this process is allotted (OpenMP), whole graph: forward over
    # rows, backward in its pull form over the transpose (a push needs atomics)
    import maxk_cuda_kernels as mk
    nt = host_cores()
    col_ptr, eid = mk.transpose_plan(col, len(rp) - 1)
    rows = torch.repeat_interleave(torch.arange(len(rp) - 1, device=col.device),
                                   torch.diff(row_ptr).long())
    t_ptr, t_src = col_ptr.cpu().numpy(), rows[eid.long()].int().cpu().numpy()
    t_val = val[eid.long()].cpu().numpy()
    del rows
    O.set_num_threads(nt)
    t0 = time.perf_counter()
    O.spgemm_fwd(rp, c, v, cvn, cin, D)
    t1 = time.perf_counter()
    O.sspmm_bwd_pull(t_ptr, t_src, t_val, Gn, cin)
    t2 = time.perf_counter()
    O.set_num_threads(1)
    out["oracle"]["multi_thread"] = {"value": round(2 * E / (t2 - t0) / 1e9, 6), "cores": nt,
                           "sample": f"whole graph, {nt} OpenMP threads (backward in pull form); "
                                     f"fwd {t1 - t0:.2f}s, bwd {t2 - t1:.2f}s"}
    out["host"] = host_info()
    return out


def host_cores() -> int:
    """Cores this process may use: OMP_NUM_THREADS when set (the GPU box allots each GPU 16
    of its host's CPUs and sets it to 16; nproc there shows the whole machine), else the
    affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)


def host_info():
    """The host the CPU baselines ran on (record nproc and the CPU model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cores_used": host_cores(),
            # the CPU baselines set torch to host_cores() threads for their timed calls and
            # restore the process default afterwards (torch_threads_default)
            "torch_threads_baselines": host_cores(),
            "torch_threads_default": torch.get_num_threads()}


def _order(row_ptr, col):
    """--reorder's vertex order: maxk_graph.locality_order, or by degree with
    MAXK_BENCH_ORDER=degree (a probe)."""
    if os.environ.get("MAXK_BENCH_ORDER") == "degree":
        return maxk_graph.degree_order(row_ptr)
    return maxk_graph.locality_order(row_ptr, col)


def cpu_spmm_baselines(row_ptr, col, val, dense, target_s=6.0):
    """The reference's CPU SpMM denominators: scipy.sparse CSR @ dense X^ on
    1 thread, and torch.sparse CSR mm on every host core this process is allotted
    (host_cores(), set for the call), each on a leading-row sample of
    the same graph sized for ~target_s seconds.  X^ = the scattered top-k input [V, D]."""
    import scipy.sparse as sp
    rp = row_ptr.cpu().numpy().astype(np.int64)
    c, v, X = col.cpu().numpy(), val.cpu().numpy(), dense.cpu().numpy()
    E = int(rp[-1])
    out = {}

    def sample_rows(time_fn):
        r = int(np.searchsorted(rp, max(1, E // 200)))
        r = max(1, min(r, len(rp) - 1))
        t = time_fn(r)
        per_edge = t / max(1, int(rp[r]))
        r1 = int(np.searchsorted(rp, min(E, int(target_s / per_edge))))
        r1 = max(1, min(r1, len(rp) - 1))
        return r1, time_fn(r1)

    def scipy_run(r1):
        A = sp.csr_matrix((v[:rp[r1]], c[:rp[r1]], rp[:r1 + 1]), shape=(r1, X.shape[0]))
        t0 = time.perf_counter()
        A @ X
        return time.perf_counter() - t0

    r1, t = sample_rows(scipy_run)
    out["cpu_spmm_scipy"] = {"value": round(int(rp[r1]) / t / 1e9, 6), "unit": "GTEPS (fwd SpMM)",
                             "cores": 1, "sample": f"rows [0,{r1}) = {int(rp[r1])} edges, {t:.2f}s"}
    Xt = torch.from_numpy(X)

    def torch_run(r1):
        A = torch.sparse_csr_tensor(torch.from_numpy(rp[:r1 + 1]), torch.from_numpy(c[:rp[r1]]).long(),
                                    torch.from_numpy(v[:rp[r1]]), (r1, X.shape[0]))
        t0 = time.perf_counter()
        A @ Xt
        return time.perf_counter() - t0

    nt, old_nt = host_cores(), torch.get_num_threads()
    torch.set_num_threads(nt)  # every core this process is allotted
    try:
        r1, t = sample_rows(torch_run)
    finally:
        torch.set_num_threads(old_nt)
    out["cpu_spmm_torch"] = {"value": round(int(rp[r1]) / t / 1e9, 6), "unit": "GTEPS (fwd SpMM)",
                             "cores": nt,
                             "sample": f"rows [0,{r1}) = {int(rp[r1])} edges, {t:.2f}s"}
    return out


# --------------------------------------------------------------------------- launcher
def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` without torch.distributed.run: start the
    N ranks as one child `python -m torch.distributed.run` on 127.0.0.1 and return its exit
    status.  This process only parses arguments and counts devices (torch.cuda.device_count()
    does not initialise HIP on this image): it makes no HIP call and never execs, so the ranks
    are fresh processes.  Rank 0's JSON line reaches the shared stdout unchanged.  With fewer
    visible GPUs than ranks the collectives are staged through the host (MAXK_DIST_BACKEND=gloo,
    the one-GPU rehearsal) unless the caller chose a backend."""
    import socket
    import subprocess
    env = dict(os.environ)
    ndev = torch.cuda.device_count()
    if ndev < n and "MAXK_DIST_BACKEND" not in env:
        env["MAXK_DIST_BACKEND"] = "gloo"
        log(f"[bench] {n} ranks on {ndev} visible GPU(s): gloo-staged collectives")
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *argv]
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=env)


# --------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)  # >= 10 warmup
    ap.add_argument("--graph", default="reddit", choices=sorted(maxk_graph.PRESETS))
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=0, help="tokens per work item (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rocsparse", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--bwd-mode", default="auto",
                    choices=["auto", "pull", "csc", "atomic", "hybrid", "bsort", "dense"])
    ap.add_argument("--graph-dir", default=None,
                    help="use <dir>/<graph>.indptr|.indices (the reference's files) when present")
    ap.add_argument("--no-cpu-spmm", action="store_true")
    ap.add_argument("--reorder", action="store_true",
                    help="relabel the graph once by maxk_graph.locality_order (communities "
                         "contiguous) before sharding and timing")
    ap.add_argument("--dist-pipeline", type=int, default=None,
                    help="N > 1, gather mode: column parts of the pipelined exchange (default: "
                         "maxk_dist's rule -- 2 when a rank's exchange is >= 64 MiB, else 1)")
    ap.add_argument("--edge-sel", default=None, choices=["auto", "0", "1"],
                    help="the forward's per-edge selector stream for a csc / bsort backward "
                         "(MAXK_EDGE_SEL: auto = k <= 16, 0 never, 1 always)")
    ap.add_argument("--dist-mode", default="auto", choices=["auto", "gather", "halo"],
                    help="N > 1: all-gather every CBSR row, or exchange only the halo rows "
                         "(auto: halo when every shard's halo is at most 60 %% of the vertices)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.edge_sel is not None:
        os.environ["MAXK_EDGE_SEL"] = args.edge_sel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MAXK_BENCH_STACKS=S: every rank logs its stages and dumps all thread stacks to stderr
    # after S seconds (diagnosing a multi-rank run that stops making progress)
    stacks_after = float(os.environ.get("MAXK_BENCH_STACKS", "0"))
    if stacks_after > 0:
        import faulthandler
        faulthandler.dump_traceback_later(stacks_after, exit=False)

    def stage(msg):
        if stacks_after > 0 or rank == 0:
            log(f"[bench] rank {rank}: {msg}")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # MAXK_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices, collectives
    # staged through host); the default is RCCL with one rank per GPU.
    backend = os.environ.get("MAXK_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()  # does not initialise HIP on this image
    if world > ndev:
        # ranks share a device (the gloo rehearsal): more than two processes with HIP's
        # default 4 hardware queues each stalled every rank's GPU work on the one-GPU box
        # (tools/share_probe.py: 4 processes hung > 150 s in make_graph, finished in 0.3 s
        # with GPU_MAX_HW_QUEUES=1), so each rank keeps one queue.  Set before HIP starts.
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
    dev_idx = local_rank % ndev if backend == "gloo" else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import maxk_cuda_kernels as mk
    build_cfg = mk._lib().maxk_build_config().decode()
    if build_cfg and "MAXK_HIP_LIB" not in os.environ:
        # the product library carries no tuning / ablation macros (tools/tune.sh variants are
        # selected with MAXK_HIP_LIB and say so in extra.build_config)
        raise SystemExit(f"libmaxk_hip.so was built with EXTRA_HIPFLAGS={build_cfg!r}; "
                         "rebuild it with `make -C spgemm-prunning_amd` before benchmarking")

    P = dict(maxk_graph.PRESETS[args.graph])
    D = args.dim or P["D"]
    k = args.k or P["k"]
    V = P["V"]
    t0 = time.time()
    gdir = maxk_graph.find_graph(args.graph, [args.graph_dir] if args.graph_dir else [])
    if gdir:
        V = maxk_graph.read_binary_array(
            os.path.join(gdir, f"{os.path.basename(args.graph)}.indptr")).size - 1

    def load_graph():
        if gdir:
            g = maxk_graph.GraphDataLoader(gdir).load_graph(args.graph)
            return (torch.from_numpy(g["indptr"]).to(dev), torch.from_numpy(g["indices"]).to(dev),
                    f"real graph {gdir}/{args.graph}.indptr|.indices; synthetic features")
        rp_, col_ = maxk_graph.synthetic_graph(args.graph, args.seed, dev)
        return rp_, col_, "synthetic"

    if world == 1:
        row_ptr, col, data = load_graph()
    else:
        # one rank loads (or builds) the graph and relabels it if asked, the others receive it
        # (one broadcast of row_ptr + col): every rank shards the same vertex order
        cdev = dev if backend == "nccl" else torch.device("cpu")
        if rank == 0:
            row_ptr, col, data = load_graph()
            if args.reorder:
                row_ptr, col, _ = maxk_graph.permute_graph(
                    row_ptr, col, _order(row_ptr, col))
            n_e = torch.tensor([col.numel()], dtype=torch.int64, device=cdev)
        else:
            n_e = torch.zeros(1, dtype=torch.int64, device=cdev)
        dist.broadcast(n_e, 0)
        if rank != 0:
            row_ptr = torch.empty(V + 1, dtype=torch.int32, device=dev)
            col = torch.empty(int(n_e), dtype=torch.int32, device=dev)
        for t in (row_ptr, col):
            if backend == "nccl":
                dist.broadcast(t, 0)
            else:
                h = t.cpu()
                dist.broadcast(h, 0)
                t.copy_(h)
        data = (f"real graph {gdir}/{args.graph}.indptr|.indices; synthetic features"
                if gdir else "synthetic") + " (loaded on rank 0, broadcast)"
    t_reorder = None
    if args.reorder:
        if world == 1:
            torch.cuda.synchronize()
            t_r = time.perf_counter()
            row_ptr, col, _ = maxk_graph.permute_graph(
                row_ptr, col, _order(row_ptr, col))
            torch.cuda.synchronize()
            t_reorder = time.perf_counter() - t_r
        data += "; vertex order by maxk_graph.locality_order (once per graph, untimed)"
    E = col.numel()
    gen = torch.Generator(device=dev).manual_seed(123)  # kernels/main.cu:74-77 seed
    val = torch.rand(E, generator=gen, device=dev)
    X = torch.rand(V, D, generator=gen, device=dev)
    G = torch.rand(V, D, generator=gen, device=dev)
    deg = torch.diff(row_ptr)
    if rank == 0:
        log(f"[bench] graph {args.graph}: V={V} E={E} max_deg={int(deg.max())} "
            f"avg_deg={E / V:.1f} gen {time.time() - t0:.1f}s")

    stage("graph and features ready")
    # ---- shard by vertex range, balanced by nnz (maxk_dist: the module the gloo tests cover)
    if world > 1:
        import maxk_dist
        shard = maxk_dist.ShardedMaxK(row_ptr, col, val, rank, world, device=dev,
                                      mode=args.dist_mode, k=k,
                                      pipeline=args.dist_pipeline)
        v0, v1, vmax, n_cols = shard.v0, shard.v1, shard.vmax, shard.n_cols
        l_row_ptr, l_col, l_val = shard.row_ptr, shard.col_idx, shard.values
        l_X = X[v0:v1]
        l_G = G[v0:v1].contiguous()
    else:
        v0, v1, vmax = 0, V, V
        l_row_ptr, l_col, l_val, l_X, l_G, n_cols = row_ptr, col, val, X, G, V
    nl = v1 - v0
    El = l_col.numel()

    # ---- CBSR of the local rows (the MaxK encode), padded to vmax rows for the collectives
    cv_loc = torch.zeros(vmax, k, device=dev)
    ci_loc = torch.zeros(vmax, k, dtype=torch.uint8, device=dev)
    cv_loc[:nl], ci_loc[:nl] = mk.topk_cbsr(l_X, k)
    if world > 1:
        # one all-gather of values + selectors per step (ShardedMaxK.gather_cbsr)
        cv_all, ci_all = shard.gather_cbsr(cv_loc[:nl], ci_loc[:nl])
        gs_all = torch.empty(n_cols, k, device=dev)
        gs_loc = torch.empty(vmax, k, device=dev)
    else:
        cv_all, ci_all = cv_loc, ci_loc
        gs_all = gs_loc = torch.empty(V, k, device=dev)
    y = torch.empty(nl, D, device=dev)
    stage(f"shard rows [{v0}, {v1}) edges {El}; CBSR gathered")
    # one validated call (row_ptr/col_idx/selector ranges) before the raw timed launches
    mk.spgemm_forward(l_row_ptr, l_col, l_val, cv_all, ci_all, D, out=y, validate=True)
    # per-graph setup (like the reference's warp4 files): the backward's bucket / transpose plan
    # "auto" -> the mode that runs
    args.bwd_mode = mk._bwd_mode(args.bwd_mode, k, El, n_cols, nl, D, (l_row_ptr, l_col))
    torch.cuda.synchronize()
    t_plan = time.perf_counter()
    plan = mk.backward_plan(l_col, n_cols, k, args.bwd_mode, indptr=l_row_ptr, values=l_val, dim=D)
    torch.cuda.synchronize()
    t_plan = time.perf_counter() - t_plan

    pipelined = world > 1 and shard.pipeline > 1
    # csc / bsort backward: the forward writes each edge's selectors, phase 1 reads them in
    # order (maxk_spgemm_forward_sel / maxk_sspmm_backward_csc_sel / _bsort) where that pays:
    # k <= 16 by default, MAXK_EDGE_SEL=0/1 off / on (mk.edge_selectors_wanted)
    es = (torch.empty(El, k, dtype=torch.uint8, device=dev)
          if (not pipelined and args.bwd_mode in ("csc", "bsort") and El > 0
              and mk.edge_selectors_wanted(k)) else None)
    if pipelined:  # the parts' plans (per-graph setup, untimed), in the bench's backward mode
        shard.kernels.bwd_mode = args.bwd_mode
        t_plan = time.perf_counter()
        for j in range(shard.pipeline):
            shard.plan(k, D, j)
        torch.cuda.synchronize()
        t_plan = time.perf_counter() - t_plan

    # HIP events on the stream the kernels run on (torch's current stream).  N > 1: the
    # forward interval holds the CBSR exchange and the backward one the gradient exchange
    # (pipelined with the kernels part by part, maxk_dist.ShardedMaxK.aggregate / grad)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    saved = None

    def step(ev=None):
        nonlocal cv_all, ci_all, saved
        if ev:
            ev[0].record()
        if pipelined:
            _, saved = shard.aggregate(cv_loc[:nl], ci_loc[:nl], D, out=y)
        else:
            if world > 1:
                cv_all, ci_all = shard.gather_cbsr(cv_loc[:nl], ci_loc[:nl])
            mk.spgemm_forward(l_row_ptr, l_col, l_val, cv_all, ci_all, D, out=y,
                              chunk=args.chunk, validate=False, edge_sel_out=es)
        if ev:
            ev[1].record()
        if pipelined:
            gs_loc[:nl] = shard.grad(l_G, saved)
        else:
            mk.sspmm_backward(l_row_ptr, l_col, l_val, l_G, ci_all, out=gs_all,
                              chunk=args.chunk, validate=False, mode=args.bwd_mode, plan=plan,
                              edge_sel=es)
            if world > 1:
                gs_loc[:nl] = shard.scatter_grad(gs_all)
        if ev:
            ev[2].record()

    stage(f"backward plan ({args.bwd_mode}) {t_plan:.3f}s")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    stage("warmup done")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    stage(f"timed steps done ({elapsed:.3f}s)")
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- sanity: forward/backward adjoint identity on the timed buffers (summed over ranks:
    # each rank's output rows against its G rows, its CBSR rows against their gradient)
    a = (y.double() * l_G.double()).sum()
    gs_own = gs_all[:nl] if world == 1 else gs_loc[:nl]
    b = (cv_loc[:nl].double() * gs_own.double()).sum()
    if dist:
        ab = torch.stack([a, b])
        if backend != "nccl":
            ab = ab.cpu()
        dist.all_reduce(ab)
        a, b = ab[0], ab[1]
    adj_err = abs(float(a) - float(b)) / max(1.0, abs(float(a)))

    if world > 1:
        # every rank holds the whole graph and X/G (same seeds): recompute its rows unsharded.
        # Ranks sharing a device (the gloo rehearsal) take turns: eight concurrent unsharded
        # products-sized backwards (a 15.8 GB contribution array each) could exhaust the one
        # GPU's memory; each rank frees its cached blocks after its turn.
        shared = world > ndev
        err_local = [0.0, 0.0]
        for turn in range(world if shared else 1):
            if not shared or turn == rank:
                cv_f, ci_f = mk.topk_cbsr(X, k)
                y_f = mk.spgemm_forward(row_ptr, col, val, cv_f, ci_f, D, validate=False)[v0:v1]
                gs_f = mk.sspmm_backward(row_ptr, col, val, G, ci_f, validate=False,
                                         mode=args.bwd_mode)[v0:v1]
                err_local = [
                    float(((y - y_f).abs() / y_f.abs().clamp(min=1)).max()) if nl else 0.0,
                    float(((gs_loc[:nl] - gs_f).abs() / gs_f.abs().clamp(min=1)).max())
                    if nl else 0.0]
                del y_f, gs_f, cv_f, ci_f
                if shared:
                    torch.cuda.synchronize()
                    torch.cuda.empty_cache()
            if shared:
                dist.barrier()
        errs = torch.tensor(err_local, dtype=torch.float64,
                            device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(errs, op=dist.ReduceOp.MAX)
        dist_err = [float(errs[0]), float(errs[1])]
        stage("unsharded self-check done")

    fwd_ms = [e[0].elapsed_time(e[1]) for e in evs]
    bwd_ms = [e[1].elapsed_time(e[2]) for e in evs]
    # per-op launch time: the median over the timed steps; means in extra
    fwd_avg = float(np.median(fwd_ms))
    bwd_avg = float(np.median(bwd_ms))
    ms_per_step = 1000.0 * elapsed / args.steps
    value = 2.0 * E * args.steps / elapsed / 1e9
    B_f, B_b = alg_bytes(nl, El, D, k, n_cols)
    C_f, C_b = compulsory_bytes(nl, El, D, k, n_cols)
    bwd_op = f"sspmm_backward_{args.bwd_mode}"
    op, t_dom, B_dom, C_dom = (bwd_op, bwd_avg, B_b, C_b) if bwd_avg >= fwd_avg else \
        ("spgemm_forward", fwd_avg, B_f, C_f)
    achieved = B_dom / (t_dom * 1e-3) / 1e9
    tkey = f"{args.graph}-D{D}-k{k}-{args.bwd_mode}-n{world}"
    rec, traffic_src = load_traffic_record(tkey, op)
    traffic = rec["bytes"] if rec else None
    f_rec, _ = load_traffic_record(tkey, "spgemm_forward")
    b_rec, _ = load_traffic_record(tkey, bwd_op)

    extra = {
        "fwd_ms": round(fwd_avg, 4), "bwd_ms": round(bwd_avg, 4),
        "fwd_ms_mean": round(float(np.mean(fwd_ms)), 4),
        "bwd_ms_mean": round(float(np.mean(bwd_ms)), 4),
        "fwd_gteps": round(El / fwd_avg / 1e6, 3), "bwd_gteps": round(El / bwd_avg / 1e6, 3),
        "fwd_alg_GBs": round(B_f / fwd_avg / 1e6, 1), "bwd_alg_GBs": round(B_b / bwd_avg / 1e6, 1),
        "adjoint_rel_err": adj_err, "max_deg": int(deg.max()), "chunk": args.chunk,
        "bwd_mode": args.bwd_mode, "backward_plan_s": round(t_plan, 4),
        "build_config": build_cfg,
        "edge_sel_stream": es is not None or (pipelined and any(
            shard._stream(k, D, j) for j in range(shard.pipeline))),
        "fwd_compulsory_GBs": round(C_f / fwd_avg / 1e6, 1),
        "bwd_compulsory_GBs": round(C_b / bwd_avg / 1e6, 1),
    }
    if args.reorder:
        extra["reorder_s"] = None if t_reorder is None else round(t_reorder, 3)
    # edges per occupied (source row, pull bucket): the locality the pull backward feeds on
    extra["pull_locality"] = round(
        mk.pull_locality(l_row_ptr, l_col, int(mk._lib().maxk_pull_shift(k))), 3)
    if args.bwd_mode == "hybrid":  # share of the edges the pulled tiles hold, and their count
        extra["hybrid_pull_edges_frac"] = round(plan[4].shape[0] / max(1, El), 4)
        extra["hybrid_pull_tiles"] = int(plan[0].numel())
    f_traffic = f_rec["bytes"] if f_rec else None
    # both ops against the ceiling that binds them (the dominant one is roofline.binding)
    extra["fwd_binding"] = binding_roofline(fwd_avg, C_f, f_rec)
    extra["bwd_binding"] = binding_roofline(bwd_avg, C_b, b_rec)
    if f_traffic:  # forward: measured (PMC) bytes per launch over its live duration
        extra["fwd_l2_miss_GB"] = round(f_traffic / 1e9, 3)
        extra["fwd_l2_miss_GBs"] = round(f_traffic / (fwd_avg * 1e-3) / 1e9, 1)
    if world > 1:
        extra.update({"dist_check_fwd_max_rel_err": dist_err[0],
                      "dist_check_bwd_max_rel_err": dist_err[1], "dist_backend": backend,
                      "dist_mode": shard.mode, "dist_pipeline": shard.pipeline,
                      # the pipelined gather exchanged transport records (maxk_dist._records)
                      "dist_records": bool(pipelined and shard._records(k, D)),
                      "dist_world_observed": dist.get_world_size(),
                      # since r03 the fwd / bwd intervals hold the CBSR / gradient exchange
                      # (pipelined or not); r02's N > 1 part times held the kernels only
                      "exchange_in_interval": True,
                      "rows_per_rank_max": vmax,
                      "edges_this_rank0": El, "cols_this_rank0": n_cols,
                      "exchange_bytes_rank0": shard.exchange_bytes(k)})

    if rank == 0 and world == 1:
        # CBSR encode (top-k) and the dense rocSPARSE SpMM denominator, outside the timed region
        for _ in range(3):
            mk.topk_cbsr(X, k)
        torch.cuda.synchronize()
        e0_, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0_.record()
        for _ in range(10):
            mk.topk_cbsr(X, k)
        e1_.record()
        e1_.synchronize()
        extra["topk_ms"] = round(e0_.elapsed_time(e1_) / 10, 4)
        if not args.no_rocsparse:
            # every rocSPARSE CSR algorithm; ALG_DEFAULT is the spmm_cusparse.cu:30-46
            # equivalent, the fastest one the fair denominator
            import maxk_kernel_test as mkt
            dense = mk.cbsr_scatter_dense(cv_all, ci_all, D)
            t_algs, y_lib = mkt.library_spmm_times(row_ptr, col, val, dense, 5, 10)
            rs = t_algs["default"]
            best_alg, rs_best = mkt.best_library(t_algs)
            err = (None if y_lib is None else
                   ((y_lib - y).abs() / y.abs().clamp(min=1)).max().item())

            def rnd(a, b=1.0, n=3):  # None when the library refused the algorithm(s)
                return None if a is None else round(a / b, n)
            extra.update({"rocsparse_spmm_ms": rnd(rs, n=4),
                          "rocsparse_spmm_ms_best": rnd(rs_best, n=4),
                          "rocsparse_best_alg": best_alg,
                          "rocsparse_spmm_ms_by_alg": {a: rnd(t, n=4) for a, t in t_algs.items()},
                          "speedup_fwd_vs_rocsparse": rnd(rs, fwd_avg),
                          "speedup_bwd_vs_rocsparse": rnd(rs, bwd_avg),
                          # the step against two library SpMMs (A X and A^T G; the symmetric
                          # synthetic graph gives A^T the same sparsity)
                          "speedup_step_vs_rocsparse": rnd(None if rs is None else 2 * rs,
                                                           fwd_avg + bwd_avg),
                          "speedup_fwd_vs_rocsparse_best": rnd(rs_best, fwd_avg),
                          "speedup_bwd_vs_rocsparse_best": rnd(rs_best, bwd_avg),
                          "speedup_step_vs_rocsparse_best": rnd(
                              None if rs_best is None else 2 * rs_best, fwd_avg + bwd_avg),
                          "rocsparse_vs_maxk_max_rel_err": err})
            del dense, y_lib

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(row_ptr, col, val, cv_all, ci_all, G, D, args.cpu_seconds, deg=deg)
        if not args.no_cpu_spmm:
            extra.update(cpu_spmm_baselines(row_ptr, col, val, mk.cbsr_scatter_dense(cv_all, ci_all, D)))

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 4), "unit": "GTEPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": data,
            "config": {
                "workload": (f"{args.graph}-{'real' if gdir else 'synthetic'} fwd SpGEMM + bwd SSpMM, V={V} E={E} D={D} "
                             f"k={k}"),
                "graph": args.graph, "V": V, "E": E, "D": D, "k": k,
                "parallelism": f"vertex-range x{world}" if world > 1 else "single-gpu",
            },
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "op": op, "kernels": OP_KERNELS[op],
                         "alg_bytes_per_launch": B_dom, "launch_ms": round(t_dom, 4),
                         # the bytes the op must move once (no re-reads) over its duration
                         "compulsory_bytes_per_launch": C_dom,
                         "compulsory_GBs": round(C_dom / (t_dom * 1e-3) / 1e9, 1),
                         "traffic_source": traffic_src, "traffic_key": tkey,
                         # `traffic` is L2 -> fabric bytes (PMC FETCH_SIZE x2 + WRITE_SIZE): it
                         # counts Infinity-Cache hits too (MI355X_MICROARCH.md, HBM), so it is
                         # an L2-miss rate, not HBM traffic
                         # FETCH_SIZE x2: validated per request size in r06 -- every product
                         # kernel's fabric reads are 128-B requests (TCC_EA0_RDREQ_128B_sum =
                         # 99.9-100 % of TCC_EA0_RDREQ_sum), sub-line record gathers included
                         "fetch_correction": "x2 (FETCH_SIZE tallies 128-B requests at 64 B; "
                                             "profiles/r06/fetch_calibration)",
                         "l2_miss_GBs": (round(traffic / (t_dom * 1e-3) / 1e9, 1)
                                         if traffic else None),
                         "l2_miss_frac_of_hbm_peak": (
                             round(traffic / (t_dom * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                             if traffic else None),
                         # `frac` above is algorithmic bytes / HBM peak; the
                         # per-edge gathers it counts are served on chip, so it can pass 1 on a
                         # cache-resident graph.  `binding` is the same launch against the
                         # ceiling that binds it (binding_roofline), <= 1
                         "binding": binding_roofline(t_dom, C_dom, rec)},
            "cpu_baseline": cpu,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    if stacks_after > 0:
        import faulthandler
        faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
