"""GPU: the sharded aggregation (maxk_dist) at world size 2 and 4 with the HIP kernels, on
the box's one MI355X (BASELINE.json configs[3], rehearsed on one device).

The parent writes a products-shaped graph (power-law degrees around 50, D = 256, k = 32),
starts N fresh worker processes (tests/dist_gpu_worker.py: gloo collectives staged through
host memory, HIP kernels on cuda:0, one hardware queue per process) and checks every rank's
forward rows and CBSR-gradient rows, in both exchange modes ("gather" and "halo"), against
the 1-process HIP result (1e-5 relative: hub rows split differently over work items, and the
gradient partials are summed in another order) and against the oracle (1e-4, north_star).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def products_like(V, avg, seed):
    """Power-law out-degrees (mean ~avg), random sorted distinct columns, self loops."""
    rng = np.random.default_rng(seed)
    w = (np.arange(V) + 30.0) ** -0.75
    deg = np.minimum(rng.poisson(avg * w / w.mean()), V - 1) + 1
    rows, cols = [], []
    for r in range(V):
        c = rng.choice(V, int(deg[r]), replace=False)
        c[0] = r  # a self loop per row
        cols.append(np.unique(c))
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum([c.size for c in cols], out=row_ptr[1:])
    return row_ptr.astype(np.int32), np.concatenate(cols).astype(np.int32)


@pytest.fixture(scope="module")
def graph(tmp_path_factory):
    V, D, k = 12000, 256, 32
    row_ptr, col = products_like(V, 50, 3)
    rng = np.random.default_rng(4)
    g = {"row_ptr": row_ptr, "col": col, "val": rng.random(col.size, dtype=np.float32),
         "x": rng.standard_normal((V, D), dtype=np.float32),
         "g": rng.standard_normal((V, D), dtype=np.float32),
         "deg": np.maximum(np.diff(row_ptr), 1).astype(np.float32), "k": k, "D": D}
    d = tmp_path_factory.mktemp("dist_gpu")
    np.savez(d / "graph.npz", **g)
    return d, g


@pytest.fixture(scope="module")
def single(graph, cuda):
    """The 1-process HIP result and the oracle, over the whole graph."""
    import maxk_cuda_kernels as mk
    _, g = graph
    to = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    k, D = g["k"], g["D"]
    cv, ci = mk.topk_cbsr(to(g["x"]), k)
    rp, cl, va, dg = to(g["row_ptr"]), to(g["col"]), to(g["val"]), to(g["deg"])
    y = mk.spgemm_forward(rp, cl, va, cv, ci, D, row_div=dg).cpu().numpy()
    gs = mk.sspmm_backward(rp, cl, va, to(g["g"]), ci, row_div=dg).cpu().numpy()
    cvn, cin = cv.cpu().numpy(), ci.cpu().numpy()
    yo = O.spgemm_fwd(g["row_ptr"], g["col"], g["val"], cvn, cin, D, row_div=g["deg"])
    go = O.sspmm_bwd(g["row_ptr"], g["col"], g["val"], g["g"], cin, row_div=g["deg"])
    return y, gs, yo, go


def close(a, ref, tol):
    err = np.abs(a.astype(np.float64) - ref.astype(np.float64))
    bad = err > tol * np.maximum(1.0, np.abs(ref.astype(np.float64)))
    assert not bad.any(), f"{bad.sum()} elements off; max err {err.max():.3e}"


def _run_world(graph, single, world, backend):
    d, g = graph
    y1, gs1, yo, go = single
    port = _free_port()
    env = dict(os.environ)
    if backend == "gloo":
        env["GPU_MAX_HW_QUEUES"] = "1"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), str(d),
                               str(r), str(world), str(port), backend], env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    V = g["row_ptr"].size - 1
    for mode in ("gather", "halo"):
        covered = 0
        for r in range(world):
            with np.load(os.path.join(d, f"rank{r}.npz"), allow_pickle=False) as z:
                b = z[f"{mode}_bounds"]
                v0, v1 = int(b[r]), int(b[r + 1])
                close(z[f"{mode}_y"], y1[v0:v1], 1e-5)
                close(z[f"{mode}_gs"], gs1[v0:v1], 1e-5)
                close(z[f"{mode}_y"], yo[v0:v1], 1e-4)
                close(z[f"{mode}_gs"], go[v0:v1], 1e-4)
                covered += v1 - v0
        assert covered == V


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_world_n_on_one_gpu(graph, single, world):
    _run_world(graph, single, world, "gloo")


@pytest.mark.parametrize("world", [2])
def test_sharded_nccl_one_gpu_per_rank(graph, single, world):
    """The RCCL path the driver's N-GPU bench takes (one rank per GPU, device collectives over
    xGMI); skipped where fewer than `world` GPUs are visible (the one-GPU box)."""
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs, {torch.cuda.device_count()} visible")
    _run_world(graph, single, world, "nccl")


@pytest.mark.parametrize("stream", ["0", "1"])
@pytest.mark.parametrize("bwd", ["bsort", "csc", "dense"])
def test_sharded_forced_backward_modes(graph, single, bwd, stream, monkeypatch):
    """World 2 with every shard's backward forced to the two-phase forms a large sparse graph
    resolves to (window-sorted at k <= 8, csc above): the shards' column spaces are the padded
    gathered ones (gather mode) or the compact halos (halo mode), their plans built per shard
    and pipeline part; with MAXK_EDGE_SEL=1 every pipeline part's forward also writes its
    edge-selector stream (the later parts through maxk_spgemm_forward_accumulate_sel) and its
    backward reads it.  "dense" (selected columns gathered along each shard's transpose, r05)
    reads no stream."""
    monkeypatch.setenv("MAXK_BWD_MODE", bwd)
    monkeypatch.setenv("MAXK_EDGE_SEL", stream)
    _run_world(graph, single, 2, "gloo")


@pytest.mark.parametrize("graph,k,gpus,records", [("products", 32, 2, True),
                                                  ("products", 32, 4, True),
                                                  ("products", 32, 8, True),
                                                  ("reddit", 16, 8, False)])
def test_bench_self_launch(graph, k, gpus, records):
    """BASELINE.json configs[3] (and the driver's default-graph SCALE shape) at real size through
    the driver's own command shape: `python bench.py --gpus N
    ...` with no WORLD_SIZE starts its N ranks itself (bench.launch_ranks: a child
    torch.distributed.run, gloo-staged collectives on this one GPU), shards the graph by vertex
    range and checks every rank's forward rows and CBSR-gradient rows against the unsharded HIP
    result, which tests/test_fullsize_gpu.py pins to the oracle on every row.  ogbn-products at
    k = 32 (V = 2,449,029, E = 123.7M) takes the pipelined transport-record exchange at N = 2, 4
    and 8 (configs[3]'s shapes); Reddit at k = 16 and N = 8 (`bench.py --gpus 8`, the driver's
    default graph) one part.
    World > 1 over RCCL itself stays unmeasured on this one-GPU box."""
    import json
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["MAXK_DIST_BACKEND"] = "gloo"
    env.pop("MAXK_VALIDATE", None)  # the bench validates its graph once itself
    root = os.path.dirname(HERE)
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", str(gpus),
                        "--graph", graph, "--k", str(k), "--steps", "2", "--warmup", "1"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=280)
    if p.returncode != 0:
        # a failing rank's own traceback sits above torch.distributed.run's summary
        lines = p.stderr.splitlines()
        hits = [i for i, ln in enumerate(lines) if "Traceback" in ln or "Error" in ln]
        first = "\n".join(lines[max(0, hits[0] - 2):hits[0] + 40]) if hits else ""
        raise AssertionError(f"rc {p.returncode}\n{first}\n...\n{p.stderr[-1500:]}")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    e = d["extra"]
    V = {"products": 2449029, "reddit": 232965}[graph]
    assert d["n_gpus"] == gpus and d["config"]["V"] == V and d["config"]["k"] == k
    assert d["config"]["parallelism"] == f"vertex-range x{gpus}"
    assert e["dist_backend"] == "gloo" and e["dist_world_observed"] == gpus
    assert e["dist_records"] == records, e
    assert e["dist_check_fwd_max_rel_err"] <= 1e-5, e
    assert e["dist_check_bwd_max_rel_err"] <= 1e-5, e
    assert e["adjoint_rel_err"] <= 1e-6, e
