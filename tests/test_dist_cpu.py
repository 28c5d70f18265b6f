"""Multi-process (gloo, CPU) tests of the sharded aggregation.

The HIP kernels are replaced by the oracle (test infrastructure) through the
`kernels=` hook, so what is checked here is the distributed logic itself:
nnz-balanced partition, column remap to the padded space ("gather" mode) or
the halo ("halo" mode), all-gather / all-to-allv of the CBSR rows,
reduce-scatter / all-to-allv + index_add of the gradient partials, autograd
plumbing.  Each
rank's slice must equal the 1-process oracle result (forward bit-exact: every
output row is computed whole on its owner; backward within 1e-5 relative,
since the reduce-scatter sums per-rank partials in a different order).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import conftest  # noqa: F401  (sys.path: package, oracle)
import maxk_dist
import oracle

BWD_ATOL = 1e-5


class OracleKernels:
    """kernels= backend for ShardedMaxK built on the CPU oracle (tests only)."""

    def spgemm_forward(self, indptr, indices, values, cbsr_val, cbsr_idx, D, row_div=None,
                       out=None, accumulate=False):
        y = torch.from_numpy(oracle.spgemm_fwd(indptr.numpy(), indices.numpy(), values.numpy(),
                                               cbsr_val.numpy(), cbsr_idx.numpy(), D,
                                               row_div=None if row_div is None
                                               else row_div.numpy()))
        if out is None:
            return y
        if accumulate:
            out += y
        else:
            out.copy_(y)
        return out

    def sspmm_backward(self, indptr, indices, values, grad, cbsr_idx, row_div=None, plan=None):
        g = oracle.sspmm_bwd(indptr.numpy(), indices.numpy(), values.numpy(), grad.numpy(),
                             cbsr_idx.numpy(),
                             row_div=None if row_div is None else row_div.numpy())
        return torch.from_numpy(g)


class OracleRecordKernels(OracleKernels):
    """OracleKernels plus the transport-record surface (records_ok / cbsr_records /
    spgemm_forward_records), so the CPU tests take ShardedMaxK's record route: records are the
    [k f32 | k u8] bytes of each CBSR row, unpacked for the oracle's forward."""

    def records_ok(self, num_rows, num_cols, num_e, dim, k):
        return k % 4 == 0 and 24 <= k <= 32

    def cbsr_records(self, cbsr_val, cbsr_idx, dim):
        k = cbsr_val.shape[1]
        return torch.cat([cbsr_val.contiguous().view(torch.uint8).view(-1, 4 * k),
                          cbsr_idx.contiguous()], 1).contiguous()

    def spgemm_forward_records(self, indptr, indices, values, rec, k, D, row_div=None, out=None,
                               accumulate=False):
        cv = rec[:, :4 * k].contiguous().view(torch.float32)
        ci = rec[:, 4 * k:].contiguous()
        return self.spgemm_forward(indptr, indices, values, cv, ci, D, row_div=row_div, out=out,
                                   accumulate=accumulate)


def make_graph(V, avg_deg, seed, hub=True):
    rng = np.random.default_rng(seed)
    deg = rng.poisson(avg_deg, V).astype(np.int64)
    if hub:
        deg[V // 3] = 8 * avg_deg * 10  # one heavy row makes the nnz split uneven in rows
    if V > 5:
        deg[5] = 0  # an empty row
    row_ptr = np.zeros(V + 1, dtype=np.int64)
    np.cumsum(deg, out=row_ptr[1:])
    E = int(row_ptr[-1])
    col = rng.integers(0, V, E).astype(np.int32)
    val = rng.standard_normal(E).astype(np.float32)
    return row_ptr.astype(np.int32), col, val


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, V, D, k, seed, use_div, q, bounds=None, mode="gather",
            pipeline=1, records=False):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        row_ptr, col, val = make_graph(V, 6, seed)
        rng = np.random.default_rng(seed + 1)
        x = rng.standard_normal((V, D)).astype(np.float32)
        tv, ti = oracle.topk(x, k)
        g = rng.standard_normal((V, D)).astype(np.float32)
        deg = np.maximum(np.diff(row_ptr), 1).astype(np.float32)

        shard = maxk_dist.ShardedMaxK(torch.from_numpy(row_ptr), torch.from_numpy(col),
                                      torch.from_numpy(val), rank, world,
                                      kernels=OracleRecordKernels() if records
                                      else OracleKernels(), bounds=bounds, mode=mode,
                                      pipeline=pipeline)
        if records:  # the record route is what runs (every part's forward over records)
            assert shard.pipeline > 1 and shard._records(k, D)
        v0, v1 = shard.v0, shard.v1
        div = torch.from_numpy(deg[v0:v1]) if use_div else None
        val_l = torch.from_numpy(tv[v0:v1]).requires_grad_(True)
        y = maxk_dist.sharded_maxk_spgemm(shard, val_l, torch.from_numpy(ti[v0:v1]), D, div)
        y.backward(torch.from_numpy(g[v0:v1]))
        q.put((rank, v0, v1, y.detach().numpy(), val_l.grad.numpy(), shard.bounds,
               shard.exchange_bytes(k), shard.n_cols))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, "error", repr(e)))
        raise


def _run(world, V=400, D=64, k=8, seed=0, use_div=True, bounds=None, mode="gather",
         pipeline=1, records=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, V, D, k, seed, use_div, q, bounds, mode,
                               pipeline, records))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for o in outs:
        assert o[1] != "error", o
    return sorted(outs)


def _single(V, D, k, seed, use_div):
    row_ptr, col, val = make_graph(V, 6, seed)
    rng = np.random.default_rng(seed + 1)
    x = rng.standard_normal((V, D)).astype(np.float32)
    tv, ti = oracle.topk(x, k)
    g = rng.standard_normal((V, D)).astype(np.float32)
    deg = np.maximum(np.diff(row_ptr), 1).astype(np.float32) if use_div else None
    y = oracle.spgemm_fwd(row_ptr, col, val, tv, ti, D, row_div=deg)
    gs = oracle.sspmm_bwd(row_ptr, col, val, g, ti, row_div=deg)
    return y, gs


@pytest.mark.parametrize("mode,pipeline", [("gather", 1), ("gather", 2), ("gather", 3),
                                           ("halo", 1), ("auto", None)])
@pytest.mark.parametrize("world,use_div,bounds", [(2, True, None), (3, False, None),
                                                  (4, True, None),
                                                  (3, True, [0, 150, 150, 400])])
def test_sharded_matches_single_process(world, use_div, bounds, mode, pipeline):
    """The last case gives rank 1 no rows: it still joins every collective (an all-padding
    chunk in "gather" mode, empty splits in "halo" mode), and the other ranks' results are
    unchanged.  pipeline > 1 ("gather"): the exchange in column parts, the forward summed
    part by part (so within 1e-6 of the one-pass sum instead of bit-exact)."""
    V, D, k, seed = 400, 64, 8, 7
    outs = _run(world, V, D, k, seed, use_div, bounds, mode, pipeline)
    y_ref, gs_ref = _single(V, D, k, seed, use_div)
    covered = 0
    for rank, v0, v1, y, gs, bounds, xb, n_cols in outs:
        assert bounds[0] == 0 and bounds[-1] == V
        if pipeline == 1 or mode == "halo":
            np.testing.assert_array_equal(y, y_ref[v0:v1])
        else:
            np.testing.assert_allclose(y, y_ref[v0:v1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(gs, gs_ref[v0:v1], rtol=1e-5, atol=BWD_ATOL)
        covered += v1 - v0
    assert covered == V


@pytest.mark.parametrize("mode,pipeline", [("gather", 1), ("gather", 2), ("halo", 1)])
def test_sharded_matches_single_process_world8(mode, pipeline):
    """The driver's scaling run goes to 8 ranks: the same check at world 8 (one rank per
    process, gloo), with the pipelined exchange and the halo mode."""
    V, D, k, seed = 600, 32, 8, 11
    outs = _run(8, V, D, k, seed, True, None, mode, pipeline)
    y_ref, gs_ref = _single(V, D, k, seed, True)
    covered = 0
    for rank, v0, v1, y, gs, bounds, xb, n_cols in outs:
        if pipeline == 1:
            np.testing.assert_array_equal(y, y_ref[v0:v1])
        else:
            np.testing.assert_allclose(y, y_ref[v0:v1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(gs, gs_ref[v0:v1], rtol=1e-5, atol=BWD_ATOL)
        covered += v1 - v0
    assert covered == V


@pytest.mark.parametrize("world,pipeline,bounds", [(2, 2, None), (4, 3, None),
                                                   (3, 2, [0, 150, 150, 400])])
def test_sharded_transport_records(world, pipeline, bounds):
    """The pipelined gather over transport records (ShardedMaxK._aggregate_records: each owner
    packs its part rows as [k f32 | k u8] records, one uint8 all-gather per part, the records
    forward per part; the backward reads the parts' selectors out of the records) against the
    single-process oracle, k = 32; the last case has an empty rank."""
    V, D, k, seed = 400, 64, 32, 5
    outs = _run(world, V, D, k, seed, True, bounds, "gather", pipeline, records=True)
    y_ref, gs_ref = _single(V, D, k, seed, True)
    covered = 0
    for rank, v0, v1, y, gs, bounds_, xb, n_cols in outs:
        np.testing.assert_allclose(y, y_ref[v0:v1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(gs, gs_ref[v0:v1], rtol=1e-5, atol=BWD_ATOL)
        covered += v1 - v0
    assert covered == V


def test_hip_backend_offers_records():
    """The HIP backend exposes the record surface ShardedMaxK._records looks for (r05 left it
    off _HipKernels, so the record route never ran outside the CPU stand-in)."""
    for f in ("records_ok", "cbsr_records", "spgemm_forward_records"):
        assert callable(getattr(maxk_dist._HipKernels, f))


def test_balanced_bounds_properties():
    row_ptr, _, _ = make_graph(1000, 5, 3)
    rp = torch.from_numpy(row_ptr)
    for world in (1, 2, 3, 8, 16):
        b = maxk_dist.balanced_bounds(rp, world)
        assert len(b) == world + 1 and b[0] == 0 and b[-1] == 1000
        assert all(b[i] <= b[i + 1] for i in range(world))
        E = int(row_ptr[-1])
        max_row = int(np.diff(row_ptr).max())
        for i in range(world):
            nnz = int(row_ptr[b[i + 1]] - row_ptr[b[i]])
            assert nnz <= E // world + max_row + 1
    # more shards than rows: some shards are empty, still a valid partition
    b = maxk_dist.balanced_bounds(torch.tensor([0, 3, 3, 5], dtype=torch.int32), 5)
    assert b[0] == 0 and b[-1] == 3 and all(b[i] <= b[i + 1] for i in range(5))


def test_column_remap_single_rank():
    """world=1 is the identity remap; the remapped column of a vertex is owner*vmax+offset."""
    row_ptr, col, val = make_graph(200, 4, 11, hub=False)
    rp, ci, va = map(torch.from_numpy, (row_ptr, col, val))
    s = maxk_dist.ShardedMaxK(rp, ci, va, 0, 1, kernels=OracleKernels())
    assert torch.equal(s.col_idx, ci) and torch.equal(s.row_ptr, rp)
    b = [0, 50, 120, 200]
    s1 = maxk_dist.ShardedMaxK(rp, ci, va, 1, 3, kernels=OracleKernels(), bounds=b)
    assert s1.vmax == 80 and s1.n_cols == 240 and (s1.v0, s1.v1) == (50, 120)
    e0, e1 = int(row_ptr[50]), int(row_ptr[120])
    cols = col[e0:e1].astype(np.int64)
    owner = np.searchsorted(np.array(b[1:]), cols, side="right")
    np.testing.assert_array_equal(s1.col_idx.numpy(), owner * 80 + cols - np.array(b)[owner])


def test_halo_exchange_smaller_on_local_graph():
    """A graph with locality (each row's columns near the row): the halo mode moves only the
    neighbouring shards' boundary rows, and its column space is the shard's halo."""
    V, D, k, world = 600, 32, 4, 3
    rng = np.random.default_rng(4)
    deg = rng.poisson(5, V).astype(np.int64)
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum(deg, out=row_ptr[1:])
    rows = np.repeat(np.arange(V), deg)
    col = np.clip(rows + rng.integers(-20, 21, rows.size), 0, V - 1).astype(np.int32)
    val = rng.random(col.size, dtype=np.float32)
    args = (torch.from_numpy(row_ptr.astype(np.int32)), torch.from_numpy(col),
            torch.from_numpy(val))
    outs = _run_local(world, args, D, k)  # each rank also checks halo == gather results
    for rank, v0, v1, y, gs, bounds, xb_halo, n_cols, xb_gather in outs:
        assert xb_halo["fwd_recv"] < xb_gather["fwd_recv"] / 4  # boundary rows only
        e0, e1 = row_ptr[v0], row_ptr[v1]
        assert n_cols == np.unique(col[e0:e1]).size


def _local_worker(rank, world, port, args, D, k, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rp, col, val = args
        V = rp.numel() - 1
        rng = np.random.default_rng(9)
        tv, ti = oracle.topk(rng.standard_normal((V, D)).astype(np.float32), k)
        g = rng.standard_normal((V, D)).astype(np.float32)
        res = {}
        for mode in ("gather", "halo", "auto"):
            shard = maxk_dist.ShardedMaxK(rp, col, val, rank, world, kernels=OracleKernels(),
                                          mode=mode)
            if mode == "auto":  # a local graph's shards need few rows: the halo exchange
                assert shard.mode == "halo" and shard.halo_share <= shard.HALO_SHARE
            v0, v1 = shard.v0, shard.v1
            val_l = torch.from_numpy(tv[v0:v1]).requires_grad_(True)
            y = maxk_dist.sharded_maxk_spgemm(shard, val_l, torch.from_numpy(ti[v0:v1]), D)
            y.backward(torch.from_numpy(g[v0:v1]))
            res[mode] = (y.detach().numpy(), val_l.grad.numpy(), shard.exchange_bytes(k),
                         shard.n_cols)
        yg, gg, xg, _ = res["gather"]
        yh, gh, xh, nh = res["halo"]
        np.testing.assert_allclose(yh, yg, rtol=1e-5, atol=1e-6)  # gather: pipelined parts
        np.testing.assert_allclose(gh, gg, rtol=1e-5, atol=BWD_ATOL)
        q.put((rank, v0, v1, yh, gh, shard.bounds, xh, nh, xg))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, "error", repr(e)))
        raise


def _run_local(world, args, D, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_worker, args=(r, world, port, args, D, k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for o in outs:
        assert o[1] != "error", o
    return sorted(outs, key=lambda o: o[0])


@pytest.mark.gpu
def test_sharded_hip_single_rank_rccl(cuda):
    """ShardedMaxK over RCCL (world 1) with the HIP kernels == the direct HIP calls == oracle;
    then the pipelined gather mode (3 column parts, async RCCL all-gathers and reduce-scatters
    waited on by the compute stream, the accumulating forward) on the same communicator."""
    import maxk_cuda_kernels as mk
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    try:
        V, D = 3000, 256
        row_ptr, col, val = make_graph(V, 9, 5)
        rng = np.random.default_rng(2)
        x = rng.standard_normal((V, D)).astype(np.float32)
        g = rng.standard_normal((V, D)).astype(np.float32)
        deg = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
        to = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
        refs = {}
        # (k, pipeline, mode): the plain and pipelined gathers at k = 16 (two async RCCL
        # all-gathers per part); k = 32 pipelined through the transport records (VERDICT r05
        # item 1: cbsr_records + one uint8 async all-gather per part, the records forward, the
        # parts' reduce-scatters); the halo exchange (all_to_all_single on RCCL, the plan's two
        # all-to-alls and the forward / backward ones) at k = 16 and 32
        for k, pipeline, mode in ((16, None, "gather"), (16, 3, "gather"), (32, 2, "gather"),
                                  (16, None, "halo"), (32, None, "halo")):
            if k not in refs:
                tv, ti = oracle.topk(x, k)
                refs[k] = (tv, ti, oracle.spgemm_fwd(row_ptr, col, val, tv, ti, D, row_div=deg),
                           oracle.sspmm_bwd(row_ptr, col, val, g, ti, row_div=deg))
            tv, ti, y_ref, gs_ref = refs[k]
            shard = maxk_dist.ShardedMaxK(to(row_ptr), to(col), to(val), 0, 1, device=cuda,
                                          pipeline=pipeline, mode=mode, k=k)
            assert shard.mode == mode
            assert shard.pipeline == (1 if pipeline is None else pipeline)
            if pipeline is not None:
                assert shard._records(k, D) == (k == 32), (k, pipeline)
            if mode == "halo":
                assert shard.n_cols == np.unique(col).size and shard.send_counts == [shard.n_cols]
            for _ in range(2):  # the second step reuses the plans and the cached graph check
                val_l = to(tv).requires_grad_(True)
                y = maxk_dist.sharded_maxk_spgemm(shard, val_l, to(ti), D, to(deg))
                y.backward(to(g))
                torch.cuda.synchronize()
                np.testing.assert_allclose(y.detach().cpu().numpy(), y_ref, rtol=1e-4, atol=1e-4)
                np.testing.assert_allclose(val_l.grad.cpu().numpy(), gs_ref, rtol=1e-4,
                                           atol=1e-4)
            if pipeline is None and mode == "gather":
                y2 = mk.spgemm_forward(to(row_ptr), to(col), to(val), to(tv), to(ti), D,
                                       row_div=to(deg))
                assert torch.equal(y.detach(), y2)
    finally:
        dist.destroy_process_group()


def test_pipeline_rule_by_exchange_bytes(monkeypatch):
    """Gather mode pipelines the exchange only where it is large enough to hide (a collective
    costs tens of microseconds however small): with k known, a rank whose step exchange
    (world - 1) * vmax * 5k bytes is below PIPELINE_MIN_BYTES keeps one part; without k, or
    with an explicit part count, the old behaviour.  No collective runs in gather-mode
    construction, so this needs no process group."""
    import maxk_dist
    rng = np.random.default_rng(7)
    V = 4000
    deg = rng.integers(1, 20, V)
    rp = np.zeros(V + 1, np.int64)
    rp[1:] = np.cumsum(deg)
    col = rng.integers(0, V, int(rp[-1])).astype(np.int32)
    args = (torch.from_numpy(rp.astype(np.int32)), torch.from_numpy(col),
            torch.rand(col.size))
    mk = lambda **kw: maxk_dist.ShardedMaxK(*args, rank=0, world=8, kernels=object(),  # noqa
                                            **kw)
    assert mk().pipeline == 2 and mk(k=16).pipeline == 1 and mk(k=16, pipeline=3).pipeline == 3
    s = mk(k=16)
    need = (8 - 1) * s.vmax * 5 * 16
    monkeypatch.setattr(maxk_dist.ShardedMaxK, "PIPELINE_MIN_BYTES", need)
    assert mk(k=16).pipeline == 2 and mk(k=15).pipeline == 1
