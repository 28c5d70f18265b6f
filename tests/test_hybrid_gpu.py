"""GPU parity of the "hybrid" backward (the pull over a plan's dense tiles through
maxk_sspmm_backward_pull_tiles, accumulating onto the two-phase csc of the other edges)
against the oracle, with the tile kernels beside the csc on a side stream or in line: on a
community-ordered graph and a randomly labelled one, at tile
densities that send every tile, none and part of them to the pull.  Tolerance as in
test_parity_gpu."""
import numpy as np
import pytest
import torch

import oracle as O
from test_parity_gpu import close

pytestmark = pytest.mark.gpu


def _graphs(cuda):
    import maxk_graph
    V, E = 6000, 6000 + 2 * 120000
    ip, ix = maxk_graph.community_graph(V, E, 0.75, 30, 12, 0.9, 5, torch.device(cuda))
    ip2, ix2, _ = maxk_graph.permute_graph(ip, ix, maxk_graph.locality_order(ip, ix))
    return {"random": (ip, ix), "ordered": (ip2, ix2)}


@pytest.mark.parametrize("streams", ["1", "0"])
@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("density", [0.0, 0.3, 1e9])
@pytest.mark.parametrize("name", ["random", "ordered"])
def test_hybrid_against_oracle(cuda, name, density, k, streams, monkeypatch):
    """streams "1": the tile kernels on a side stream beside the csc (the default), "0": in
    line after it."""
    import maxk_cuda_kernels as mk
    monkeypatch.setenv("MAXK_HYBRID_STREAMS", streams)
    ip, ix = _graphs(cuda)[name]
    V, D = ip.numel() - 1, 256
    rng = np.random.default_rng(k)
    val = torch.rand(ix.numel(), device=cuda)
    x = rng.standard_normal((V, D), dtype=np.float32)
    cv, ci = O.topk(x, k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = torch.clamp(torch.diff(ip).float(), min=1.0)
    plan = mk.hybrid_plan(ip, ix, val, V, k, D, density=density)
    tl, _, _, _, ent_d, _, _, off = plan
    if density == 0.0:
        assert off[1].numel() == 0  # every non-empty tile pulls
    if density == 1e9:
        assert tl.numel() == 0 and ent_d.shape[0] == 0  # everything through csc
    assert ent_d.shape[0] + off[1].numel() == ix.numel()
    ci_t = torch.from_numpy(ci).to(cuda)
    gs = mk.sspmm_backward(ip, ix, val, torch.from_numpy(g).to(cuda), ci_t, row_div=div,
                           mode="hybrid", plan=plan)
    go = O.sspmm_bwd(ip.cpu().numpy(), ix.cpu().numpy(), val.cpu().numpy(), g, ci,
                     row_div=div.cpu().numpy())
    close(gs, go)


@pytest.mark.parametrize("k", [16, 32])
def test_hybrid_rectangular(cuda, k):
    """A shard's view (maxk_dist): the first rows of the ordered graph against all its
    columns, so rows != columns and "auto" resolves on the shard's own locality."""
    import maxk_cuda_kernels as mk
    ip, ix = _graphs(cuda)["ordered"]
    V, D = ip.numel() - 1, 256
    n = V // 3
    ip_s, ix_s = ip[:n + 1].contiguous(), ix[:int(ip[n])].contiguous()
    rng = np.random.default_rng(7 + k)
    val = torch.rand(ix_s.numel(), device=cuda)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    g = rng.standard_normal((n, D), dtype=np.float32)
    div = torch.clamp(torch.diff(ip_s).float(), min=1.0)
    for density in (0.3, 1.0, 3.0, 10.0, 30.0):  # the first that pulls some tiles, not all
        plan = mk.hybrid_plan(ip_s, ix_s, val, V, k, D, density=density, cache=False)
        if 0 < plan[4].shape[0] < ix_s.numel():
            break
    assert 0 < plan[4].shape[0] < ix_s.numel()
    gs = mk.sspmm_backward(ip_s, ix_s, val, torch.from_numpy(g).to(cuda),
                           torch.from_numpy(ci).to(cuda), row_div=div, mode="hybrid", plan=plan)
    go = O.sspmm_bwd(ip_s.cpu().numpy(), ix_s.cpu().numpy(), val.cpu().numpy(), g, ci,
                     row_div=div.cpu().numpy())
    close(gs, go)


@pytest.mark.parametrize("mode", ["pull", "hybrid"])
def test_prescaled_entries(cuda, mode, monkeypatch):
    """With a row_div the pull gathers G itself from entries whose weights are pre-divided
    (cached per plan and divisor tensor/version) instead of a G / row_div copy: both ways
    against the oracle, and the cache follows an in-place change of the divisor and a new
    divisor tensor."""
    import maxk_cuda_kernels as mk
    ip, ix = _graphs(cuda)["ordered"]
    V, D, k = ip.numel() - 1, 256, 16
    rng = np.random.default_rng(11)
    val = torch.rand(ix.numel(), device=cuda)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    gt, ct = torch.from_numpy(g).to(cuda), torch.from_numpy(ci).to(cuda)
    args = (ip.cpu().numpy(), ix.cpu().numpy(), val.cpu().numpy(), g, ci)
    div = torch.clamp(torch.diff(ip).float(), min=1.0)
    plan = (mk.hybrid_plan(ip, ix, val, V, k, D, density=0.3) if mode == "hybrid"
            else mk.pull_plan(ip, ix, val, V, k, D))
    for pre in ("1", "0"):
        monkeypatch.setenv("MAXK_PULL_PRESCALE", pre)
        gs = mk.sspmm_backward(ip, ix, val, gt, ct, row_div=div, mode=mode, plan=plan)
        close(gs, O.sspmm_bwd(*args, row_div=div.cpu().numpy()))
    monkeypatch.setenv("MAXK_PULL_PRESCALE", "1")
    div.mul_(2.0)  # in place: the scaled entries are rebuilt
    gs = mk.sspmm_backward(ip, ix, val, gt, ct, row_div=div, mode=mode, plan=plan)
    close(gs, O.sspmm_bwd(*args, row_div=div.cpu().numpy()))
    div2 = div + 1.0  # another divisor tensor
    gs = mk.sspmm_backward(ip, ix, val, gt, ct, row_div=div2, mode=mode, plan=plan)
    close(gs, O.sspmm_bwd(*args, row_div=div2.cpu().numpy()))


@pytest.mark.parametrize("density", [0.0, 0.3, 2.0, 1e9])
def test_hybrid_plan_against_numpy(cuda, density):
    """maxk_hybrid_plan (C ABI) against a numpy restatement: tiles with at least density x
    (rows of their slice) entries are listed in increasing order with their entry runs, each
    bucket lists its tiles' positions in slice order, the pulled entries are the plan's runs of
    those tiles, and every other edge forms a CSR in CSR order."""
    import maxk_cuda_kernels as mk
    ip, ix = _graphs(cuda)["ordered"]
    V, D, k = ip.numel() - 1, 256, 16
    val = torch.rand(ix.numel(), device=cuda)
    tptr, ent, shift, S = mk.pull_plan(ip, ix, val, V, k, D, cache=False)
    tl, te, bp, bt, ent_d, shift2, S2, (oip, oix, oval, _) = mk.hybrid_plan(
        ip, ix, val, V, k, D, density=density, cache=False)
    assert (shift2, S2) == (shift, S)
    nb = -(-V // (1 << shift))
    rps = -(-V // S)
    cnt = np.diff(tptr.cpu().numpy().astype(np.int64))
    t_all = np.arange(S * nb)
    rows_in = np.clip(V - (t_all // nb) * rps, 1, rps)
    dense = (cnt > 0) & (cnt >= density * rows_in)
    want_tl = np.nonzero(dense)[0]
    assert np.array_equal(tl.cpu().numpy(), want_tl)
    assert np.array_equal(te.cpu().numpy(), np.concatenate([[0], np.cumsum(cnt[want_tl])]))
    j = want_tl % nb
    assert np.array_equal(bp.cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(j, minlength=nb))]))
    assert np.array_equal(bt.cpu().numpy(), np.argsort(j * S + want_tl // nb, kind="stable"))
    tp, e = tptr.cpu().numpy(), ent.cpu().numpy()
    want_ent = np.concatenate([e[tp[t]:tp[t + 1]] for t in want_tl]) if want_tl.size else e[:0]
    assert np.array_equal(ent_d.cpu().numpy(), want_ent)
    rp, cx, vv = ip.cpu().numpy(), ix.cpu().numpy(), val.cpu().numpy()
    rows = np.repeat(np.arange(V), np.diff(rp))
    keep = ~dense[(rows // rps) * nb + (cx >> shift)]
    assert np.array_equal(oip.cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(rows[keep], minlength=V))]))
    assert np.array_equal(oix.cpu().numpy(), cx[keep])
    assert np.array_equal(oval.cpu().numpy(), vv[keep])


def test_pull_locality_and_auto_rule(cuda):
    """maxk_pull_locality (edges per occupied (row, bucket) pair) against numpy on a banded
    graph (neighbours close: high locality) and a randomly labelled one, and "auto" choosing
    "hybrid" / "csc" on an ogbn-products-sized problem from it."""
    import maxk_cuda_kernels as mk
    V, deg = 1 << 20, 8
    rows = torch.arange(V).repeat_interleave(deg)
    band = (rows + torch.arange(deg).repeat(V)) % V
    ip = torch.arange(0, V * deg + 1, deg, dtype=torch.int32)
    ix_band = torch.sort(band.view(V, deg), 1).values.flatten().to(torch.int32)
    ix_rand = torch.sort(torch.randint(0, V, (V, deg), generator=torch.Generator().manual_seed(0)),
                         1).values.flatten().to(torch.int32)
    products = dict(num_e=123_718_280, num_cols=2_449_029, num_rows=2_449_029)
    shift = int(mk._lib().maxk_pull_shift(32))
    for ix, want_mode in ((ix_band, "hybrid"), (ix_rand, "csc")):
        b = ix.numpy().astype(np.int64) >> shift
        new = np.ones(b.size, bool)
        new[1:] = b[1:] != b[:-1]
        new[ip.numpy()[:-1]] = True
        ipc, ixc = ip.to(cuda), ix.to(cuda)
        assert abs(mk.pull_locality(ipc, ixc, shift) - b.size / new.sum()) < 1e-9
        assert mk._bwd_mode("auto", 32, **products, dim=256, graph=(ipc, ixc)) == want_mode
    assert mk._bwd_mode("auto", 30, **products, dim=256, graph=(ip.to(cuda), ix_band.to(cuda))) == "csc"


def test_scaled_pull_entries(cuda):
    """maxk_pull_entries_scale: entry {row in slice | column << 16, weight bits} of tile
    t = s*nb + j belongs to row s*rps + (row in slice); the weight becomes weight /
    row_div[row], the key word is unchanged; the copy is cached per (entries, divisor tensor,
    version); listed tiles map runs to their tile ids."""
    import maxk_cuda_kernels as mk
    g = torch.Generator().manual_seed(3)
    S, shift, V = 3, 4, 13
    num_cols = 60
    nb = -(-num_cols // (1 << shift))
    rps = -(-V // S)
    counts = torch.randint(0, 4, (S * nb,), generator=g)
    E = int(counts.sum())
    tiles = torch.arange(S * nb)
    t_of = torch.repeat_interleave(tiles, counts)
    rin = torch.randint(0, rps, (E,), generator=g)
    rin = torch.where(t_of // nb * rps + rin < V, rin, 0)
    col = torch.randint(0, 1 << shift, (E,), generator=g)
    w = torch.rand(E, generator=g)
    ent = torch.stack([rin | (col << 16), w.view(torch.int32).long()], 1).to(torch.int32).to(cuda)
    div = (torch.rand(V, generator=g) + 0.5).to(cuda)
    tptr = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(counts, 0)]).int().to(cuda)
    sc = mk._scaled_entries(ent, None, tptr, V, num_cols, shift, S, div)
    assert torch.equal(sc[:, 0], ent[:, 0])
    rows = (t_of // nb * rps + rin).to(cuda)
    assert torch.equal(sc[:, 1].view(torch.float32), ent[:, 1].view(torch.float32) / div[rows])
    assert mk._scaled_entries(ent, None, tptr, V, num_cols, shift, S, div) is sc  # cached
    div.mul_(2.0)
    sc2 = mk._scaled_entries(ent, None, tptr, V, num_cols, shift, S, div)  # version moved
    assert sc2 is not sc
    assert torch.equal(sc2[:, 1].view(torch.float32), ent[:, 1].view(torch.float32) / div[rows])
    # listed tiles: only some tiles' runs, mapped through their ids
    lt = torch.nonzero(counts > 0).flatten()[::2]
    sub = torch.cat([ent[int(tptr[t]):int(tptr[t + 1])] for t in lt.tolist()])
    te = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(counts[lt], 0)]).int().to(cuda)
    sc3 = mk._scaled_entries(sub, lt.int().to(cuda), te, V, num_cols, shift, S, div)
    rows3 = torch.cat([rows[int(tptr[t]):int(tptr[t + 1])] for t in lt.tolist()])
    assert torch.equal(sc3[:, 1].view(torch.float32), sub[:, 1].view(torch.float32) / div[rows3])


@pytest.mark.parametrize("side", [False, True])
def test_c_abi_hybrid_backward(cuda, side):
    """maxk_sspmm_backward_hybrid called through the C ABI directly (what a non-Python host
    does): in line on one stream, and with the tile kernels on a side stream forked and joined
    by the caller's two events; twice each, against the oracle."""
    import ctypes
    import maxk_cuda_kernels as mk
    from maxk_cuda_kernels import _capi
    L = _capi.load()
    ip, ix = _graphs(cuda)["ordered"]
    V, D, k = ip.numel() - 1, 256, 16
    rng = np.random.default_rng(5)
    val = torch.rand(ix.numel(), device=cuda)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = torch.clamp(torch.diff(ip).float(), min=1.0)
    # a density between the sparsest tile's and the others': some tiles pulled, some not
    tptr, _, _, S0 = mk.pull_plan(ip, ix, val, V, k, D, cache=False)
    cnt = torch.diff(tptr.long()).double()
    rows_in = -(-V // S0)
    dens = torch.unique(cnt[cnt > 0] / rows_in).sort().values
    assert dens.numel() >= 2
    plan = mk.hybrid_plan(ip, ix, val, V, k, D, density=float(dens[0] + dens[1]) / 2,
                          cache=False)
    tl, te, bp, bt, ent, shift, S, (oip, oix, oval, (ocp, oeid)) = plan
    assert tl.numel() > 0 and oix.numel() > 0
    gt, ct = torch.from_numpy(g).to(cuda), torch.from_numpy(ci).to(cuda)
    out = torch.empty(V, k, device=cuda)
    ws = torch.empty(L.maxk_sspmm_backward_hybrid_workspace_size(V, V, oix.numel(), D, k,
                                                                 tl.numel()),
                     dtype=torch.uint8, device=cuda)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = torch.cuda.Stream()
    evs = (torch.cuda.Event(), torch.cuda.Event())
    for e in evs:
        e.record()
    ref = O.sspmm_bwd(ip.cpu().numpy(), ix.cpu().numpy(), val.cpu().numpy(), g, ci,
                      row_div=div.cpu().numpy())
    for _ in range(2):
        out.fill_(float("nan"))
        _capi.check(L.maxk_sspmm_backward_hybrid(
            p(gt), p(div), p(ct), p(tl), p(te), tl.numel(), p(bp), p(bt), p(ent), ent.shape[0],
            shift, S, p(oip), p(oix), p(oval), oix.numel(), p(ocp), p(oeid), 0, p(out), V, V, D,
            k, p(ws), ws.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
            ctypes.c_void_p(st.cuda_stream) if side else None,
            evs[0]._as_parameter_ if side else None, evs[1]._as_parameter_ if side else None),
            "maxk_sspmm_backward_hybrid")
        torch.cuda.synchronize()
        close(out, ref)
