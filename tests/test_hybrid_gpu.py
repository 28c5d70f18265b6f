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
