"""MaxK-GNN layers (maxk_layers) on the HIP aggregation vs the same layers on a dense PyTorch
aggregation (test-only reference): forward outputs and every gradient, fp32, rtol/atol 1e-4."""
import numpy as np
import pytest
import torch

import conftest  # noqa: F401  (sys.path)

RTOL = ATOL = 1e-4


class DenseGraph:
    """Same interface as maxk_layers.CSRGraph, aggregation by a dense matmul (reference)."""

    def __init__(self, g):
        self.g = g
        self.num_nodes = g.num_nodes
        self.indices, self.indptr, self.values = g.indices, g.indptr, g.values
        self.in_degrees, self.out_degrees = g.in_degrees, g.out_degrees
        self.edge_rows = g.edge_rows

    def aggregate(self, topk_values, topk_indices, dim, values=None, row_div=None):
        V = self.num_nodes
        A = torch.zeros(V, V, device=topk_values.device)
        A.index_put_((self.edge_rows().long(), self.indices.long()),
                     self.values if values is None else values, accumulate=True)
        x = torch.zeros(V, dim, device=topk_values.device).scatter(1, topk_indices.long(),
                                                                   topk_values)
        y = A @ x
        return y if row_div is None else y / row_div[:, None]


def _graph(cuda, V=400, m=3000, seed=0):
    import maxk_graph
    import maxk_layers
    rng = np.random.default_rng(seed)
    ip, ix = maxk_graph.build_csr(torch.from_numpy(rng.integers(0, V, m)).to(cuda),
                                  torch.from_numpy(rng.integers(0, V, m)).to(cuda), V)
    vals = torch.rand(ix.numel(), device=cuda)
    return maxk_layers.CSRGraph(ip, ix, vals)


def _compare(run, cuda, seed=0):
    """run(graph, gen) -> (output, [tensors whose .grad to compare]) ; same weights both times."""
    import maxk_layers  # noqa: F401
    g = _graph(cuda, seed=seed)
    torch.manual_seed(seed)
    out1, leaves1 = run(g)
    torch.manual_seed(seed)
    out2, leaves2 = run(DenseGraph(g))
    torch.testing.assert_close(out1, out2, rtol=RTOL, atol=ATOL)
    gout = torch.randn_like(out1)
    out1.backward(gout)
    out2.backward(gout)
    for a, b in zip(leaves1, leaves2):
        torch.testing.assert_close(a.grad, b.grad, rtol=RTOL, atol=ATOL)


@pytest.mark.gpu
def test_maxk_nonlinearity_grad(cuda):
    import maxk_layers
    x = torch.randn(300, 64, device=cuda, requires_grad=True)
    dense, vals, idx = maxk_layers.maxk(x, 8)
    tv, ti = torch.topk(x.detach(), 8, dim=1)
    assert torch.equal(idx.long(), ti) and torch.equal(vals.detach(), tv)
    mask = torch.zeros_like(x).scatter(1, ti, 1.0)
    assert torch.equal(dense.detach(), x.detach() * mask)
    w1, w2 = torch.randn_like(x), torch.randn(300, 8, device=cuda)
    ((dense * w1).sum() + (vals * w2).sum()).backward()
    ref = w1 * mask + torch.zeros_like(x).scatter(1, ti, w2)  # both paths reach the input
    torch.testing.assert_close(x.grad, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,k", [(64, 8), (256, 32), (64, 32), (64, 64)])  # k >= dim / 2: dense route
def test_sage_conv(cuda, dim, k):
    import maxk_layers

    def run(g):
        x = torch.randn(g.num_nodes, dim, device=cuda, requires_grad=True)
        conv = maxk_layers.MaxKSAGEConv(dim, 48).to(cuda)
        xs, v, i = maxk_layers.maxk(x, k)
        return conv(g, xs, v, i), [x, conv.fc_neigh.weight, conv.fc_self.weight, conv.fc_self.bias]
    _compare(run, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("norm", ["both", "right", "left", "none"])
def test_gcn_conv(cuda, norm):
    import maxk_layers

    def run(g):
        x = torch.randn(g.num_nodes, 64, device=cuda, requires_grad=True)
        conv = maxk_layers.MaxKGraphConv(64, 32, norm=norm).to(cuda)
        xs, v, i = maxk_layers.maxk(x, 16)
        return conv(g, xs, v, i), [x, conv.weight, conv.bias]
    _compare(run, cuda)


@pytest.mark.gpu
def test_gin_conv(cuda):
    import maxk_layers

    def run(g):
        x = torch.randn(g.num_nodes, 64, device=cuda, requires_grad=True)
        mlp = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(),
                                  torch.nn.Linear(64, 32)).to(cuda)
        conv = maxk_layers.MaxKGINConv(mlp, init_eps=0.1, learn_eps=True).to(cuda)
        xs, v, i = maxk_layers.maxk(x, 16)
        return conv(g, xs, v, i), [x, conv.eps, mlp[0].weight, mlp[2].weight]
    _compare(run, cuda)


@pytest.mark.gpu
def test_sage_model_training_step(cuda):
    import maxk_layers

    def run(g):
        x = torch.randn(g.num_nodes, 100, device=cuda)
        model = maxk_layers.MaxKSAGE(100, 128, 3, 10, maxk=16, norm=True,
                                     feat_drop=0.0).to(cuda)
        return model(g, x), [model.lin_in.weight, model.layers[0].fc_neigh.weight,
                             model.layers[2].fc_self.weight, model.lin_out.weight]
    _compare(run, cuda)
    # a few SGD steps on a fixed target reduce the loss through the HIP path
    g = _graph(cuda, seed=3)
    torch.manual_seed(3)
    x = torch.randn(g.num_nodes, 100, device=cuda)
    y = torch.randint(0, 10, (g.num_nodes,), device=cuda)
    model = maxk_layers.MaxKSAGE(100, 128, 2, 10, maxk=16, feat_drop=0.0).to(cuda)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    losses = []
    for _ in range(20):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(g, x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.8 * losses[0], losses


@pytest.mark.gpu
def test_train_bench_matches_library(cuda):
    """One epoch of the 3-layer MaxK-SAGE on the HIP aggregation and on rocSPARSE
    (torch.sparse CSR): same first loss (BASELINE configs[2] driver, small graph)."""
    import maxk_train_bench
    out = maxk_train_bench.main(["flickr", "--hidden", "64", "--k", "16", "--epochs", "1",
                                 "--warmup", "1"])
    assert out["loss_match"], out
    assert out["maxk_epoch_ms"] > 0 and out["library_epoch_ms"] > 0


@pytest.mark.gpu
def test_train_bench_products_epoch(cuda):
    """BASELINE.json configs[2] at its real shape: the 3-layer MaxK-SAGE
    (hidden 256, k = 32) on the ogbn-products-sized graph (V = 2,449,029, E = 123.7M), two
    epochs on the HIP aggregation and two on rocSPARSE from the same weights: the first loss
    (forward) within 1e-4 and the second (after an Adam step on each side's gradients) within
    1e-3."""
    import maxk_train_bench
    out = maxk_train_bench.main(["products", "--k", "32", "--epochs", "2", "--warmup", "0"])
    assert out["V"] == 2449029 and out["hidden"] == 256 and out["layers"] == 3
    assert out["loss_match"], out
    assert out["last_loss_match"], out


@pytest.mark.gpu
@pytest.mark.parametrize("model_cls", ["MaxKGCN", "MaxKGIN"])
def test_gcn_gin_models(cuda, model_cls):
    """The GCN / GIN models (model_integrated_v3.py:590-752) on the HIP aggregation vs the
    dense one: outputs and the weights of every stage."""
    import maxk_layers

    def run(g):
        x = torch.randn(g.num_nodes, 100, device=cuda)
        model = getattr(maxk_layers, model_cls)(100, 64, 2, 10, maxk=16, feat_drop=0.0,
                                                norm=True).to(cuda)
        return model(g, x), [model.lin_in.weight, model.linlayers[0].weight,
                             model.linlayers[1].weight, model.lin_out.weight]
    _compare(run, cuda)


@pytest.mark.gpu
def test_dropout_reaches_the_aggregated_values(cuda):
    """Fixed mode: with feat_drop active the aggregation sees the dropped features (the
    CBSR of dropout(x_sparse)); reference_compat aggregates the undropped top-k values."""
    import maxk_layers
    g = _graph(cuda, seed=5)
    x = torch.randn(g.num_nodes, 64, device=cuda)
    xs, v, i = maxk_layers.maxk(x, 16)
    for compat in (False, True):
        conv = maxk_layers.MaxKSAGEConv(64, 32, feat_drop=0.5, reference_compat=compat).to(cuda)
        torch.manual_seed(0)
        out = conv(g, xs, v, i)
        torch.manual_seed(0)
        xd = torch.nn.functional.dropout(xs, 0.5, training=True)
        vals = xd.gather(1, i.long()) if not compat else v
        agg = DenseGraph(g).aggregate(vals, i, 64, row_div=g.in_degrees.clamp(min=1.0))
        ref = conv.fc_self(xd) + conv.fc_neigh(agg)
        torch.testing.assert_close(out, ref, rtol=RTOL, atol=ATOL)


# ---- reference_compat: the reference's caller behaviour, restated densely from its lines ----

def _dense_adj(g):
    V = g.num_nodes
    A = torch.zeros(V, V, device=g.values.device)
    A.index_put_((g.edge_rows().long(), g.indices.long()), g.values, accumulate=True)
    return A


def _ref_optmaxk(x, k):
    """OPTMaxK (model_integrated_v3.py:28-43): topk_values carry no gradient to x."""
    tv, ti = x.topk(k, dim=1)
    mask = torch.zeros_like(x).scatter(1, ti, 1.0)
    return x * mask, tv.detach(), ti


def _ref_spmm(A, tv, ti, D, deg):
    """MaxKSpmmWrapper.spmm with degrees (spgemmfunction_v4): A . scatter(topk) / degrees."""
    x = torch.zeros(A.shape[0], D, device=A.device).scatter(1, ti, tv)
    return (A @ x) / deg[:, None]


@pytest.mark.gpu
def test_maxk_reference_compat_drops_topk_grad(cuda):
    import maxk_layers
    x = torch.randn(300, 64, device=cuda, requires_grad=True)
    dense, vals, idx = maxk_layers.maxk(x, 8, reference_compat=True)
    mask = torch.zeros_like(x).scatter(1, idx.long(), 1.0)
    w1, w2 = torch.randn_like(x), torch.randn(300, 8, device=cuda)
    ((dense * w1).sum() + (vals * w2).sum()).backward()
    torch.testing.assert_close(x.grad, w1 * mask)  # OPTMaxK.backward: grad_output * mask


@pytest.mark.gpu
@pytest.mark.parametrize("norm", ["both", "right", "left", "none"])
def test_gcn_conv_reference_compat(cuda, norm):
    """:301-310 left norm on feat_src (unused by the kernel), :341-348 kernel on the raw
    topk_values divided by in-degree then @ weight, :381-389 right norm, :392 bias."""
    import maxk_layers
    g = _graph(cuda, seed=1)
    A, deg = _dense_adj(g), g.in_degrees.clamp(min=1.0)
    x = torch.randn(g.num_nodes, 64, device=cuda, requires_grad=True)
    conv = maxk_layers.MaxKGraphConv(64, 64, norm=norm, reference_compat=True).to(cuda)
    torch.nn.init.normal_(conv.bias)
    xs, v, i = maxk_layers.maxk(x, 16, reference_compat=True)
    out = conv(g, xs, v, i)
    x2 = x.detach().clone().requires_grad_(True)
    _, tv, ti = _ref_optmaxk(x2, 16)
    ref = _ref_spmm(A, tv, ti, 64, deg) @ conv.weight
    if norm in ("right", "both"):
        ref = ref * (deg.pow(-0.5) if norm == "both" else 1.0 / deg)[:, None]
    ref = ref + conv.bias
    torch.testing.assert_close(out, ref, rtol=RTOL, atol=ATOL)
    gout = torch.randn_like(out)
    gw = torch.autograd.grad(out, conv.weight, gout, retain_graph=True)[0]
    gw_ref = torch.autograd.grad(ref, conv.weight, gout)[0]
    torch.testing.assert_close(gw, gw_ref, rtol=RTOL, atol=ATOL)


@pytest.mark.gpu
def test_gin_conv_reference_compat(cuda):
    """:491-495 the "sum" call passes the degrees: (1 + eps) x + mean of the neighbours."""
    import maxk_layers
    g = _graph(cuda, seed=2)
    A, deg = _dense_adj(g), g.in_degrees.clamp(min=1.0)
    x = torch.randn(g.num_nodes, 64, device=cuda)
    conv = maxk_layers.MaxKGINConv(None, init_eps=0.25, reference_compat=True).to(cuda)
    xs, v, i = maxk_layers.maxk(x, 16, reference_compat=True)
    ref = 1.25 * xs + _ref_spmm(A, v, i.long(), 64, deg)
    torch.testing.assert_close(conv(g, xs, v, i), ref, rtol=RTOL, atol=ATOL)


@pytest.mark.gpu
@pytest.mark.parametrize("model_cls", ["MaxKSAGE", "MaxKGCN", "MaxKGIN"])
def test_models_reference_compat(cuda, model_cls):
    """Each model with reference_compat=True against a dense restatement of the reference's
    forward (model_integrated_v3.py:569-588 / 644-670 / 726-752, OPTMaxK, the wrapper's
    degree division): outputs and every weight gradient, including the ones the reference's
    dropped top-k gradient leaves at zero (MaxKGCN's lin_in and per-layer Linears)."""
    import maxk_layers
    g = _graph(cuda, seed=4)
    A, deg = _dense_adj(g), g.in_degrees.clamp(min=1.0)
    torch.manual_seed(4)
    x = torch.randn(g.num_nodes, 100, device=cuda)
    model = getattr(maxk_layers, model_cls)(100, 64, 2, 10, maxk=16, feat_drop=0.0,
                                            reference_compat=True).to(cuda)
    out = model(g, x)
    P = dict(model.named_parameters())

    def lin(t, name):
        return torch.nn.functional.linear(t, P[name + ".weight"], P.get(name + ".bias"))

    if model_cls == "MaxKSAGE":  # :575-586, MaxKSAGEConv :152-192
        h = lin(x, "lin_in")
        for li in range(2):
            xs, tv, ti = _ref_optmaxk(h, 16)
            h = lin(xs, f"layers.{li}.fc_self") + lin(_ref_spmm(A, tv, ti, 64, deg),
                                                      f"layers.{li}.fc_neigh")
    else:  # :649-669 / :731-751
        h = lin(x, "lin_in").relu()
        for li in range(2):
            h = lin(h, f"linlayers.{li}")
            xs, tv, ti = _ref_optmaxk(h, 16)
            if model_cls == "MaxKGCN":  # norm "both", no weight, no bias
                h = _ref_spmm(A, tv, ti, 64, deg) * deg.pow(-0.5)[:, None]
            else:  # GIN "sum" as called: a mean; eps starts at 0
                h = (1 + P[f"convs.{li}.eps"]) * xs + _ref_spmm(A, tv, ti, 64, deg)
    ref = lin(h, "lin_out")
    torch.testing.assert_close(out, ref, rtol=RTOL, atol=ATOL)
    gout = torch.randn_like(out)
    names = [n for n in P if P[n].requires_grad]
    ga = torch.autograd.grad(out, [P[n] for n in names], gout, retain_graph=True,
                             allow_unused=True)
    gb = torch.autograd.grad(ref, [P[n] for n in names], gout, allow_unused=True)
    for n, a, b in zip(names, ga, gb):
        a = torch.zeros_like(P[n]) if a is None else a
        b = torch.zeros_like(P[n]) if b is None else b
        torch.testing.assert_close(a, b, rtol=RTOL, atol=ATOL, msg=lambda m: f"{n}: {m}")
    if model_cls == "MaxKGCN":
        gi = ga[names.index("lin_in.weight")]
        assert gi is None or not gi.any()  # the reference trains only lin_out here
