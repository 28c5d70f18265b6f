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
@pytest.mark.parametrize("dim,k", [(64, 8), (256, 32)])
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
        model = maxk_layers.MaxKSAGE(100, 128, 10, num_layers=3, maxk=16, norm=True).to(cuda)
        return model(g, x), [model.lin_in.weight, model.layers[0].fc_neigh.weight,
                             model.layers[2].fc_self.weight, model.lin_out.weight]
    _compare(run, cuda)
    # a few SGD steps on a fixed target reduce the loss through the HIP path
    g = _graph(cuda, seed=3)
    torch.manual_seed(3)
    x = torch.randn(g.num_nodes, 100, device=cuda)
    y = torch.randint(0, 10, (g.num_nodes,), device=cuda)
    model = maxk_layers.MaxKSAGE(100, 128, 10, num_layers=2, maxk=16).to(cuda)
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
