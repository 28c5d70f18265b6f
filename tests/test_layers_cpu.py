"""maxk_layers host logic without a GPU: argument checks, graph bookkeeping, and that the
aggregation refuses CPU tensors (no CPU fallback on the product path)."""
import pytest
import torch

import conftest  # noqa: F401  (sys.path)
import maxk_layers


def _toy():
    # 0 <- {0,1}, 1 <- {0,1,2}, 2 <- {2}
    return maxk_layers.CSRGraph(torch.tensor([0, 2, 5, 6]), torch.tensor([0, 1, 0, 1, 2, 2]))


def test_csr_graph_degrees():
    g = _toy()
    assert g.num_nodes == 3
    assert g.in_degrees.tolist() == [2.0, 3.0, 1.0]
    assert g.out_degrees.tolist() == [2.0, 2.0, 2.0]
    assert g.edge_rows().tolist() == [0, 0, 1, 1, 1, 2]
    assert torch.equal(g.values, torch.ones(6))


def test_gcn_norm_values():
    g = _toy()
    conv = maxk_layers.MaxKGraphConv(4, 2, norm="both")
    v = conv._norm_values(g)
    exp = [(2 * 2) ** -0.5, (2 * 2) ** -0.5, (3 * 2) ** -0.5, (3 * 2) ** -0.5, (3 * 2) ** -0.5,
           (1 * 2) ** -0.5]
    torch.testing.assert_close(v, torch.tensor(exp))
    torch.testing.assert_close(maxk_layers.MaxKGraphConv(4, 2, norm="right")._norm_values(g),
                               torch.tensor([.5, .5, 1 / 3, 1 / 3, 1 / 3, 1.]))
    torch.testing.assert_close(maxk_layers.MaxKGraphConv(4, 2, norm="left")._norm_values(g),
                               torch.full((6,), 0.5))
    with pytest.raises(ValueError):
        maxk_layers.MaxKGraphConv(4, 2, norm="sym")


def test_aggregation_refuses_cpu_tensors():
    g = _toy()
    vals = torch.rand(3, 2)
    idx = torch.tensor([[0, 1], [2, 3], [1, 0]], dtype=torch.uint8)
    with pytest.raises(RuntimeError):
        g.aggregate(vals, idx, 4)
    with pytest.raises(RuntimeError):
        maxk_layers.maxk(torch.rand(3, 4), 2)


@pytest.mark.parametrize("n", [1000, 256 * 1024 + 37])
def test_linear_tall_gradients_match_nn_linear(n):
    """_Linear (single and the SAGE fc_self + fc_neigh pair) against nn.Linear autograd,
    including the chunked weight / bias gradients used for N >= 256 * 1024 rows."""
    import maxk_layers as L
    torch.manual_seed(0)
    a, b = torch.nn.Linear(6, 5), torch.nn.Linear(6, 5, bias=False)
    x1 = torch.randn(n, 6, dtype=torch.float64, requires_grad=True)
    x2 = torch.randn(n, 6, dtype=torch.float64, requires_grad=True)
    a, b = a.double(), b.double()
    g = torch.randn(n, 5, dtype=torch.float64)
    ref = a(x1) + b(x2)
    ref_grads = torch.autograd.grad(ref, [x1, x2, a.weight, a.bias, b.weight], g)
    out = L.linear(x1, a, x2, b)
    grads = torch.autograd.grad(out, [x1, x2, a.weight, a.bias, b.weight], g)
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-10)
    for got, want in zip(grads, ref_grads):
        assert torch.allclose(got, want, rtol=1e-10, atol=1e-8)
    single = L.linear(x1, a)
    assert torch.allclose(single, a(x1), rtol=1e-12, atol=1e-10)


def test_cross_entropy_matches_torch():
    import maxk_layers as L
    torch.manual_seed(1)
    logits = torch.randn(500, 47, dtype=torch.float64, requires_grad=True)
    y = torch.randint(0, 47, (500,))
    a = L.cross_entropy(logits, y)
    b = torch.nn.functional.cross_entropy(logits, y)
    assert torch.allclose(a, b, rtol=1e-12)
    ga, = torch.autograd.grad(a, logits)
    gb, = torch.autograd.grad(b, logits)
    assert torch.allclose(ga, gb, rtol=1e-10, atol=1e-14)
