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
