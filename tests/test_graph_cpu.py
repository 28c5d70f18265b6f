"""On-disk graph format + preprocessing (maxk_graph), against the reference's semantics
(dataset_gen.py:59-115, graph_loader.py:19-85) restated as plain Python sets here."""
import os

import numpy as np
import pytest
import torch

import conftest  # noqa: F401  (sys.path)
import maxk_graph as mg


def _reference_edges(src, dst, V):
    """dataset_gen.py:59-101: reverse edges added, a self loop on every vertex, duplicates
    dropped (the reference's edge_set loop)."""
    s = list(src) + list(dst) + list(range(V))
    d = list(dst) + list(src) + list(range(V))
    return sorted(set(zip(s, d)))


def _csr_edges(indptr, indices):
    indptr, indices = np.asarray(indptr), np.asarray(indices)
    rows = np.repeat(np.arange(indptr.size - 1), np.diff(indptr))
    return list(zip(rows.tolist(), indices.tolist()))


@pytest.mark.parametrize("V,m,seed", [(1, 0, 0), (7, 20, 1), (300, 2000, 2)])
def test_build_csr_matches_reference_pipeline(V, m, seed):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, V, m)
    dst = rng.integers(0, V, m)
    if m:
        src[:3], dst[:3] = src[0], dst[0]  # multi-edges
        dst[3] = src[3]                    # an existing self loop
    indptr, indices = mg.build_csr(torch.from_numpy(src), torch.from_numpy(dst), V)
    assert indptr.dtype == torch.int32 and indices.dtype == torch.int32
    assert _csr_edges(indptr, indices) == _reference_edges(src.tolist(), dst.tolist(), V)
    # columns sorted inside each row, every vertex has its self loop
    ip, ix = indptr.numpy(), indices.numpy()
    for r in range(V):
        row = ix[ip[r]:ip[r + 1]]
        assert (np.diff(row) > 0).all() and r in row


def test_build_csr_options():
    src = torch.tensor([0, 0, 2])
    dst = torch.tensor([1, 1, 0])
    ip, ix = mg.build_csr(src, dst, 3, symmetrize=False, self_loops=False, dedupe=False)
    assert _csr_edges(ip, ix) == [(0, 1), (0, 1), (2, 0)]
    ip, ix = mg.build_csr(src, dst, 3, symmetrize=False, self_loops=False)
    assert _csr_edges(ip, ix) == [(0, 1), (2, 0)]
    with pytest.raises(ValueError):
        mg.build_csr(torch.tensor([0]), torch.tensor([3]), 3)


def test_save_load_roundtrip(tmp_path):
    rng = np.random.default_rng(5)
    ip, ix = mg.build_csr(torch.from_numpy(rng.integers(0, 50, 400)),
                          torch.from_numpy(rng.integers(0, 50, 400)), 50)
    mg.save_graph(ip, ix, str(tmp_path), "toy")
    # raw int32 files, no header (dataset_gen.py:109-110)
    assert os.path.getsize(tmp_path / "toy.indptr") == 4 * 51
    assert os.path.getsize(tmp_path / "toy.indices") == 4 * ix.numel()
    g = mg.GraphDataLoader(str(tmp_path)).load_graph("toy.dgl")  # extension stripped (:49)
    assert g["graph_name"] == "toy" and g["v_num"] == 50 and g["e_num"] == ix.numel()
    np.testing.assert_array_equal(g["indptr"], ip.numpy())
    np.testing.assert_array_equal(g["indices"], ix.numpy())
    np.random.seed(123)
    np.testing.assert_array_equal(g["values"],
                                  np.random.uniform(0, 1, ix.numel()).astype(np.float32))
    t = mg.GraphDataLoader(str(tmp_path)).to_cuda_tensors(g, device="cpu")
    assert t["indptr"].dtype == torch.int32 and t["values"].dtype == torch.float32
    assert mg.find_graph("toy", [str(tmp_path)]) == str(tmp_path)
    assert mg.find_graph("missing", [str(tmp_path)]) is None


def test_loader_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        mg.GraphDataLoader(str(tmp_path)).load_graph("nope")
    np.array([0, 2, 1], dtype=np.int32).tofile(tmp_path / "bad.indptr")
    np.array([0, 1], dtype=np.int32).tofile(tmp_path / "bad.indices")
    with pytest.raises(ValueError):
        mg.GraphDataLoader(str(tmp_path)).load_graph("bad")
    np.array([0, 1], dtype=np.int32).tofile(tmp_path / "oob.indptr")
    np.array([7], dtype=np.int32).tofile(tmp_path / "oob.indices")
    with pytest.raises(ValueError):
        mg.GraphDataLoader(str(tmp_path)).load_graph("oob")


@pytest.mark.gpu
def test_build_csr_on_device_matches_cpu(cuda):
    rng = np.random.default_rng(9)
    src, dst = rng.integers(0, 5000, 60000), rng.integers(0, 5000, 60000)
    a = mg.build_csr(torch.from_numpy(src), torch.from_numpy(dst), 5000)
    b = mg.build_csr(torch.from_numpy(src).to(cuda), torch.from_numpy(dst).to(cuda), 5000)
    assert torch.equal(a[0], b[0].cpu()) and torch.equal(a[1], b[1].cpu())


def test_synthetic_generator_properties():
    """make_graph (bench / maxk_kernel_test stand-ins): exact E, symmetric, self loop on every
    vertex, no duplicates, sorted columns."""
    V, E = 3000, 3000 + 2 * 25000
    ip, ix = mg.make_graph(V, E, 0.7, 30, 1, torch.device("cpu"))
    assert ip.dtype == torch.int32 and ix.dtype == torch.int32 and ix.numel() == E
    edges = set(_csr_edges(ip, ix))
    assert len(edges) == E
    assert all((d, s) in edges for s, d in edges)
    assert all((v, v) in edges for v in range(V))
    ipn, ixn = ip.numpy(), ix.numpy()
    assert all((np.diff(ixn[ipn[r]:ipn[r + 1]]) > 0).all() for r in range(V))
    deg = np.diff(ipn)
    assert deg.max() > 5 * deg.mean()  # power-law skew
    ip2, ix2 = mg.make_graph(V, E, 0.7, 30, 1, torch.device("cpu"))
    assert torch.equal(ip, ip2) and torch.equal(ix, ix2)  # seeded


@pytest.mark.gpu
def test_kernel_test_cli(cuda, capsys):
    import maxk_kernel_test
    res = maxk_kernel_test.main(["flickr", "--k", "16", "32", "--dim", "64", "--warmup", "1",
                                 "--runs", "3", "--json"])
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "num graph dim_origin dim_k kernel time(ms)"
    assert out[1].startswith("1/1 flickr 64 16 cusparse ")
    assert [r["k"] for r in res] == [16, 32]
    assert all(r["max_rel_err"] < 1e-3 and r["maxk_ms"] > 0 for r in res)


# ---- planted communities and the locality order (maxk_graph.community_graph etc.) ----------

def test_community_graph_shape():
    import maxk_graph
    V, E = 3000, 3000 + 2 * 30000
    ip, ix = maxk_graph.community_graph(V, E, 0.75, 30, 10, 0.9, 1, torch.device("cpu"))
    assert ip.numel() == V + 1 and int(ip[-1]) == E == ix.numel()
    rows = torch.repeat_interleave(torch.arange(V), torch.diff(ip.long()))
    key = rows * V + ix.long()
    assert bool((key[1:] > key[:-1]).all())  # sorted columns, no multi-edges
    rev = torch.sort(ix.long() * V + rows).values
    assert torch.equal(rev, key)  # symmetric
    assert int((rows == ix.long()).sum()) == V  # one self loop per vertex


def test_permute_graph_relabels_rows_columns_and_values():
    import maxk_graph
    g = torch.Generator().manual_seed(3)
    V = 200
    ip, ix = maxk_graph.build_csr(torch.randint(0, V, (900,), generator=g),
                                  torch.randint(0, V, (900,), generator=g), V)
    val = torch.rand(ix.numel(), generator=g)
    perm = torch.randperm(V, generator=g)
    ip2, ix2, ep = maxk_graph.permute_graph(ip, ix, perm)

    def dense(p, x, v):
        A = torch.zeros(V, V)
        A[torch.repeat_interleave(torch.arange(V), torch.diff(p.long())), x.long()] = v
        return A
    A, A2 = dense(ip, ix, val), dense(ip2, ix2, val[ep])
    assert torch.equal(A2, A[perm][:, perm])  # row/column i of the result is vertex perm[i]


def test_locality_order_groups_planted_communities():
    import maxk_graph
    V, E, C = 4000, 4000 + 2 * 60000, 8
    ip, ix = maxk_graph.community_graph(V, E, 0.75, 30, C, 0.95, 2, torch.device("cpu"))
    perm = maxk_graph.locality_order(ip, ix)
    assert torch.equal(torch.sort(perm).values, torch.arange(V))
    ip2, ix2, _ = maxk_graph.permute_graph(ip, ix, perm)
    rows = torch.repeat_interleave(torch.arange(V), torch.diff(ip.long()))
    rows2 = torch.repeat_interleave(torch.arange(V), torch.diff(ip2.long()))
    near = lambda r, c: float(((r - c.long()).abs() < V // C).float().mean())  # noqa: E731
    assert near(rows2, ix2) > 0.85 > 0.35 > near(rows, ix)


@pytest.mark.gpu
def test_pull_locality(cuda):
    """maxk_pull_locality (C ABI, one kernel pass): a community graph in locality order has
    far more edges per occupied (row, bucket) than randomly labelled."""
    import maxk_cuda_kernels as mk
    import maxk_graph
    V, E = 4000, 4000 + 2 * 60000
    ip, ix = maxk_graph.community_graph(V, E, 0.75, 30, 8, 0.95, 2, torch.device("cpu"))
    rnd = mk.pull_locality(ip.to(cuda), ix.to(cuda), 7)
    ip2, ix2, _ = maxk_graph.permute_graph(ip, ix, maxk_graph.locality_order(ip, ix))
    ordered = mk.pull_locality(ip2.to(cuda), ix2.to(cuda), 7)
    assert ordered > 2 * rnd
    # one row, columns 0..9 and 200..204 -> buckets of 128: {0}, {1}: 15 edges in 2 pairs
    one = torch.tensor([0, 15], dtype=torch.int32, device=cuda)
    cols = torch.tensor(list(range(10)) + list(range(200, 205)), dtype=torch.int32, device=cuda)
    assert mk.pull_locality(one, cols, 7) == 7.5
