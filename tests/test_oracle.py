"""CPU: the oracle (oracle/maxk_oracle.c) against the reference's own outputs.

Pins the restatement before anything is compared with it: tests/golden/*.npz
were produced by the reference's maxk_spgemm_function (forward + autograd
gradient) and generate_meta_csc (warp4) -- see tests/golden/make_golden.py.
"""
import numpy as np
import pytest

import oracle as O
from conftest import golden_cases, load_golden

CASES = golden_cases()
TOL = 1e-4  # |a - b| <= TOL * max(1, |ref|)  (north_star: 1e-4 fp32)


def close(a, ref, tol=TOL):
    err = np.abs(a.astype(np.float64) - ref.astype(np.float64))
    return bool(np.all(err <= tol * np.maximum(1.0, np.abs(ref))))


def test_golden_present():
    assert len(CASES) >= 8


@pytest.mark.parametrize("path", CASES, ids=lambda p: p.split("/")[-1][:-4])
def test_topk_matches_torch_topk(path):
    z = load_golden(path)
    v, i = O.topk(z["x"], int(z["k"]))
    assert np.array_equal(i, z["topk_idx"])
    assert np.array_equal(v, z["topk_val"])


@pytest.mark.parametrize("path", CASES, ids=lambda p: p.split("/")[-1][:-4])
def test_forward_matches_reference(path):
    z = load_golden(path)
    y = O.spgemm_fwd(z["row_ptr"], z["col_idx"], z["val"], z["topk_val"], z["topk_idx"],
                     int(z["D"]), row_div=z["deg"])
    assert close(y, z["y_ref"])


@pytest.mark.parametrize("path", CASES, ids=lambda p: p.split("/")[-1][:-4])
def test_backward_matches_reference_autograd(path):
    z = load_golden(path)
    gs = O.sspmm_bwd(z["row_ptr"], z["col_idx"], z["val"], z["g"], z["topk_idx"], row_div=z["deg"])
    assert close(gs, z["grad_cbsr_ref"])
    tp, ts, tv = O.transpose_csr(z["row_ptr"], z["col_idx"], z["val"])
    gp = O.sspmm_bwd_pull(tp, ts, tv, z["g"], z["topk_idx"], row_div=z["deg"])
    assert close(gp, gs, 1e-6)
    V = z["row_ptr"].size - 1
    tc = O.transpose(z["row_ptr"], z["col_idx"], z["val"], V)  # the C counting sort
    assert all(np.array_equal(a, b) for a, b in zip(tc, (tp, ts, tv)))
    dense = O.scatter_dense(gs, z["topk_idx"], int(z["D"]))
    assert np.array_equal(np.take_along_axis(dense, z["topk_idx"].astype(np.int64), 1), gs)
    assert np.count_nonzero(dense) <= gs.size


@pytest.mark.parametrize("path", CASES, ids=lambda p: p.split("/")[-1][:-4])
def test_warp4_matches_reference(path):
    z = load_golden(path)
    assert np.array_equal(O.warp4(z["row_ptr"], 64), z["warp4_ref"])


def test_backward_reference_divisor_rule():
    """asym_outdeg_d256_k16: in- and out-degrees differ; the reference's v1 backward rule
    (grad_output / out_degrees through A^T, maxk_spgemm_function.py:154-175) is the oracle's
    backward with row_div = out_degrees, and differs from the exact adjoint there."""
    import os
    from conftest import GOLDEN
    z = load_golden(os.path.join(GOLDEN, "asym_outdeg_d256_k16.npz"))
    gs = O.sspmm_bwd(z["row_ptr"], z["col_idx"], z["val"], z["g"], z["topk_idx"],
                     row_div=z["out_deg"])
    assert close(gs, z["grad_cbsr_refrule"])
    assert not close(gs, z["grad_cbsr_ref"])


def test_oracle_adjoint_identity():
    """<A.scatter(v), G> == <v, gather(A^T G)>: forward and backward are adjoint."""
    z = load_golden(CASES[0])
    rng = np.random.default_rng(3)
    k, D = int(z["k"]), int(z["D"])
    V = z["row_ptr"].size - 1
    v = rng.standard_normal((V, k)).astype(np.float32)
    g = rng.standard_normal((V, D)).astype(np.float32)
    y = O.spgemm_fwd(z["row_ptr"], z["col_idx"], z["val"], v, z["topk_idx"], D)
    gs = O.sspmm_bwd(z["row_ptr"], z["col_idx"], z["val"], g, z["topk_idx"])
    a = float(np.dot(y.ravel().astype(np.float64), g.ravel()))
    b = float(np.dot(v.ravel().astype(np.float64), gs.ravel()))
    assert abs(a - b) <= 1e-4 * max(1.0, abs(a))


def test_oracle_row_range_sample():
    z = load_golden(CASES[0])
    D = int(z["D"])
    full = O.spgemm_fwd(z["row_ptr"], z["col_idx"], z["val"], z["topk_val"], z["topk_idx"], D)
    part = O.spgemm_fwd(z["row_ptr"], z["col_idx"], z["val"], z["topk_val"], z["topk_idx"], D,
                        rows=(10, 50))
    assert np.array_equal(part[10:50], full[10:50])
    assert not part[:10].any() and not part[50:].any()


def test_topk_tail_fixture_pins_the_oracle():
    """tests/golden/topk/topk_tail_overflow.npz (tools/make_topk_tail_fixture.py): the rows of
    the seed-0 Gaussian input behind r02's four-row k=48 mismatch, with their top-k as the
    oracle computed them on the box; the oracle here reproduces them bit for bit, and they
    agree with numpy's stable descending sort (ties to the lower column)."""
    import os
    from conftest import GOLDEN
    z = load_golden(os.path.join(GOLDEN, "topk", "topk_tail_overflow.npz"))
    for k in (16, 32, 48, 64):
        v, i = O.topk(z["x"], k)
        assert np.array_equal(v, z[f"val_k{k}"]) and np.array_equal(i, z[f"idx_k{k}"])
        order = np.argsort(-z["x"], axis=1, kind="stable")[:, :k]
        assert np.array_equal(order.astype(np.uint8), i)


def test_topk_u8_reference_restatement():
    """The reference's uint8 top-k, by hand on one row (kernels/maxk_kernel.cu:21-90): the
    threshold after 8 bisection steps is 179 for k = 4; the picks > 179 in ascending columns are
    3, 31, 40, 63, but the pick in column 31 (lane 31 of the first 32-column step) is not
    counted and is overwritten by the next step's first pick (column 40); the last slot stays
    0."""
    x = np.zeros((2, 256), np.uint8)
    x[0, [3, 31, 40, 63, 100]] = [200, 250, 180, 220, 90]
    x[1, :] = np.arange(256)[::-1]  # 255 .. 0: the first k columns are the largest
    v, i = O.topk_u8_reference(x, 4)
    assert v[0].tolist() == [200, 180, 220, 0] and i[0].tolist() == [3, 40, 63, 0]
    assert i[1].tolist() == [0, 1, 2, 3] and v[1].tolist() == [255, 254, 253, 252]


def test_topk_u8_as_built_model():
    """The CUDA kernel as built (oracle.topk_u8_reference_as_built): every warp
    takes its threshold from the block's first row, per lane.  By hand: a block whose first row
    is all zero bisects every lane's mid down to 0, so row 1 (255 .. 0) picks every nonzero byte
    in column order -- columns 0..30, then column 32 over lane 31's uncounted pick -- while its
    own threshold (the intended convention) would pick its 32 largest; row 0 picks nothing.
    On uniform bytes the two conventions disagree on most rows, which is why the product keeps
    the intended one (reference_compat) and calls parity with the CUDA kernel unpinned."""
    x = np.zeros((16, 256), np.uint8)
    x[1] = np.arange(256)[::-1]
    x[2:] = np.random.default_rng(0).integers(0, 256, (14, 256), dtype=np.uint8)
    v, i, w = O.topk_u8_reference_as_built(x, 32)
    assert not w[0].any()
    assert i[1].tolist() == list(range(31)) + [32] and w[1].all()
    assert v[1].tolist() == list(range(255, 224, -1)) + [223]
    vi, ii = O.topk_u8_reference(x, 32)
    assert ii[1].tolist() != i[1].tolist()
    with pytest.raises(ValueError):
        O.topk_u8_reference_as_built(x, 16)
    u = np.random.default_rng(1).integers(0, 256, (256, 256), dtype=np.uint8)
    va, ia, wa = O.topk_u8_reference_as_built(u, 32)
    vi, ii = O.topk_u8_reference(u, 32)
    differ = np.mean([not (np.array_equal(ia[r][wa[r]], ii[r][:wa[r].sum()]) and wa[r].all())
                      for r in range(256)])
    assert differ > 0.5, differ
