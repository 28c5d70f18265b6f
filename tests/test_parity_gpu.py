"""GPU parity: the HIP path (through the C ABI) against the reference's golden
outputs and the pinned CPU oracle.

Tolerances: fp32 outputs |hip - ref| <= 1e-4 * max(1, |ref|) (north_star);
index vectors (top-k selectors, warp4, row_ptr) bit-exact.
"""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden_cases, load_golden

pytestmark = pytest.mark.gpu

CASES = golden_cases()
IDS = [p.split("/")[-1][:-4] for p in CASES]
TOL = 1e-4


def close(a, ref, tol=TOL):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    err = np.abs(a.astype(np.float64) - ref.astype(np.float64))
    bound = tol * np.maximum(1.0, np.abs(ref.astype(np.float64)))
    bad = err > bound
    assert not bad.any(), f"{bad.sum()} elements off; max err {err.max():.3e}"
    return True


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


@pytest.fixture(scope="module")
def mk(cuda):
    import maxk_cuda_kernels
    return maxk_cuda_kernels


@pytest.fixture(scope="module")
def F(cuda):
    import maxk_spgemm_function
    assert maxk_spgemm_function.MAXK_KERNELS_AVAILABLE
    return maxk_spgemm_function


# --------------------------------------------------------------------------- golden
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_topk_bit_exact(mk, cuda, path):
    z = load_golden(path)
    v, i, i32 = mk.topk_cbsr(T(z["x"], cuda), int(z["k"]), with_int32=True)
    assert np.array_equal(i.cpu().numpy(), z["topk_idx"])
    assert np.array_equal(i32.cpu().numpy(), z["topk_idx"].astype(np.int32))
    assert np.array_equal(v.cpu().numpy(), z["topk_val"])


@pytest.mark.parametrize("k", [2, 4, 8, 16, 32])
@pytest.mark.parametrize("D,chunk", [(256, 0), (256, 97), (64, 0)])
def test_forward_dense_small_k(mk, cuda, k, D, chunk):
    """The forward's dense-graph rules (average degree >= 128): 8 lanes per edge at k <= 8
    (fwd_lanes_per_edge; a sparser graph takes 16) and 16 wave steps of loads per batch
    (FwdLayout::deep).  The golden graphs are sparse, so this dense one (average degree ~170,
    one hub row split over items at chunk 97) covers those kernels -- plain, with the degree
    division, and the stream-writing one (which keeps 8 steps) -- against the oracle."""
    rng = np.random.default_rng(1000 + k + D)
    V = 900
    deg = rng.integers(120, 220, V)
    deg[7] = V - 1  # a hub row
    rp = np.zeros(V + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    E = int(rp[-1])
    assert E >= 128 * V
    col = np.concatenate([np.sort(rng.choice(V, int(d), replace=False)) for d in deg]).astype(np.int32)
    val = rng.random(E, dtype=np.float32)
    x = rng.standard_normal((V, D)).astype(np.float32)
    tv, ti = O.topk(x, k)
    div = np.maximum(deg, 1).astype(np.float32)
    ref = O.spgemm_fwd(rp, col, val, tv, ti, D, row_div=div)
    args = (T(rp, cuda), T(col, cuda), T(val, cuda), T(tv, cuda), T(ti, cuda), D)
    close(mk.spgemm_forward(*args, row_div=T(div, cuda), chunk=chunk), ref)
    es = torch.empty(E, k, dtype=torch.uint8, device=cuda)
    close(mk.spgemm_forward(*args, row_div=T(div, cuda), chunk=chunk, edge_sel_out=es), ref)
    assert torch.equal(es, T(ti, cuda)[T(col, cuda).long()])


@pytest.mark.parametrize("k", [8, 16, 24, 32])
@pytest.mark.parametrize("D,chunk", [(256, 0), (256, 97), (64, 0)])
def test_forward_emit_sparse_repeats(mk, cuda, k, D, chunk):
    """The stream-writing forward on a sparse graph with rows past the streaming walker's 64
    edges, a hub row split over items and repeated selectors (which the records fold into
    their first occurrence): its output matches the oracle and the plain call (the plain one
    streams rows, over 5k-byte transport records at k = 24 / 32), and the stream holds the
    caller's selector bytes, repeats included."""
    rng = np.random.default_rng(2000 + k + D + chunk)
    V = 3000
    deg = np.minimum(rng.geometric(1 / 20, V), 300)
    deg[11] = 2500  # a hub row, split over items at chunk 97
    deg[12] = 0
    rp = np.zeros(V + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    E = int(rp[-1])
    assert E < 128 * V  # sparse: the streaming forward
    col = np.concatenate([np.sort(rng.choice(V, int(d), replace=False)) for d in deg]).astype(np.int32)
    val = rng.random(E, dtype=np.float32)
    x = rng.standard_normal((V, D)).astype(np.float32)
    tv, ti = O.topk(x, k)
    dup = rng.random(V) < 0.2
    ti[dup, 1] = ti[dup, 0]  # repeated selectors
    div = np.maximum(deg, 1).astype(np.float32)
    ref = O.spgemm_fwd(rp, col, val, tv, ti, D, row_div=div)
    args = (T(rp, cuda), T(col, cuda), T(val, cuda), T(tv, cuda), T(ti, cuda), D)
    y = mk.spgemm_forward(*args, row_div=T(div, cuda), chunk=chunk)
    close(y, ref)
    es = torch.full((E, k), 0xAB, dtype=torch.uint8, device=cuda)
    ye = mk.spgemm_forward(*args, row_div=T(div, cuda), chunk=chunk, edge_sel_out=es)
    close(ye, ref)
    assert torch.equal(es, T(ti, cuda)[T(col, cuda).long()])


@pytest.mark.parametrize("chunk", [0, 5, 37, 300])
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_forward_golden(mk, cuda, path, chunk):
    z = load_golden(path)
    y = mk.spgemm_forward(T(z["row_ptr"], cuda), T(z["col_idx"], cuda), T(z["val"], cuda),
                          T(z["topk_val"], cuda), T(z["topk_idx"], cuda), int(z["D"]),
                          row_div=T(z["deg"], cuda), chunk=chunk)
    close(y, z["y_ref"])


@pytest.mark.parametrize("chunk", [0, 5, 37])
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_forward_accumulate_golden(mk, cuda, path, chunk):
    """maxk_spgemm_forward_accumulate: the golden graph's edges split into two sub-CSRs by
    column parity (the sharded forward's pipelined parts, maxk_dist); the first product
    written, the second added onto it, must equal the whole graph's (small chunks cut hub
    rows into slabs, whose fixup then adds onto the accumulated rows)."""
    z = load_golden(path)
    rp, col, val = z["row_ptr"], z["col_idx"], z["val"]
    rows = np.repeat(np.arange(rp.size - 1), np.diff(rp))
    parts = []
    for par in (0, 1):
        m = (col % 2) == par
        rpj = np.zeros_like(rp)
        rpj[1:] = np.cumsum(np.bincount(rows[m], minlength=rp.size - 1))
        parts.append((T(rpj, cuda), T(col[m], cuda), T(val[m], cuda)))
    args = (T(z["topk_val"], cuda), T(z["topk_idx"], cuda), int(z["D"]))
    div = T(z["deg"], cuda)
    y = mk.spgemm_forward(*parts[0], *args, row_div=div, chunk=chunk)
    y2 = mk.spgemm_forward(*parts[1], *args, row_div=div, chunk=chunk, out=y, accumulate=True)
    assert y2 is y
    close(y, z["y_ref"])
    # the same, the second part also writing its edge-selector stream
    # (maxk_spgemm_forward_accumulate_sel)
    es = torch.full((parts[1][1].numel(), args[1].shape[1]), 0xAB, dtype=torch.uint8,
                    device=cuda)
    y = mk.spgemm_forward(*parts[0], *args, row_div=div, chunk=chunk)
    mk.spgemm_forward(*parts[1], *args, row_div=div, chunk=chunk, out=y, accumulate=True,
                      edge_sel_out=es)
    close(y, z["y_ref"])
    assert torch.equal(es, args[1][parts[1][1].long()])
    with pytest.raises(RuntimeError):
        mk.spgemm_forward(*parts[1], *args, accumulate=True)  # needs out=


@pytest.mark.parametrize("chunk", [0, 5, 37])
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_edge_selector_stream_golden(mk, cuda, path, chunk):
    """maxk_spgemm_forward_sel writes edge_sel[e] = cbsr_idx[col_idx[e]] beside the unchanged
    forward output (short rows, long rows and hub-row slabs at small chunks), and
    maxk_sspmm_backward_csc_sel reading that stream equals the csc backward bitwise (the same
    contributions, the same sum order) and the fixture.  (The emitting forward walks short
    rows one at a time instead of in batches, which keeps its register use down: its output
    matches the fixture, not the plain call bit for bit.)"""
    z = load_golden(path)
    rp, col, val = T(z["row_ptr"], cuda), T(z["col_idx"], cuda), T(z["val"], cuda)
    cv, ci, D = T(z["topk_val"], cuda), T(z["topk_idx"], cuda), int(z["D"])
    k = ci.shape[1]
    E = col.numel()
    div = T(z["deg"], cuda)
    es = torch.full((E, k), 0xAB, dtype=torch.uint8, device=cuda)
    y = mk.spgemm_forward(rp, col, val, cv, ci, D, row_div=div, chunk=chunk, edge_sel_out=es)
    close(y, z["y_ref"])  # short rows take the one-row path here, so not bitwise the plain call
    assert torch.equal(es, ci[col.long()])
    if k % 4:
        return
    assert torch.equal(mk.edge_selectors(col, ci), es)
    g = T(z["g"], cuda)
    ref = mk.sspmm_backward(rp, col, val, g, ci, row_div=div, chunk=chunk, mode="csc")
    got = mk.sspmm_backward(rp, col, val, g, ci, row_div=div, chunk=chunk, mode="csc",
                            edge_sel=es)
    assert torch.equal(got, ref)
    close(got, z["grad_cbsr_ref"])


@pytest.mark.parametrize("mode", ["auto", "pull", "bsort", "csc", "atomic", "dense"])
@pytest.mark.parametrize("chunk", [0, 5, 37, 300])
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_backward_golden(mk, cuda, path, chunk, mode):
    z = load_golden(path)
    if mode == "bsort" and z["topk_idx"].shape[1] % 4:
        pytest.skip(f"{mode} mode needs k % 4 == 0")
    if mode == "pull" and int(z["D"]) % 4:
        pytest.skip("pull mode needs D % 4 == 0")
    if mode == "dense" and (int(z["D"]) % 4 or z["topk_idx"].shape[1] % 4):
        pytest.skip("dense mode needs D % 4 == 0 and k % 4 == 0")
    gs = mk.sspmm_backward(T(z["row_ptr"], cuda), T(z["col_idx"], cuda), T(z["val"], cuda),
                           T(z["g"], cuda), T(z["topk_idx"], cuda), row_div=T(z["deg"], cuda),
                           chunk=chunk, mode=mode)
    close(gs, z["grad_cbsr_ref"])


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_transpose_plan(mk, cuda, path):
    z = load_golden(path)
    V = z["row_ptr"].size - 1
    col_ptr, eid = mk.transpose_plan(T(z["col_idx"], cuda), V)
    tp, _, _ = O.transpose_csr(z["row_ptr"], z["col_idx"], z["val"])
    assert np.array_equal(col_ptr.cpu().numpy(), tp)
    order = np.argsort(z["col_idx"], kind="stable")  # CSC slot t holds CSR edge order[t]
    assert np.array_equal(eid.cpu().numpy(), order)


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_dense_plan(mk, cuda, path):
    """The dense backward's plan: the transpose plus, per CSC slot, the CSR row of its edge and
    its weight (maxk_dense_plan), checked against numpy."""
    z = load_golden(path)
    V = z["row_ptr"].size - 1
    col_ptr, t_src, t_w = mk.dense_plan(T(z["row_ptr"], cuda), T(z["col_idx"], cuda),
                                        T(z["val"], cuda), V, cache=False)
    order = np.argsort(z["col_idx"], kind="stable")
    rows = np.repeat(np.arange(V), np.diff(z["row_ptr"]))
    tp, _, _ = O.transpose_csr(z["row_ptr"], z["col_idx"], z["val"])
    assert np.array_equal(col_ptr.cpu().numpy(), tp)
    assert np.array_equal(t_src.cpu().numpy(), rows[order])
    assert np.array_equal(t_w.cpu().numpy(), z["val"][order])


def bsort_layout(col, k, shift, W, nb):
    """numpy restatement of maxk_bsort_plan: windows of W CSR edges, each sorted by
    destination bucket (stable); T row p holds edge perm[p]."""
    e = np.arange(col.size)
    perm = np.lexsort((e, np.clip(col >> shift, 0, nb - 1), e // W))
    pos = np.empty(col.size, np.int64)
    pos[perm] = e
    return perm, pos


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_bsort_plan(mk, cuda, path):
    """The window-sorted plan: the bucket plan with T rows in place of edge ids, and per T row
    its edge relative to the window (checked against numpy at the real window and at a forced
    small one through a 16-edge graph slice)."""
    z = load_golden(path)
    V = z["row_ptr"].size - 1
    col = z["col_idx"].astype(np.int64)
    for k in (4, 8, 16, 64):
        bptr, bpos, bdst, wsrc, wrow, shift = mk.bsort_plan(T(z["row_ptr"], cuda),
                                                            T(z["col_idx"], cuda), V, k,
                                                            cache=False)
        assert shift == mk._lib().maxk_bucket_shift(k)
        W = mk._lib().maxk_bsort_window(k)
        assert W == min(65536, 160 * 1024 // (4 * k))
        nb = (V + (1 << shift) - 1) >> shift
        perm, pos = bsort_layout(col, k, shift, W, nb)
        order = np.argsort(col >> shift, kind="stable")
        assert np.array_equal(bptr.cpu().numpy(),
                              np.searchsorted(col[order] >> shift, np.arange(nb + 1)))
        assert np.array_equal(bdst.cpu().numpy().astype(np.int64), col[order] & ((1 << shift) - 1))
        assert np.array_equal(bpos.cpu().numpy(), pos[order])
        assert np.array_equal(wsrc.cpu().numpy().astype(np.int64),
                              perm - np.arange(col.size) // W * W)
        assert np.array_equal(wrow.cpu().numpy(), np.repeat(np.arange(V), np.diff(z["row_ptr"])))
    assert mk._lib().maxk_bsort_window(6) == -1 and mk._lib().maxk_bsort_window(0) == -1


@pytest.mark.filterwarnings("ignore:backward mode 'bsort'")
@pytest.mark.parametrize("k", [1, 8, 16, 32, 64, 100, 256])
def test_topk_u8_reference_convention(mk, cuda, k):
    """cuda_topk_maxk(reference_compat=True): the reference uint8 kernel's own convention
    (threshold bisection, ascending columns, the lane-31 overwrite, zero-filled slots) against
    the oracle's restatement, on uint8 rows with many ties, rows of few distinct values and a
    row of all equal bytes; and the float binding's quantisation round(x * 255)."""
    rng = np.random.default_rng(1000 + k)
    x = rng.integers(0, 256, (700, 256)).astype(np.uint8)
    x[:100] = rng.integers(0, 4, (100, 256)).astype(np.uint8) * 60   # 4 values, heavy ties
    x[100] = 77
    x[101, 31::32] = 255  # every step's lane-31 column the largest
    v, i = mk.cuda_topk_maxk(T(x, cuda), k, reference_compat=True)
    vo, io = O.topk_u8_reference(x, k)
    assert np.array_equal(v.cpu().numpy(), vo) and np.array_equal(i.cpu().numpy(), io)
    xf = rng.random((300, 256), dtype=np.float32) * 1.2 - 0.1
    vf, i32 = mk.cuda_topk_maxk_float(T(xf, cuda), k, reference_compat=True)
    q = np.clip(np.round(xf.astype(np.float32) * np.float32(255.0)), 0, 255).astype(np.uint8)
    vq, iq = O.topk_u8_reference(q, k)
    assert np.array_equal(i32.cpu().numpy(), iq.astype(np.int32))
    assert np.array_equal(vf.cpu().numpy(), vq.astype(np.float32) / np.float32(255.0))


@pytest.mark.parametrize("k", [4, 8, 16, 32, 64, 256])
def test_bsort_windows_against_oracle(mk, cuda, k):
    """Window-sorted backward on a products-like graph of many windows (hub rows cut by window
    and wave boundaries, empty rows, a rectangular column space): equal to the oracle, and the
    edge-selector stream form bitwise equal to the selector-table form (same rows, same
    order)."""
    rng = np.random.default_rng(500 + k)
    R, C, D = 3000, 3500, 256
    row_ptr, col = rand_graph(rng, R, 50, hubs=((5, 3400), (2999, 1200)), empty=40, cols=C)
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((C, D), dtype=np.float32), k)
    g = rng.standard_normal((R, D), dtype=np.float32)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    assert col.size > 10 * mk._lib().maxk_bsort_window(k)
    args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda), T(ci, cuda))
    a = mk.sspmm_backward(*args, row_div=T(div, cuda), mode="bsort")
    close(a, O.sspmm_bwd(row_ptr, col, val, g, ci, row_div=div))
    es = mk.edge_selectors(T(col, cuda), T(ci, cuda))
    b = mk.sspmm_backward(*args, row_div=T(div, cuda), mode="bsort", edge_sel=es)
    assert torch.equal(a, b)


@pytest.mark.parametrize("k", [1, 3, 4, 10, 16, 32])
@pytest.mark.parametrize("offset", [0, 1, 4])
def test_edge_selectors_any_k_and_alignment(mk, cuda, k, offset):
    """maxk_edge_selectors (the forward's stream fallback past 2^24 columns): any k and any
    alignment of both arrays give cbsr_idx[col_idx] (it had required k % 4 == 0 and
    16-B alignment while the _sel entry points accept 4-B aligned streams)."""
    rng = np.random.default_rng(k * 10 + offset)
    C, E = 1000, 20000
    col = T(rng.integers(0, C, E).astype(np.int32), cuda)
    ci_buf = torch.randint(0, 256, (C * k + offset,), dtype=torch.uint8, device=cuda)
    ci = ci_buf[offset:].view(C, k)
    es_buf = torch.zeros(E * k + offset, dtype=torch.uint8, device=cuda)
    es = es_buf[offset:].view(E, k)
    mk.edge_selectors(col, ci, out=es)
    assert torch.equal(es, ci[col.long()])
    assert not es_buf[:offset].any()  # nothing written before the stream


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_pull_plan(mk, cuda, path):
    """Tiles t = slice(row) * nb + bucket(col): per tile the CSR edges in CSR order, with
    their source row, weight and column inside the bucket (checked against numpy)."""
    z = load_golden(path)
    V = z["row_ptr"].size - 1
    col = z["col_idx"].astype(np.int64)
    rows = np.repeat(np.arange(V), np.diff(z["row_ptr"]))
    for k, S in ((4, 1), (16, 3), (16, 50)):
        tptr, ent, shift, s_ = mk.pull_plan(T(z["row_ptr"], cuda), T(z["col_idx"], cuda),
                                            T(z["val"], cuda), V, k, slices=S, cache=False)
        assert s_ == S and shift == mk._lib().maxk_pull_shift(k)
        nb = (V + (1 << shift) - 1) >> shift
        rps = -(-V // S)
        key = (rows // rps) * nb + (col >> shift)
        order = np.argsort(key, kind="stable")
        assert np.array_equal(tptr.cpu().numpy(), np.searchsorted(key[order], np.arange(S * nb + 1)))
        e = ent.cpu().numpy().view(np.uint32)
        assert np.array_equal(e[:, 0] & 0xffff, rows[order] % rps)
        assert np.array_equal(e[:, 0] >> 16, col[order] & ((1 << shift) - 1))
        assert np.array_equal(e[:, 1].view(np.float32), z["val"][order])


def test_pull_plan_follows_values(mk, cuda):
    """The pull plan copies the edge weights: an in-place update of `values` (version
    counter) rebuilds it, a different values tensor gets its own plan."""
    z = load_golden(CASES[2])
    rp, ci, va, g, cs = [T(z[n], cuda).clone() for n in ("row_ptr", "col_idx", "val", "g",
                                                         "topk_idx")]
    a = mk.sspmm_backward(rp, ci, va, g, cs, mode="pull")
    va.mul_(2.0)
    b = mk.sspmm_backward(rp, ci, va, g, cs, mode="pull")
    close(b, 2.0 * a.cpu().numpy())
    c = mk.sspmm_backward(rp, ci, va * 0.5, g, cs, mode="pull")
    close(c, a.cpu().numpy())


@pytest.mark.parametrize("k", [8, 16, 32, 64])
def test_pull_backward_other_shifts(mk, cuda, k):
    """A pull plan built with a bucket shift other than maxk_pull_shift(k) (any shift in
    [4, max(maxk_bucket_shift, maxk_pull_shift)]) runs in a workspace of the documented size
    (maxk_sspmm_backward_pull_workspace_size) -- ADVICE r02: the call used to size its tile
    partials at the largest shift and refuse the documented workspace."""
    z = load_golden(next(c for c in CASES if "sym_d256_k16" in c))
    V = z["row_ptr"].size - 1
    rng = np.random.default_rng(k)
    sel = np.stack([rng.choice(256, k, replace=False) for _ in range(V)]).astype(np.uint8)
    g = rng.standard_normal((V, 256), dtype=np.float32)
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val")]
    ref = O.sspmm_bwd(z["row_ptr"], z["col_idx"], z["val"], g, sel, row_div=z["deg"])
    L = mk._lib()
    top = max(L.maxk_bucket_shift(k), L.maxk_pull_shift(k))
    for shift in sorted({4, L.maxk_bucket_shift(k), L.maxk_pull_shift(k), top - 1}):
        plan = mk.pull_plan(*args, V, k, 256, slices=3, cache=False, shift=shift)
        gs = mk.sspmm_backward(*args, T(g, cuda), T(sel, cuda), row_div=T(z["deg"], cuda),
                               mode="pull", plan=plan)
        close(gs, ref)


def test_pull_backward_repeats(mk, cuda):
    """fp64 tile sums, slices added in a fixed order: two runs agree to fp32 rounding."""
    z = load_golden(CASES[2])
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val", "g", "topk_idx")]
    a = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), mode="pull")
    b = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), mode="pull")
    assert torch.allclose(a, b, rtol=1e-6, atol=0)


@pytest.mark.parametrize("dup", [False, True])
@pytest.mark.parametrize("k", [4, 12, 16, 32, 64, 128])
def test_pull_selector_kernels(mk, cuda, k, dup):
    """The pull's selector ordering runs four selectors per thread (pull_sel4_kernel) on a
    4-byte-aligned selector buffer and one per thread otherwise: both against the oracle, on
    distinct selectors and on rows with repeated ones (ranked by (selector, l))."""
    z = load_golden(next(c for c in CASES if "sym_d256_k16" in c))
    V = z["row_ptr"].size - 1
    rng = np.random.default_rng(k)
    sel = np.stack([rng.choice(256, k, replace=False) for _ in range(V)]).astype(np.uint8)
    if dup:
        sel[::3, 1] = sel[::3, 0]
    g = rng.standard_normal((V, 256), dtype=np.float32)
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val")]
    ref = O.sspmm_bwd(z["row_ptr"], z["col_idx"], z["val"], g, sel)
    aligned = T(sel, cuda)
    raw = torch.empty(V * k + 1, dtype=torch.uint8, device=cuda)
    odd = raw[1:].view(V, k)  # contiguous, one byte off the allocation
    odd.copy_(aligned)
    for cs in (aligned, odd):
        close(mk.sspmm_backward(*args, T(g, cuda), cs, mode="pull"), ref)


@pytest.mark.filterwarnings("ignore:backward mode 'bsort'")
@pytest.mark.parametrize("mode", ["bsort", "pull"])
@pytest.mark.parametrize("k", [8, 16])
def test_bucket_backward_many_parts(mk, cuda, k, mode):
    """A graph large enough that every bucket is cut into many parts (6M edges, parts of
    16384 entries, ~20 parts per bucket): the bucketed phase 2's slab partials and their fixup
    (bsort; r05's plain "bucket" mode ran the same phase 2), and buckets whose parts start and
    end mid-bucket, against the oracle."""
    rng = np.random.default_rng(123 + k)
    V, D, avg = 20000, 256, 300
    deg = rng.poisson(avg, V).astype(np.int64)
    deg[[5, 9999]] = 15000  # hubs
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum(deg, out=row_ptr[1:])
    # sorted random columns per row (vectorised: sort keys row * V + col, duplicates allowed)
    cols = rng.integers(0, V, int(row_ptr[-1]))
    rows = np.repeat(np.arange(V), deg)
    col = cols[np.lexsort((cols, rows))].astype(np.int32)
    row_ptr = row_ptr.astype(np.int32)
    val = rng.random(col.size, dtype=np.float32)
    _, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    gs = mk.sspmm_backward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda), T(ci, cuda),
                           row_div=T(div, cuda), mode=mode)
    go = O.sspmm_bwd(row_ptr, col, val, g, ci, row_div=div)
    close(gs, go)
    if mode == "pull":  # other slicings of the same graph: 1, 7 and 100 row slices
        tc, vc = T(col, cuda), T(val, cuda)
        for S in (1, 7, 100):
            plan = mk.pull_plan(T(row_ptr, cuda), tc, vc, V, k, D, slices=S, cache=False)
            assert plan[3] == S
            gs = mk.sspmm_backward(T(row_ptr, cuda), tc, vc, T(g, cuda), T(ci, cuda),
                                   row_div=T(div, cuda), mode="pull", plan=plan)
            close(gs, go)


@pytest.mark.filterwarnings("ignore:backward mode 'bsort'")
def test_bucket_backward_repeats(mk, cuda):
    """fp64 bucket accumulation (bsort's phase 2): two runs agree to fp32 rounding (bitwise in
    practice)."""
    z = load_golden(CASES[2])
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val", "g", "topk_idx")]
    a = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), mode="bsort")
    b = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), mode="bsort")
    assert torch.allclose(a, b, rtol=1e-6, atol=0)


def test_csc_backward_is_deterministic(mk, cuda):
    z = load_golden(CASES[2])
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val", "g", "topk_idx")]
    a = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), chunk=11, mode="csc")
    b = mk.sspmm_backward(*args, row_div=T(z["deg"], cuda), chunk=11, mode="csc")
    assert torch.equal(a, b)


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_warp4_build_and_inverse(mk, cuda, path):
    z = load_golden(path)
    ip = T(z["row_ptr"], cuda)
    w4 = mk.build_warp4_metadata(ip, 64)
    assert np.array_equal(w4.cpu().numpy(), z["warp4_ref"])
    back = mk.warp4_to_indptr(w4, z["row_ptr"].size - 1)
    assert np.array_equal(back.cpu().numpy(), z["row_ptr"])


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_reference_binding_signatures(mk, cuda, path):
    """spmm_maxk_forward/backward(warp4, ...) exactly as the reference callers use them."""
    z = load_golden(path)
    V, k, D = z["row_ptr"].size - 1, int(z["k"]), int(z["D"])
    w4 = T(z["warp4_ref"], cuda)
    idx, val = T(z["col_idx"], cuda), T(z["val"], cuda)
    sel = T(z["topk_idx"], cuda)
    raw = mk.spmm_maxk_forward(w4, idx, val, T(z["topk_val"], cuda), sel, w4.numel() // 4, k,
                               dim_origin=D)
    deg = T(z["deg"], cuda)
    close(raw / deg.unsqueeze(-1), z["y_ref"])
    g = T(z["g"], cuda)
    gs = mk.spmm_maxk_backward(w4, idx, val, g / deg.unsqueeze(-1), sel, w4.numel() // 4, k)
    close(gs, z["grad_cbsr_ref"])
    if D == 256:  # the reference binding's default output width
        assert mk.spmm_maxk_forward(w4, idx, val, T(z["topk_val"], cuda), sel, w4.numel() // 4,
                                    k).shape == (V, 256)


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_autograd_v1_golden(F, cuda, path):
    z = load_golden(path)
    x = T(z["x"], cuda).requires_grad_(True)
    y = F.maxk_spgemm(T(z["col_idx"], cuda), T(z["val"], cuda), x, int(z["k"]),
                      graph_indptr=T(z["row_ptr"], cuda), in_degrees=T(z["deg"], cuda),
                      out_degrees=T(z["deg"], cuda))
    close(y, z["y_ref"])
    y.backward(T(z["g"], cuda))
    ref = O.scatter_dense(z["grad_cbsr_ref"], z["topk_idx"], int(z["D"]))
    close(x.grad, ref)


@pytest.mark.parametrize("via", ["function", "wrapper"])
def test_autograd_v1_out_degrees(F, cuda, via):
    """a graph whose in- and out-degrees differ.  By default the v1
    backward is the exact adjoint of the normalised forward (G / in_degrees); with
    backward_divisor="reference" it follows the reference's rule, G / out_degrees
    (maxk_spgemm_function.py:154-159), both against fixtures made by the reference's code."""
    from conftest import GOLDEN
    z = load_golden(f"{GOLDEN}/asym_outdeg_d256_k16.npz")
    D = int(z["D"])
    ip, col, val = T(z["row_ptr"], cuda), T(z["col_idx"], cuda), T(z["val"], cuda)
    din, dout = T(z["deg"], cuda), T(z["out_deg"], cuda)
    w = F.MaxKSpmmWrapper("outdeg")
    assert w.build_metadata(ip)
    for rule, want in ((None, "grad_cbsr_ref"), ("adjoint", "grad_cbsr_ref"),
                       ("reference", "grad_cbsr_refrule")):
        x = T(z["x"], cuda).requires_grad_(True)
        kw = {} if rule is None else {"backward_divisor": rule}
        if via == "function":
            y = F.maxk_spgemm(col, val, x, int(z["k"]), graph_indptr=ip, in_degrees=din,
                              out_degrees=dout, **kw)
        else:
            y = w.spmm(col, val, x, int(z["k"]), ip, din, dout, **kw)
        close(y, z["y_ref"])
        y.backward(T(z["g"], cuda))
        close(x.grad, O.scatter_dense(z[want], z["topk_idx"], D))
    with pytest.raises(ValueError):
        F.maxk_spgemm(col, val, T(z["x"], cuda), int(z["k"]), graph_indptr=ip,
                      backward_divisor="out")


def test_autograd_v1_inference_mode_bf16(F, cuda):
    """a bf16 (or non-contiguous) activation under torch.inference_mode() goes
    through the v1 path (its fp32 copy is made per call, never cached), and equals the fp32
    call on the same values."""
    from conftest import GOLDEN
    import maxk_spgemm_function as Fm
    z = load_golden(f"{GOLDEN}/sym_d256_k16.npz")
    ip, col, val = T(z["row_ptr"], cuda), T(z["col_idx"], cuda), T(z["val"], cuda)
    deg = T(z["deg"], cuda)
    xb = T(z["x"], cuda).to(torch.bfloat16)
    n0 = len(Fm._CONVERTED)
    with torch.inference_mode():
        y = F.maxk_spgemm(col, val, xb, int(z["k"]), graph_indptr=ip, in_degrees=deg)
        y_nc = F.maxk_spgemm(col, val, xb.float().t().contiguous().t(), int(z["k"]),
                             graph_indptr=ip.long(), in_degrees=deg.double())
    assert len(Fm._CONVERTED) == n0  # nothing cached: inference tensors, activations
    y32 = F.maxk_spgemm(col, val, xb.float(), int(z["k"]), graph_indptr=ip, in_degrees=deg)
    assert torch.equal(y, y32.detach()) and torch.equal(y_nc, y32.detach())
    # an int64 graph loaded outside inference mode and evaluated inside it is
    # converted once (a normal, versioned int32 copy), so every later call hits the caches
    ip64 = ip.long()
    with torch.inference_mode():
        ys = [F.maxk_spgemm(col, val, xb, int(z["k"]), graph_indptr=ip64, in_degrees=deg)
              for _ in range(2)]
    hit = Fm._CONVERTED[(id(ip64), "i32")]
    assert len(Fm._CONVERTED) == n0 + 1 and not hit[2].is_inference()
    assert torch.equal(ys[0], y32.detach()) and torch.equal(ys[1], y32.detach())


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_autograd_v4_wrapper_golden(F, cuda, path):
    z = load_golden(path)
    ip = T(z["row_ptr"], cuda)
    w = F.MaxKSpmmWrapper("golden")
    assert w.build_metadata(ip)
    tv = T(z["topk_val"], cuda).requires_grad_(True)
    ti = T(z["topk_idx"], cuda, torch.int64)
    y = w.spmm(T(z["col_idx"], cuda), T(z["val"], cuda), tv, ti, ip, T(z["deg"], cuda),
               dim_origin=int(z["D"]))
    close(y, z["y_ref"])
    y.backward(T(z["g"], cuda))
    close(tv.grad, z["grad_cbsr_ref"])


@pytest.mark.parametrize("k", [8, 16])
def test_autograd_sparse_graph_stream(F, mk, cuda, monkeypatch, k):
    """A sparse graph whose G is too large for the pull (70k rows, average degree 6): the
    autograd forward writes the edge-selector stream and its backward reads it in the mode
    "auto" resolves to -- window-sorted ("bsort") at k = 8, csc at k = 16 -- and the input
    gradient equals the one through the bitwise csc form without the stream."""
    torch.manual_seed(k)
    V, D, E = 70_000, 256, 420_000
    key = torch.unique(torch.randint(0, V, (E,), device=cuda).long() * V
                       + torch.randint(0, V, (E,), device=cuda).long())
    src, dst = (key // V).int(), (key % V).int()
    ip = torch.zeros(V + 1, dtype=torch.int32, device=cuda)
    ip[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0).int()
    val = torch.rand(dst.numel(), device=cuda)
    deg = torch.bincount(src, minlength=V).clamp(min=1).float()
    assert mk.edge_selector_mode(ip, dst, k, V, D) == ("bsort" if k == 8 else "csc")
    g = torch.randn(V, D, device=cuda)
    grads = []
    for env in ("auto", "csc"):
        monkeypatch.setenv("MAXK_BWD_MODE", env)
        monkeypatch.setenv("MAXK_EDGE_SEL", "1" if env == "auto" else "0")
        torch.manual_seed(0)
        x = torch.randn(V, D, device=cuda).requires_grad_(True)
        y = F.maxk_spgemm(dst, val, x, k, graph_indptr=ip, in_degrees=deg, out_degrees=deg)
        y.backward(g)
        grads.append(x.grad)
    close(grads[0], grads[1].cpu().numpy(), tol=1e-5)


def test_autograd_plans_built_once(F, mk, cuda, monkeypatch):
    """Steps through the warp4 call shape with int64 indices and float64 weights (each call's
    int32 / fp32 conversions are cached per source tensor): on a sparse graph where
    "auto" picks the window-sorted backward at k = 8, the bsort plan and the locality pass are
    built on the first step only, and every step's gradient is the same."""
    monkeypatch.delenv("MAXK_BWD_MODE", raising=False)
    monkeypatch.delenv("MAXK_EDGE_SEL", raising=False)
    torch.manual_seed(3)
    V, D, E, k = 70_000, 256, 420_000, 8
    key = torch.unique(torch.randint(0, V, (E,), device=cuda).long() * V
                       + torch.randint(0, V, (E,), device=cuda).long())
    src, dst = key // V, key % V  # int64
    ip = torch.zeros(V + 1, dtype=torch.int64, device=cuda)
    ip[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0)
    val = torch.rand(dst.numel(), device=cuda, dtype=torch.float64)
    deg = torch.bincount(src, minlength=V).clamp(min=1).double()
    w = F.MaxKSpmmWrapper("plans")
    assert w.build_metadata(ip)
    w._indptr_cache = None  # force the warp4 -> indptr route on every call
    built = []
    real = mk.bsort_plan

    def spy(indptr, indices, num_cols, kk, cache=True):
        n = len(mk._BSORT_CACHE)
        plan = real(indptr, indices, num_cols, kk, cache)
        built.append(len(mk._BSORT_CACHE) > n)
        return plan
    monkeypatch.setattr(mk, "bsort_plan", spy)
    tv = torch.rand(V, k, device=cuda)
    ti = torch.stack([torch.randperm(D, device=cuda)[:k] for _ in range(4)]).repeat(V // 4, 1)
    g = torch.randn(V, D, device=cuda)
    loc0 = len(mk._LOCALITY)
    grads = []
    for _ in range(3):
        x = tv.clone().requires_grad_(True)
        y = F.maxk_spgemm(dst, val, x, ti, w.warp4_metadata, w.num_warps, None, deg,
                          dim_origin=D)
        y.backward(g)
        grads.append(x.grad)
    assert built == [True, False, False], built
    assert len(mk._LOCALITY) == loc0 + 1
    assert torch.equal(grads[0], grads[1]) or close(grads[1], grads[0].cpu().numpy(), 1e-6)
    close(grads[2], grads[0].cpu().numpy(), 1e-6)


# --------------------------------------------------------------------------- oracle, edge cases
def rand_graph(rng, V, avg, hubs=(), empty=0, cols=None):
    cols = V if cols is None else cols
    deg = rng.poisson(avg, V).astype(np.int64)
    for r, d in hubs:
        deg[r] = d
    if empty:
        deg[rng.choice(V, empty, replace=False)] = 0
    rows = []
    for r in range(V):
        d = min(int(deg[r]), cols)
        rows.append(np.sort(rng.choice(cols, d, replace=False)) if d else np.zeros(0, np.int64))
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum([len(x) for x in rows], out=row_ptr[1:])
    col = np.concatenate(rows) if row_ptr[-1] else np.zeros(0, np.int64)
    return row_ptr.astype(np.int32), col.astype(np.int32)


def run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, div=None, chunk=0, mode=None):
    y = mk.spgemm_forward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda), T(ci, cuda),
                          D, row_div=None if div is None else T(div, cuda), chunk=chunk)
    gs = mk.sspmm_backward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda), T(ci, cuda),
                           row_div=None if div is None else T(div, cuda), chunk=chunk, mode=mode)
    yo = O.spgemm_fwd(row_ptr, col, val, cv, ci, D, row_div=div)
    go = O.sspmm_bwd(row_ptr, col, val, g, ci, row_div=div)
    return y, yo, gs, go


@pytest.mark.parametrize("k,D", [(1, 64), (2, 64), (3, 64), (8, 256), (16, 256), (24, 256),
                                 (32, 256), (48, 256), (64, 256), (96, 256), (128, 256),
                                 (255, 256), (256, 256), (16, 100), (7, 9), (32, 64),
                                 (64, 64), (52, 100), (64, 128), (128, 128)])
def test_all_k_against_oracle(mk, cuda, k, D):
    rng = np.random.default_rng(k * 1000 + D)
    V = 600
    row_ptr, col = rand_graph(rng, V, 12, hubs=((3, 590), (100, 200)), empty=20)
    val = rng.random(col.size, dtype=np.float32)
    x = rng.standard_normal((V, D), dtype=np.float32)
    cv, ci = O.topk(x, k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    # csc: chunk 2048 is the largest item whose eid slots are staged in LDS, 4096 reads them
    # from global memory (csc_sum_kernel STAGED)
    modes = [(0, "auto"), (0, "csc"), (13, "csc"), (2048, "csc"), (4096, "csc"), (13, "atomic")]
    if k % 4 == 0:
        modes += [(0, "bsort")]
    if D % 4 == 0 and (k % 4 == 0 or k <= 64):
        modes.append((0, "pull"))
    if D % 4 == 0 and k % 4 == 0:
        modes += [(0, "dense"), (13, "dense"), (600, "dense")]
    for chunk, mode in modes:
        y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, div, chunk, mode)
        close(y, yo)
        close(gs, go)
    v, i = mk.topk_cbsr(T(x, cuda), k)
    assert np.array_equal(i.cpu().numpy(), ci) and np.array_equal(v.cpu().numpy(), cv)


@pytest.mark.parametrize("k", [16, 12, 10, 64])
def test_high_degree_against_oracle(mk, cuda, k):
    """Average degree ~500 (Reddit-like): the backward picks its deepest batches (phase 1
    U=16, phase 2 U=8); k=16/64 take the float4 phase 2, 12 the padded 4-l-per-lane phase 1,
    10 the one-l-per-lane path."""
    rng = np.random.default_rng(77 + k)
    V, D = 2000, 256
    row_ptr, col = rand_graph(rng, V, 500, hubs=((7, 1999),))
    val = rng.random(col.size, dtype=np.float32)
    x = rng.standard_normal((V, D), dtype=np.float32)
    cv, ci = O.topk(x, k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    for mode in ("csc", "bsort", "pull") if k % 4 == 0 else ("csc", "pull"):
        y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, div, 0, mode)
        close(y, yo)
        close(gs, go)


def test_empty_graph_and_empty_rows(mk, cuda):
    D, k, V = 64, 16, 50
    rng = np.random.default_rng(1)
    cv = rng.random((V, k), dtype=np.float32)
    ci = np.stack([rng.choice(D, k, replace=False) for _ in range(V)]).astype(np.uint8)
    g = rng.standard_normal((V, D), dtype=np.float32)
    row_ptr = np.zeros(V + 1, np.int32)
    col = np.zeros(0, np.int32)
    val = np.zeros(0, np.float32)
    y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D)
    assert not y.cpu().numpy().any() and not gs.cpu().numpy().any()
    # only the last row has edges; many leading empty rows share work items
    row_ptr = np.zeros(V + 1, np.int32)
    row_ptr[-1] = 3
    col = np.array([0, 5, 49], np.int32)
    val = np.array([1.0, 2.0, 3.0], np.float32)
    for chunk in (0, 1, 2, 7):
        for mode in ("pull", "bsort", "csc", "atomic", "dense"):
            y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, chunk=chunk,
                                     mode=mode)
            close(y, yo)
            close(gs, go)


def test_zero_rows(mk, cuda):
    """A shard that owns no rows (maxk_dist with more ranks than hub-balanced ranges): the
    forward returns [0, D]; the backward still returns the full [num_cols, k] gradient, all
    zero, in both modes."""
    D, k, ncols = 64, 16, 50
    rng = np.random.default_rng(3)
    cv = torch.from_numpy(rng.random((ncols, k), dtype=np.float32)).to(cuda)
    ci = torch.from_numpy(np.stack([rng.choice(D, k, replace=False) for _ in range(ncols)])
                          .astype(np.uint8)).to(cuda)
    row_ptr = torch.zeros(1, dtype=torch.int32, device=cuda)
    col = torch.zeros(0, dtype=torch.int32, device=cuda)
    val = torch.zeros(0, dtype=torch.float32, device=cuda)
    y = mk.spgemm_forward(row_ptr, col, val, cv, ci, D)
    assert y.shape == (0, D)
    g = torch.zeros(0, D, device=cuda)
    for mode in ("pull", "bsort", "csc", "atomic", "dense"):
        gs = torch.full((ncols, k), 7.0, device=cuda)
        mk.sspmm_backward(row_ptr, col, val, g, ci, out=gs, mode=mode)
        torch.cuda.synchronize()
        assert gs.shape == (ncols, k) and not gs.cpu().numpy().any(), mode


def test_output_fully_overwritten(mk, cuda):
    """No zero-init contract: pre-filled output buffers must be overwritten everywhere."""
    rng = np.random.default_rng(5)
    V, D, k = 300, 256, 16
    row_ptr, col = rand_graph(rng, V, 8, empty=30)
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    g = rng.standard_normal((V, D), dtype=np.float32)
    out = torch.full((V, D), float("nan"), device=cuda)
    y = mk.spgemm_forward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda), T(ci, cuda),
                          D, out=out, chunk=9)
    close(y, O.spgemm_fwd(row_ptr, col, val, cv, ci, D))
    for mode in ("pull", "bsort", "csc", "atomic", "dense"):
        gout = torch.full((V, k), float("nan"), device=cuda)
        gs = mk.sspmm_backward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda),
                               T(ci, cuda), out=gout, mode=mode, chunk=7)
        close(gs, O.sspmm_bwd(row_ptr, col, val, g, ci))


def test_duplicate_selectors_accumulate(mk, cuda):
    """Selectors with repeated columns (the reference's random test harness produces them):
    the kernels accumulate, like the reference's shared-memory sum."""
    rng = np.random.default_rng(9)
    V, D, k = 200, 64, 16
    row_ptr, col = rand_graph(rng, V, 20)
    val = rng.random(col.size, dtype=np.float32)
    cv = rng.random((V, k), dtype=np.float32)
    ci = rng.integers(0, 8, (V, k)).astype(np.uint8)  # heavy duplication
    g = rng.standard_normal((V, D), dtype=np.float32)
    y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, chunk=17)
    close(y, yo)
    close(gs, go)


@pytest.mark.parametrize("D,k", [(64, 16), (64, 32), (64, 64), (100, 52), (128, 32), (128, 64),
                                 (128, 8), (256, 16)])
def test_forward_small_sparse_paths(mk, cuda, D, k):
    """The small sparse graphs' forwards (r05): the streaming rows over packed records and, at
    k >= D / 2 (D <= 128), the dense route (CBSR scattered to dense rows, lane groups walking
    rows into registers) in both directions, with repeated selectors, selectors >= D, empty
    rows, hub rows split over items (chunk 40) and rows past the lane groups' limit, against
    the oracle; the full-width oracle cut back to D is the reference for selectors past D (they
    contribute nothing).  The dense backward is bitwise repeatable."""
    rng = np.random.default_rng(D * 100 + k)
    V = 3000
    row_ptr, col = rand_graph(rng, V, 9, hubs=((7, 900), (11, 70), (1500, 130)), empty=40)
    val = rng.random(col.size, dtype=np.float32)
    cv = rng.standard_normal((V, k)).astype(np.float32)
    ci = np.stack([rng.choice(D, k, replace=False) for _ in range(V)]).astype(np.uint8)
    ci[rng.choice(V, 50, replace=False), 0] = ci[rng.choice(V, 50, replace=False), 1]
    dup = rng.choice(V, 60, replace=False)
    ci[dup, -1] = ci[dup, 0]                      # repeated selectors sum
    past = rng.choice(V, 60, replace=False)
    if D < 256:
        ci[past, 1] = rng.integers(D, 256, 60).astype(np.uint8)  # contribute nothing
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    yo = O.spgemm_fwd(row_ptr, col, val, cv, ci, 256, row_div=div)[:, :D]
    for chunk in (0, 40):
        y = mk.spgemm_forward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda),
                              T(ci, cuda), D, row_div=T(div, cuda), chunk=chunk, validate=False)
        close(y, yo)
        acc = torch.ones(V, D, device=cuda)
        mk.spgemm_forward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda),
                          T(ci, cuda), D, row_div=T(div, cuda), chunk=chunk, validate=False,
                          out=acc, accumulate=True)
        close(acc, yo + 1.0)
    assert mk._lib().maxk_dense_route(D, k) == int(k % 4 == 0 and D <= 128 and 2 * k >= D)
    if k % 4 == 0 and D % 4 == 0:
        g = rng.standard_normal((V, D), dtype=np.float32)
        gpad = np.zeros((V, 256), np.float32)  # selectors >= D read 0
        gpad[:, :D] = g
        go = O.sspmm_bwd(row_ptr, col, val, gpad, ci, row_div=div)
        args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda), T(ci, cuda))
        for chunk in (0, 40):
            gs = mk.sspmm_backward(*args, row_div=T(div, cuda), chunk=chunk, mode="dense",
                                   validate=False)
            close(gs, go)
            again = mk.sspmm_backward(*args, row_div=T(div, cuda), chunk=chunk, mode="dense",
                                      validate=False)
            assert torch.equal(gs, again)


@pytest.mark.parametrize("D,k", [(256, 32), (128, 24), (100, 28), (256, 28)])
def test_forward_stream_wide_records(mk, cuda, D, k):
    """The streaming forward over records past one 128-B line (k >= 22, sparse graph), clean
    and dirty CBSR (a repeated selector, a selector >= D) against the oracle, with hub rows split
    over items (chunk 40), rows past the lane groups' limit, accumulate and 4-B (not 16-B)
    aligned values; an extra dirty vertex that no edge reads changes nothing, bitwise.  (r05
    measured reading the caller's arrays instead of records here, guarded by a device check,
    and rejected it: profiles/r05/tune/split_source/.)"""
    rng = np.random.default_rng(D * 1000 + k)
    V = 3000
    row_ptr, col = rand_graph(rng, V, 9, hubs=((7, 900), (11, 70), (1500, 130)), empty=40)
    val = rng.random(col.size, dtype=np.float32)
    cv = rng.standard_normal((V, k)).astype(np.float32)
    ci = np.stack([rng.choice(D, k, replace=False) for _ in range(V)]).astype(np.uint8)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda))

    def fwd(cvv, civ, **kw):
        return mk.spgemm_forward(*args, T(cvv, cuda) if isinstance(cvv, np.ndarray) else cvv,
                                 T(civ, cuda) if isinstance(civ, np.ndarray) else civ, D,
                                 row_div=T(div, cuda), validate=False, **kw)

    yo = O.spgemm_fwd(row_ptr, col, val, cv, ci, 256, row_div=div)[:, :D]
    for chunk in (0, 40):
        y = fwd(cv, ci, chunk=chunk)
        close(y, yo)
        # one more vertex, with a repeated selector, that no edge reads
        cvx = np.concatenate([cv, cv[:1]])
        cix = np.concatenate([ci, ci[:1]])
        cix[-1, 1] = cix[-1, 0]
        assert torch.equal(fwd(cvx, cix, chunk=chunk), y)
        acc = torch.ones(V, D, device=cuda)
        fwd(cv, ci, chunk=chunk, out=acc, accumulate=True)
        close(acc, yo + 1.0)
    fv = torch.empty(V * k + 1, device=cuda)[1:].view(V, k)  # 4-B, not 16-B aligned
    fv.copy_(T(cv, cuda))
    close(fwd(fv, ci), yo)
    # dirty inputs: repeated selectors sum, selectors >= D contribute nothing
    cid = ci.copy()
    dup = rng.choice(V, 60, replace=False)
    cid[dup, -1] = cid[dup, 0]
    if D < 256:
        cid[rng.choice(V, 60, replace=False), 1] = rng.integers(D, 256, 60).astype(np.uint8)
    yd = O.spgemm_fwd(row_ptr, col, val, cv, cid, 256, row_div=div)[:, :D]
    for chunk in (0, 40):
        close(fwd(cv, cid, chunk=chunk), yd)


@pytest.mark.parametrize("k", [8, 32])
def test_tables_past_2_24_columns(mk, cuda, k):
    """Maximum sizes of the column space: num_cols = 2^24 + 4099 source vertices, so record
    offsets no longer fit the 24-bit multiply (the forward's 64-bit-address walker, WIDE; at
    k = 32 the record table also passes 4 GiB) and phase 1 of the two-phase backward takes its
    32-bit selector multiply (kStoreX4W).  A 1,500-row graph whose edges reach every part of
    that range, including the last columns and a hub row split over items at chunk 50; the
    forward and the csc / atomic / bsort / pull backwards against the oracle over the columns
    the edges read (compacted), and every other gradient row exactly zero."""
    rng = np.random.default_rng(77 + k)
    NC = (1 << 24) + 4099
    V, D = 1500, 256
    deg = rng.integers(0, 40, V)
    deg[5] = 900
    rows = [np.sort(rng.choice(NC, int(d), replace=False)) for d in deg]
    rows[9] = np.sort(np.concatenate([rows[9], NC - 1 - np.arange(3)]))  # the table's end
    rp = np.zeros(V + 1, np.int64)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    rp = rp.astype(np.int32)
    col = np.concatenate(rows).astype(np.int32)
    assert int(col.max()) == NC - 1 and (col >= (1 << 24)).sum() > 0
    val = rng.random(col.size, dtype=np.float32)
    uc = np.unique(col)
    colc = np.searchsorted(uc, col).astype(np.int32)
    cvc = rng.standard_normal((uc.size, k)).astype(np.float32)
    cic = np.stack([rng.choice(D, k, replace=False) for _ in range(uc.size)]).astype(np.uint8)
    div = np.maximum(np.diff(rp), 1).astype(np.float32)
    G = rng.standard_normal((V, D)).astype(np.float32)
    ucg = torch.from_numpy(uc.astype(np.int64)).to(cuda)
    cv = torch.zeros(NC, k, device=cuda)
    cv[ucg] = T(cvc, cuda)
    ci = torch.arange(k, device=cuda, dtype=torch.uint8).repeat(NC, 1)
    ci[ucg] = T(cic, cuda)
    args = (T(rp, cuda), T(col, cuda), T(val, cuda))
    yo = O.spgemm_fwd(rp, colc, val, cvc, cic, D, row_div=div)
    go = O.sspmm_bwd(rp, colc, val, G, cic, row_div=div)
    for chunk in (0, 50):
        close(mk.spgemm_forward(*args, cv, ci, D, row_div=T(div, cuda), chunk=chunk), yo)
    modes = ["csc", "atomic", "pull"] + (["bsort"] if k <= 8 else [])
    for mode in modes:
        for chunk in ((0, 50) if mode != "pull" else (0,)):
            gs = mk.sspmm_backward(*args, T(G, cuda), ci, row_div=T(div, cuda), chunk=chunk,
                                   mode=mode)
            close(gs[ucg], go)
            gs[ucg] = 0.0
            assert not gs.any(), f"{mode}: rows no edge reads are not zero"
            del gs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [4, 12, 16, 32])
def test_forward_pack_aligned_and_not(mk, cuda, k):
    """The forward's record pack runs four l per thread (cbsr_pack4_kernel) on aligned CBSR
    buffers and one per thread otherwise: both against the oracle, with repeated selectors
    on some rows and selectors past D."""
    rng = np.random.default_rng(31 + k)
    V, D = 300, 100
    row_ptr, col = rand_graph(rng, V, 25)
    val = rng.random(col.size, dtype=np.float32)
    cv = rng.standard_normal((V, k)).astype(np.float32)
    ci = np.stack([rng.choice(256, k, replace=False) for _ in range(V)]).astype(np.uint8)
    ci[::5, 1] = ci[::5, 0]  # duplicates
    ci[::7, 2] = 200         # past D
    ref = O.spgemm_fwd(row_ptr, col, val, cv, ci, 256)[:, :D]  # selectors >= D drop out
    args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda))
    close(mk.spgemm_forward(*args, T(cv, cuda), T(ci, cuda), D, validate=False), ref)
    fv = torch.empty(V * k + 1, device=cuda)[1:].view(V, k)  # 4-B, not 16-B aligned
    fi = torch.empty(V * k + 1, dtype=torch.uint8, device=cuda)[1:].view(V, k)
    fv.copy_(T(cv, cuda))
    fi.copy_(T(ci, cuda))
    close(mk.spgemm_forward(*args, fv, fi, D, validate=False), ref)
    # the edge-selector stream keeps the caller's bytes (duplicates, past D) whichever pack
    # folded them, and the csc backward reading it matches the oracle (selectors >= D read 0)
    for cvv, civ in ((T(cv, cuda), T(ci, cuda)), (fv, fi)):
        es = torch.zeros(col.size, k, dtype=torch.uint8, device=cuda)
        close(mk.spgemm_forward(*args, cvv, civ, D, validate=False, edge_sel_out=es), ref)
        assert np.array_equal(es.cpu().numpy(), ci[col])
    if k % 4 == 0:
        g = rng.standard_normal((V, D), dtype=np.float32)
        g_pad = np.zeros((V, 256), np.float32)
        g_pad[:, :D] = g
        gs = mk.sspmm_backward(*args, T(g, cuda), T(ci, cuda), mode="csc", validate=False,
                               edge_sel=es)
        close(gs, O.sspmm_bwd(row_ptr, col, val, g_pad, ci))


def test_selectors_past_D_read_zero(mk, cuda):
    """A selector >= D (possible when D < 256; the reference does no bounds check,
    cuda_kernel_bindings.cpp:106-161) contributes nothing, in the forward and in every
    backward mode: D = 100 with selector 200 on the last row (whose G row ends the
    allocation) and on random other rows.  Expected: the oracle on G padded with zero
    columns to 256 (backward) and on the full-width forward cut back to D."""
    rng = np.random.default_rng(21)
    V, D, k = 300, 100, 16
    row_ptr, col = rand_graph(rng, V, 30, hubs=((V - 1, 250),))
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    ci[V - 1, 3] = 200
    bad = rng.choice(V - 1, 40, replace=False)
    ci[bad, rng.integers(0, k, 40)] = rng.integers(D, 256, 40).astype(np.uint8)
    g = rng.standard_normal((V, D), dtype=np.float32)
    g_pad = np.zeros((V, 256), np.float32)
    g_pad[:, :D] = g
    go = O.sspmm_bwd(row_ptr, col, val, g_pad, ci)
    yo = O.spgemm_fwd(row_ptr, col, val, cv, ci, 256)[:, :D]
    y = mk.spgemm_forward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda),
                          T(ci, cuda), D, validate=False)
    close(y, yo)
    for mode in ("pull", "bsort", "csc", "atomic", "dense"):
        gs = mk.sspmm_backward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda),
                               T(ci, cuda), mode=mode, validate=False)
        close(gs, go)
    with pytest.raises(RuntimeError):  # and the validating call rejects the input
        mk.sspmm_backward(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(g, cuda),
                          T(ci, cuda), validate=True)


def test_rectangular_shard(mk, cuda):
    """num_rows != num_cols: a vertex-range shard's rows against the full CBSR."""
    rng = np.random.default_rng(11)
    R, C, D, k = 150, 700, 256, 32
    row_ptr, col = rand_graph(rng, R, 40, cols=C)
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((C, D), dtype=np.float32), k)
    g = rng.standard_normal((R, D), dtype=np.float32)
    for mode in ("pull", "bsort", "csc", "atomic", "dense"):
        y, yo, gs, go = run_both(mk, cuda, row_ptr, col, val, cv, ci, g, D, chunk=64, mode=mode)
        assert y.shape == (R, D) and gs.shape == (C, k)
        close(y, yo)
        close(gs, go)


def test_topk_ties_nan_and_uint8(mk, cuda):
    x = torch.tensor([[1.0, 3.0, 3.0, 2.0, float("nan"), 3.0, -1.0, 0.0]], device=cuda)
    v, i = mk.topk_cbsr(x, 4)
    assert i.cpu().tolist() == [[4, 1, 2, 5]]  # NaN largest; ties by ascending column
    assert torch.isnan(v[0, 0]) and v[0, 1:].cpu().tolist() == [3.0, 3.0, 3.0]
    rng = np.random.default_rng(2)
    xu = rng.integers(0, 256, (300, 256)).astype(np.uint8)
    vu, iu = mk.cuda_topk_maxk(T(xu, cuda), 32)
    order = np.lexsort((np.tile(np.arange(256), (300, 1)), -xu.astype(np.int32)), axis=1)[:, :32]
    assert np.array_equal(iu.cpu().numpy(), order.astype(np.uint8))
    assert np.array_equal(vu.cpu().numpy(), np.take_along_axis(xu, order, 1))


@pytest.mark.parametrize("D", [256, 100, 64, 7])
def test_topk_threshold_search_edges(mk, cuda, D):
    """The threshold search of the top-k kernels (bisection from a lower bound of the k-th
    key) on rows built to stress it, bit-exact against the oracle for every k up to 32 and a
    few above: all-equal rows, few distinct values (many ties at the threshold), neighbouring
    fp32 values (ulp steps), +-inf, -0.0 beside 0.0, NaN, mixed signs, one huge value."""
    rng = np.random.default_rng(D)
    rows = [np.full(D, 1.5), np.full(D, -2.0), rng.integers(0, 3, D).astype(np.float64),
            rng.integers(-2, 2, D) * 0.5,
            np.nextafter(np.float32(1.0), np.float32(2.0)) + np.arange(D) * 0.0,
            rng.standard_normal(D), rng.random(D), -rng.random(D)]
    u = np.float32(1.0)
    steps = np.array([u] * D, np.float32)
    for j in range(1, D):  # consecutive floats: keys one apart
        steps[j] = np.nextafter(steps[j - 1], np.float32(2.0))
    rows.append(rng.permutation(steps))
    special = rng.standard_normal(D)
    special[rng.choice(D, min(D, 6), replace=False)] = [np.inf, -np.inf, np.nan, -0.0, 0.0,
                                                         3e38][:min(D, 6)]
    rows.append(special)
    big = rng.random(D)
    big[0] = 1e30
    rows.append(big)
    x = np.stack(rows).astype(np.float32)
    x = np.concatenate([x, rng.permutation(x, axis=1)])
    for k in sorted({1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 32, min(D, 33), min(D, 64), D}):
        if k > D:
            continue
        v, i = mk.topk_cbsr(T(x, cuda), k)
        cv, ci = O.topk(x, k)
        assert np.array_equal(i.cpu().numpy(), ci), (D, k)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), cv.view(np.uint32)), (D, k)


@pytest.mark.parametrize("D", [7, 64, 100])
@pytest.mark.parametrize("tail", [1, 2, 3])
def test_topk_grid_stride_tails(mk, cuda, D, tail):
    """The top-k winner compaction over several grid-stride rounds with a last row group of
    1-3 live rows (V % 4 = tail) and three (or one, two) dead sub-rows: r02's fault was such a
    group's dead rows compacting past their LDS region into the next wave's winners while it was
    still ranking.  Rows of all-equal keys, +-0, NaN runs, +-inf, few distinct
    values and random rows, each row's columns shuffled; every row bit-exact against the oracle
    for k up to D, through both kernels (four rows per wave up to k = 48, one above), the fused
    dense form too, and the kernels' own count of rows with other than k winners stays 0
    (maxk_topk_error_rows; MAXK_VALIDATE=1 also checks it after every call)."""
    rng = np.random.default_rng(100 * D + tail)
    V = 2 * 262144 + 4 * 1000 + tail  # > 2 rounds of the four-row grid (16384 x 16 rows)
    base = [np.full(D, 1.5), np.zeros(D), np.where(rng.random(D) < .5, 0.0, -0.0),
            np.full(D, np.nan), np.where(rng.random(D) < .3, np.nan, 1.0),
            np.where(rng.random(D) < .5, np.inf, -np.inf), rng.integers(0, 3, D) * 1.0,
            rng.standard_normal(D)]
    kinds = rng.integers(0, len(base) + 2, V)  # two kinds of fresh random rows as well
    x = np.empty((V, D), np.float32)
    for j, row in enumerate(base):
        x[kinds == j] = row
    m = kinds == len(base)
    x[m] = rng.standard_normal((int(m.sum()), D))
    m = kinds == len(base) + 1
    x[m] = rng.integers(-1, 2, (int(m.sum()), D)) * 0.0  # +-0 and 0 only
    x = rng.permuted(x, axis=1)
    xt = T(x, cuda)
    mk.topk_error_rows(cuda)  # start from a zero count
    for k in sorted({1, 3, D, min(D, 8), min(D, 16), min(D, 32), min(D, 33), min(D, 48),
                     min(D, 64)}):
        v, i = mk.topk_cbsr(xt, k)
        cv, ci = O.topk(x, k)
        bad = np.nonzero((i.cpu().numpy() != ci).any(1) |
                         (v.cpu().numpy().view(np.uint32) != cv.view(np.uint32)).any(1))[0]
        assert bad.size == 0, (D, tail, k, bad[:10])
        dense, v2, i2 = mk.topk_cbsr_dense(xt, k)
        assert torch.equal(i2, i) and torch.equal(v2.view(torch.int32), v.view(torch.int32))
        assert mk.topk_error_rows(cuda) == 0, (D, tail, k)


def test_scatter_dense_and_selector_gen(mk, cuda):
    rng = np.random.default_rng(4)
    cv, ci = O.topk(rng.standard_normal((100, 256), dtype=np.float32), 16)
    d = mk.cbsr_scatter_dense(T(cv, cuda), T(ci, cuda), 256)
    assert np.array_equal(d.cpu().numpy(), O.scatter_dense(cv, ci, 256))
    sel = mk.generate_sparse_selector(1000, 256, 32)
    s = sel.cpu().numpy().astype(np.int64)
    assert s.shape == (1000, 32)
    assert all(len(set(r)) == 32 for r in s)


@pytest.mark.parametrize("D,k", [(256, 16), (256, 1), (100, 32), (7, 7)])
def test_fused_maxk_forward_backward(mk, cuda, D, k):
    """maxk_topk_cbsr_dense == (topk, scatter) and maxk_topk_backward == scatter(gv + gd[sel]),
    bit-exact (one fp32 add per output), ties (quantised values) and a NaN included."""
    rng = np.random.default_rng(D + k)
    V = 700
    x = np.round(rng.standard_normal((V, D)) * 4).astype(np.float32) / 4  # many ties
    x[3, D // 2] = np.nan
    dense, v, i = mk.topk_cbsr_dense(T(x, cuda), k)
    cv, ci = O.topk(x, k)
    assert np.array_equal(i.cpu().numpy(), ci)
    assert np.array_equal(v.cpu().numpy(), cv, equal_nan=True)
    assert np.array_equal(dense.cpu().numpy(), O.scatter_dense(cv, ci, D), equal_nan=True)
    # a strided input (ld_x > D) gives the same result
    wide = np.zeros((V, D + 5), np.float32)
    wide[:, :D] = x
    d2, v2, i2 = mk.topk_cbsr_dense(T(wide, cuda)[:, :D], k)
    assert torch.equal(i2, i) and torch.equal(d2.nan_to_num(), dense.nan_to_num())

    gv = rng.standard_normal((V, k)).astype(np.float32)
    gd = rng.standard_normal((V, D)).astype(np.float32)
    picked = np.take_along_axis(gd, ci.astype(np.int64), 1)
    for a, b, want in ((gv, None, gv), (None, gd, picked), (gv, gd, gv + picked)):
        got = mk.topk_backward(None if a is None else T(a, cuda),
                               None if b is None else T(b, cuda), i, D)
        assert np.array_equal(got.cpu().numpy(), O.scatter_dense(want, ci, D))
    gd_t = T(gd, cuda)  # in place: grad_x aliases grad_dense
    mk.topk_backward(T(gv, cuda), gd_t, i, D, out=gd_t)
    assert np.array_equal(gd_t.cpu().numpy(), O.scatter_dense(gv + picked, ci, D))
    with pytest.raises(RuntimeError):
        mk.topk_backward(T(gv, cuda), None, i, D + 1, out=torch.empty(V, D, device=cuda))


def test_rocsparse_baseline_matches_oracle(mk, cuda):
    rng = np.random.default_rng(6)
    V, D, k = 500, 256, 16
    row_ptr, col = rand_graph(rng, V, 30)
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((V, D), dtype=np.float32), k)
    dense = O.scatter_dense(cv, ci, D)
    y = mk.cusparse_spmm(T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(dense, cuda))
    close(y, O.spgemm_fwd(row_ptr, col, val, cv, ci, D))


def test_runs_on_current_stream(mk, cuda):
    rng = np.random.default_rng(8)
    z = load_golden(CASES[0])
    s = torch.cuda.Stream()
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val", "topk_val", "topk_idx")]
    with torch.cuda.stream(s):
        y = mk.spgemm_forward(*args, int(z["D"]), row_div=T(z["deg"], cuda))
    s.synchronize()
    close(y, z["y_ref"])


def test_hipgraph_capture(mk, cuda):
    """The launch path allocates/synchronises nothing: it can be captured and replayed."""
    z = load_golden(CASES[2])
    args = [T(z[n], cuda) for n in ("row_ptr", "col_idx", "val", "topk_val", "topk_idx")]
    deg = T(z["deg"], cuda)
    out = torch.empty(z["row_ptr"].size - 1, int(z["D"]), device=cuda)
    mk.spgemm_forward(*args, int(z["D"]), row_div=deg, out=out)  # warm up allocator
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mk.spgemm_forward(*args, int(z["D"]), row_div=deg, out=out, validate=False)
    out.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    close(out, z["y_ref"])


@pytest.mark.parametrize("mode", ["pull", "bsort", "csc", "hybrid", "atomic", "dense"])
def test_hipgraph_capture_default_validation(mk, cuda, monkeypatch, mode):
    """Default (validate-once) mode: the first call may be inside a capture; forward and the
    two-phase backward (with its plan built beforehand) both replay correctly."""
    monkeypatch.setenv("MAXK_VALIDATE", "")
    z = load_golden(CASES[2])
    rp, ci, va, cv, cs = [T(z[n], cuda).clone() for n in ("row_ptr", "col_idx", "val", "topk_val",
                                                         "topk_idx")]
    deg, g_in = T(z["deg"], cuda), T(z["g"], cuda)
    D = int(z["D"])
    V = rp.numel() - 1
    out = torch.empty(V, D, device=cuda)
    gs = torch.empty(cs.shape, device=cuda)
    plan = mk.backward_plan(ci, cs.shape[0], cs.shape[1], mode, indptr=rp, values=va, dim=D)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mk.spgemm_forward(rp, ci, va, cv, cs, D, row_div=deg, out=out)
        mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, out=gs, plan=plan, mode=mode)
    out.fill_(float("nan"))
    gs.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    close(out, z["y_ref"])
    close(gs, z["grad_cbsr_ref"])
    # eager after the capture: the pull's pre-divided entries are built now, not in the graph
    gs2 = mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, plan=plan, mode=mode)
    close(gs2, z["grad_cbsr_ref"])
    g.replay()
    torch.cuda.synchronize()
    close(gs, z["grad_cbsr_ref"])


# --------------------------------------------------------------------------- size-independent
def test_adjoint_identity_large(mk, cuda):
    """<fwd(v), G> == <v, bwd(G)> on a 2M-edge power-law graph (no oracle needed)."""
    torch.manual_seed(0)
    V, E, D, k = 60000, 2_000_000, 256, 16
    w = torch.arange(1, V + 1, device=cuda, dtype=torch.float32).pow(-0.6)
    src = torch.multinomial(w, E, replacement=True)
    dst = torch.randint(0, V, (E,), device=cuda)
    key = torch.unique(src.long() * V + dst.long())
    src, dst = (key // V).int(), (key % V).int()
    row_ptr = torch.zeros(V + 1, dtype=torch.int32, device=cuda)
    row_ptr[1:] = torch.cumsum(torch.bincount(src, minlength=V), 0).int()
    val = torch.rand(dst.numel(), device=cuda)
    v = torch.randn(V, k, device=cuda)
    sel = mk.generate_sparse_selector(V, D, k)
    G = torch.randn(V, D, device=cuda)
    y = mk.spgemm_forward(row_ptr, dst, val, v, sel, D)
    gs = mk.sspmm_backward(row_ptr, dst, val, G, sel)
    a = (y.double() * G.double()).sum().item()
    b = (v.double() * gs.double()).sum().item()
    assert abs(a - b) <= 1e-4 * max(1.0, abs(a))
    gs_atomic = mk.sspmm_backward(row_ptr, dst, val, G, sel, mode="atomic")
    assert torch.allclose(gs, gs_atomic, rtol=1e-4, atol=1e-4)
    # row sums: sum_j Y[r, j] == A . (sum_l v[c, l])
    rs = torch.sparse_csr_tensor(row_ptr.long(), dst.long(), val, (V, V)) @ v.sum(1, keepdim=True)
    assert torch.allclose(y.sum(1), rs[:, 0], rtol=1e-4, atol=1e-3)


def test_graph_checked_once_by_default(mk, cuda, monkeypatch):
    """MAXK_VALIDATE unset: a bad graph is refused on first use (no out-of-bounds launch); a
    checked graph is not re-checked until one of its tensors is modified in place."""
    monkeypatch.setenv("MAXK_VALIDATE", "")
    rng = np.random.default_rng(5)
    row_ptr, col = rand_graph(rng, 300, 8)
    val = rng.random(col.size, dtype=np.float32)
    cv, ci = O.topk(rng.standard_normal((300, 64), dtype=np.float32), 8)
    rp, cl, vl, cvt, cit = (T(row_ptr, cuda), T(col, cuda), T(val, cuda), T(cv, cuda),
                            T(ci, cuda))
    y = mk.spgemm_forward(rp, cl, vl, cvt, cit, 64)
    close(y, O.spgemm_fwd(row_ptr, col, val, cv, ci, 64))
    cl[5] = 300  # out of range, in place: the version bump forces a new check
    with pytest.raises(RuntimeError, match="col_idx out of range"):
        mk.spgemm_forward(rp, cl, vl, cvt, cit, 64)
    with pytest.raises(RuntimeError, match="col_idx out of range"):
        mk.sspmm_backward(rp, cl, vl, T(rng.standard_normal((300, 64), dtype=np.float32), cuda),
                          cit)
    bad_rp = rp.clone()
    bad_rp[-1] += 1
    with pytest.raises(RuntimeError, match="row_ptr"):
        mk.spgemm_forward(bad_rp, T(col, cuda), vl, cvt, cit, 64)


@pytest.mark.parametrize("D,k", [(256, 32), (256, 24), (100, 28), (128, 32)])
def test_forward_transport_records(mk, cuda, D, k):
    """The sharded forward's transport records (maxk_cbsr_records, [k f32 | k u8] at 5k bytes)
    walked by maxk_spgemm_forward_records: bitwise equal to maxk_spgemm_forward on the same CBSR
    (which packs the same records itself for these shapes; before it did, the packed 256-B
    records' walk was bitwise equal too, profiles/r05/tune/transport_records/) and against the
    oracle, with repeated selectors and selectors >= D among clean rows, hub rows split over
    items (chunk 40), accumulate, and zero edges; the records keep the caller's selector bytes."""
    rng = np.random.default_rng(D * 7 + k)
    V = 3000
    row_ptr, col = rand_graph(rng, V, 9, hubs=((7, 900), (11, 70), (1500, 130)), empty=40)
    val = rng.random(col.size, dtype=np.float32)
    cv = rng.standard_normal((V, k)).astype(np.float32)
    ci = np.stack([rng.choice(D, k, replace=False) for _ in range(V)]).astype(np.uint8)
    dup = rng.choice(V, 60, replace=False)
    ci[dup, -1] = ci[dup, 0]
    if D < 256:
        ci[rng.choice(V, 60, replace=False), 1] = rng.integers(D, 256, 60).astype(np.uint8)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32)
    args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda))
    assert mk.records_ok(V, V, col.size, D, k)
    assert not mk.records_ok(V, V, col.size, D, 16)  # one-line records: the packed form
    rec = mk.cbsr_records(T(cv, cuda), T(ci, cuda), D)
    assert np.array_equal(rec.cpu().numpy()[:, 4 * k:], ci)
    for chunk in (0, 40):
        y = mk.spgemm_forward(*args, T(cv, cuda), T(ci, cuda), D, row_div=T(div, cuda),
                              chunk=chunk, validate=False)
        yr = mk.spgemm_forward_records(*args, rec, k, D, row_div=T(div, cuda), chunk=chunk,
                                       validate=False)
        assert torch.equal(y, yr)
        acc = torch.ones(V, D, device=cuda)
        mk.spgemm_forward_records(*args, rec, k, D, row_div=T(div, cuda), chunk=chunk, out=acc,
                                  accumulate=True, validate=False)
        ref = torch.ones(V, D, device=cuda)
        mk.spgemm_forward(*args, T(cv, cuda), T(ci, cuda), D, row_div=T(div, cuda), chunk=chunk,
                          out=ref, accumulate=True, validate=False)
        assert torch.equal(acc, ref)
    yo = O.spgemm_fwd(row_ptr, col, val, cv, ci, 256, row_div=div)[:, :D]
    close(yr, yo)
    empty = (T(np.zeros(V + 1, np.int32), cuda), T(np.zeros(0, np.int32), cuda),
             T(np.zeros(0, np.float32), cuda))
    # the input checks spgemm_forward makes: graph ranges, out / row_div shapes
    if D < 256:
        with pytest.raises(RuntimeError, match="sparse_selector"):
            mk.spgemm_forward_records(*args, rec, k, D, validate=True)
    bad = args[1].clone()
    bad[5] = V
    with pytest.raises(RuntimeError, match="col_idx out of range"):
        mk.spgemm_forward_records(args[0], bad, args[2], rec, k, D, validate=True)
    with pytest.raises(RuntimeError, match="out must be"):
        mk.spgemm_forward_records(*args, rec, k, D, out=torch.empty(V, D + 1, device=cuda),
                                  validate=False)
    with pytest.raises(RuntimeError, match="row_div"):
        mk.spgemm_forward_records(*args, rec, k, D, row_div=T(div[:-1], cuda), validate=False)
    with pytest.raises(RuntimeError, match="same length"):
        mk.spgemm_forward_records(args[0], args[1], args[2][:-1], rec, k, D, validate=False)
    z = torch.full((V, D), 7.0, device=cuda)
    mk.spgemm_forward_records(*empty, rec, k, D, out=z, validate=False)
    assert not z.any()
