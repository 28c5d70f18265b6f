"""Property-based GPU parity (hypothesis, derandomized so every run draws the same cases): the
HIP forward, every backward mode (hybrid included) and the top-k against the pinned oracle on random graphs
the hand-written cases do not reach -- rectangular (num_cols != num_rows), duplicate edges,
empty rows, hub rows up to every column, D not a multiple of 4, k from 1 to D, work items
from 1 token up.  Tolerance as in test_parity_gpu: |hip - oracle| <= 1e-4 * max(1, |oracle|);
selectors bit-exact."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle as O
from test_parity_gpu import T, close

pytestmark = pytest.mark.gpu


@st.composite
def cases(draw):
    V = draw(st.integers(1, 300))
    C = draw(st.integers(1, 300))
    D = draw(st.sampled_from([1, 3, 4, 8, 9, 16, 33, 64, 100, 128, 252, 256]))
    k = draw(st.integers(1, D))
    avg = draw(st.floats(0.0, 30.0))
    hub = draw(st.booleans())
    dup = draw(st.booleans())
    chunk = draw(st.sampled_from([0, 1, 2, 7, 64, 513]))
    use_div = draw(st.booleans())
    seed = draw(st.integers(0, 2**31 - 1))
    return V, C, D, k, avg, hub, dup, chunk, use_div, seed


def graph(rng, V, C, avg, hub, dup):
    deg = rng.poisson(avg, V).astype(np.int64)
    if hub:
        deg[rng.integers(V)] = C if not dup else 2 * C
    rows = []
    for r in range(V):
        d = int(deg[r]) if dup else min(int(deg[r]), C)
        c = rng.integers(0, C, d) if dup else rng.choice(C, d, replace=False)
        rows.append(np.sort(c).astype(np.int64))
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum([len(x) for x in rows], out=row_ptr[1:])
    col = np.concatenate(rows) if row_ptr[-1] else np.zeros(0, np.int64)
    return row_ptr.astype(np.int32), col.astype(np.int32)


@settings(max_examples=200, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(c=cases())
def test_random_graphs_every_mode(cuda, c):
    import maxk_cuda_kernels as mk
    V, C, D, k, avg, hub, dup, chunk, use_div, seed = c
    rng = np.random.default_rng(seed)
    row_ptr, col = graph(rng, V, C, avg, hub, dup)
    val = rng.random(col.size, dtype=np.float32)
    x = rng.standard_normal((C, D), dtype=np.float32)
    cv, ci = O.topk(x, k)
    v, i = mk.topk_cbsr(T(x, cuda), k)
    assert np.array_equal(i.cpu().numpy(), ci) and np.array_equal(v.cpu().numpy(), cv)
    g = rng.standard_normal((V, D), dtype=np.float32)
    div = np.maximum(np.diff(row_ptr), 1).astype(np.float32) if use_div else None
    dv = None if div is None else T(div, cuda)
    args = (T(row_ptr, cuda), T(col, cuda), T(val, cuda))
    y = mk.spgemm_forward(*args, T(cv, cuda), T(ci, cuda), D, row_div=dv, chunk=chunk)
    close(y, O.spgemm_fwd(row_ptr, col, val, cv, ci, D, row_div=div))
    go = O.sspmm_bwd(row_ptr, col, val, g, ci, row_div=div)
    modes = ["auto", "csc", "atomic"]
    if k % 4 == 0:
        modes += ["bsort"]
    if D % 4 == 0 and (k % 4 == 0 or k <= 64):
        modes.append("pull")
    if D % 4 == 0 and k % 4 == 0:
        modes.append("dense")
    # "atomic" adds in fp32 in whatever order the atomics land (not repeatable): thousands of
    # edges into one column with cancelling signs leave a rounding error relative to the sum of
    # the terms' magnitudes, not to the (small) result -- so it is bounded by that sum
    go_abs = O.sspmm_bwd(row_ptr, col, np.abs(val), np.abs(g), ci, row_div=div)
    for mode in modes:
        gs = mk.sspmm_backward(*args, T(g, cuda), T(ci, cuda), row_div=dv, chunk=chunk,
                               mode=mode)
        if mode == "atomic":
            err = np.abs(gs.cpu().numpy().astype(np.float64) - go)
            assert (err <= 1e-5 * np.maximum(1.0, go_abs)).all(), mode
        else:
            close(gs, go)
    if D % 4 == 0 and k % 4 == 0:  # hybrid: every tile pulled, a mix, or none
        plan = mk.hybrid_plan(*args, C, k, D, density=(0.0, 0.5, 3.0)[seed % 3], cache=False)
        gs = mk.sspmm_backward(*args, T(g, cuda), T(ci, cuda), row_div=dv, chunk=chunk,
                               mode="hybrid", plan=plan)
        close(gs, go)
