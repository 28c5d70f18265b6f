"""Probe: maxk_sspmm_backward_pull_tiles alone inside a hipGraph, replayed three times, in
variants (out zeroed by torch or by the C hybrid call's memset; the tile kernels and the
reduce in one call or two)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("spgemm-prunning_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import maxk_cuda_kernels as mk  # noqa: E402
from maxk_cuda_kernels import _capi  # noqa: E402
from conftest import golden_cases, load_golden  # noqa: E402

L = _capi.load()
z = load_golden(golden_cases()[2])
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
rp, ci, va, cs = [T(z[n]).clone() for n in ("row_ptr", "col_idx", "val", "topk_idx")]
g_in = T(z["g"])
D = int(z["D"])
V = rp.numel() - 1
k = cs.shape[1]
tl, te, bp, bt, ent, shift, S, off = mk.hybrid_plan(rp, ci, va, V, k, D, density=0.0, cache=False)
p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
ws = torch.empty(L.maxk_sspmm_backward_pull_tiles_workspace_size(V, V, D, k, tl.numel()),
                 dtype=torch.uint8, device=dev)


def tiles(out, flags):
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _capi.check(L.maxk_sspmm_backward_pull_tiles(
        p(g_in), None, p(cs), p(tl), p(te), tl.numel(), p(bp), p(bt), p(ent), shift, S, flags,
        p(out), V, V, ent.shape[0], D, k, p(ws), ws.numel(), st), "pull_tiles")


variants = {
    "zero_ + tiles(acc)": lambda o: (o.zero_(), tiles(o, 1)),
    "tiles(store)": lambda o: tiles(o, 0),
    "zero_ + noreduce + reduceonly": lambda o: (o.zero_(), tiles(o, 2), tiles(o, 4 | 1)),
}
eager = torch.zeros(V, k, device=dev)
tiles(eager, 1)
torch.cuda.synchronize()
for name, fn in variants.items():
    out = torch.empty(V, k, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn(out)
    res = []
    for _ in range(3):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        a = out.cpu().numpy()
        res.append((float(np.nanmax(np.abs(a - eager.cpu().numpy()))), int(np.isnan(a).sum())))
    print(f"{name}: {res}", flush=True)
    del g
