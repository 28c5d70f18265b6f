"""Probe: the hybrid backward captured in a hipGraph, replayed, then something eager, then
replayed again: which eager step breaks the second replay."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("spgemm-prunning_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import maxk_cuda_kernels as mk  # noqa: E402
from conftest import golden_cases, load_golden  # noqa: E402

z = load_golden(golden_cases()[2])
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
ref = z["grad_cbsr_ref"].astype(np.float64)
os.environ["MAXK_HYBRID_STREAMS"] = "0"
os.environ["MAXK_PULL_PRESCALE"] = "0"


def err(a):
    a = a.cpu().numpy()
    return float(np.nanmax(np.abs(a - ref) / np.maximum(1, np.abs(ref)))), int(np.isnan(a).sum())


def run(cap_mode, eager):
    rp, ci, va, cs = [T(z[n]).clone() for n in ("row_ptr", "col_idx", "val", "topk_idx")]
    deg, g_in = T(z["deg"]), T(z["g"])
    D = int(z["D"])
    gs = torch.empty(cs.shape, device=dev)
    plan = mk.backward_plan(ci, cs.shape[0], cs.shape[1], cap_mode, indptr=rp, values=va, dim=D)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, out=gs, plan=plan, mode=cap_mode)
    gs.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    e1 = err(gs)
    if eager == "same":
        mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, plan=plan, mode=cap_mode)
    elif eager == "garbage":
        x = torch.empty(64 << 20, device=dev).fill_(float("nan"))
        del x
    elif eager == "csc":
        mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, mode="csc")
    elif eager == "pull":
        mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=deg, mode="pull")
    torch.cuda.synchronize()
    gs.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    e3 = err(gs)
    print(f"capture {cap_mode}, eager {eager}: replay1 {e1} replay2 {e3}", flush=True)


for cap_mode in ("hybrid", "csc", "pull"):
    for eager in ("none", "garbage", "same", "csc", "pull"):
        run(cap_mode, eager)
