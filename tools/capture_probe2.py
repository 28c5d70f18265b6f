"""Probe: which part of the hybrid backward breaks a second hipGraph replay -- all tiles
pulled (no csc edges), none (csc only), a mix; the C call in line (MAXK_HYBRID_STREAMS=0)."""
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
os.environ["MAXK_HYBRID_STREAMS"] = os.environ.get("STREAMS", "0")
os.environ["MAXK_PULL_PRESCALE"] = "0"


def err(a):
    a = a.cpu().numpy()
    return float(np.nanmax(np.abs(a - ref) / np.maximum(1, np.abs(ref)))), int(np.isnan(a).sum())


rp, ci, va, cs = [T(z[n]).clone() for n in ("row_ptr", "col_idx", "val", "topk_idx")]
deg, g_in = T(z["deg"]), T(z["g"])
D = int(z["D"])
V = rp.numel() - 1
for density in (0.0, 1e9, 0.5, 2.0, 5.0):
    for div in (True, False):
        plan = mk.hybrid_plan(rp, ci, va, cs.shape[0], cs.shape[1], D, density=density, cache=False)
        rd = deg if div else None
        want = ref if div else None
        gs = torch.empty(cs.shape, device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=rd, out=gs, plan=plan, mode="hybrid")
        res = []
        eager = mk.sspmm_backward(rp, ci, va, g_in, cs, row_div=rd, plan=plan, mode="hybrid")
        for _ in range(3):
            gs.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize()
            a = gs.cpu().numpy()
            res.append((float(np.nanmax(np.abs(a - eager.cpu().numpy()))), int(np.isnan(a).sum())))
        print(f"density {density} div {div}: tiles {plan[0].numel()} off edges {plan[7][1].numel()}"
              f" replays vs eager {res}", flush=True)
        del g
