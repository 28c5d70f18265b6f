"""Probe (tools build with MAXK_TOPK_DIAG=1, MAXK_TOPK_ROWS4_KMAX=64): the four-row top-k's
per-row search state (winners taken, threshold, need, tie flag, lower bound, max, equal-key
count) around the row of the seed-0 Gaussian input that differs at k=48
(tools/topk_rows_probe.py), repeated runs to see whether the same rows fail every time, and
the state of every failing row.  Usage: python tools/topk_diag_probe.py [k]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import maxk_cuda_kernels as mk  # noqa: E402
import oracle as O  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 48
g = torch.Generator(device="cuda").manual_seed(0)
V = 2_449_029
x = torch.randn(V, 256, generator=g, device="cuda")
ref_v, ref_i = torch.topk(x, k, dim=1)  # values are unique per row here; order by value
bad_sets = []
for run in range(5):
    v, i, d = mk.topk_cbsr(x, k, with_int32=True)
    bad = torch.nonzero((v != ref_v).any(1)).flatten().cpu().numpy()
    bad_sets.append(set(bad.tolist()))
    print(f"run {run}: {len(bad)} rows differ: {bad[:12].tolist()}", flush=True)
dh = d[:, :7].cpu().numpy()
tot = dh[:, 0]
print("rows whose winners taken != k:", np.nonzero(tot != k)[0][:20].tolist(),
      "count", int((tot != k).sum()))
print("rows with the tie path:", int((dh[:, 3] != 0).sum()))
allbad = sorted(set().union(*bad_sets))
for r in allbad[:6]:
    print(f"-- bad row {r} (wave rows {r - r % 4}..{r - r % 4 + 3}), neighbours:")
    for rr in range(max(0, r - 8), min(V, r + 8)):
        t, thr, need, ties, lb, mx, neq = (int(a) & 0xffffffff for a in dh[rr])
        print(f"   row {rr}: taken {t} thr {thr:08x} need {need} ties {ties} lb {lb:08x} "
              f"mx {mx:08x} neq {neq}{'  <-- differs' if rr in allbad else ''}")
np.savez(os.path.join(ROOT, "gpurun_out", f"topk_diag_k{k}.npz"), bad=np.array(allbad),
         diag=dh[max(0, (allbad or [0])[0] - 64):(allbad or [0])[0] + 64],
         x=x[max(0, (allbad or [0])[0] - 64):(allbad or [0])[0] + 64].cpu().numpy())
