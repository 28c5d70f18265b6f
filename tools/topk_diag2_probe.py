"""Probe (tools build, MAXK_TOPK_DIAG=2, MAXK_TOPK_ROWS4_KMAX=64): for the rows of the seed-0
Gaussian input that differ at k=48, the four-row kernel's LDS winner slots as the ranking
read them (column, computed rank, key low bits) against the row itself."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 48
g = torch.Generator(device="cuda").manual_seed(0)
V = 2_449_029
x = torch.randn(V, 256, generator=g, device="cuda")
ref_v = torch.topk(x, k, dim=1).values
v, i, d = mk.topk_cbsr(x, k, with_int32=True)
bad = torch.nonzero((v != ref_v).any(1)).flatten().cpu().numpy()
print("bad rows", bad.tolist())
for r in bad[:3]:
    xr = x[r].cpu().numpy()
    u = xr.view(np.uint32).astype(np.int64)
    key = np.where(u & 0x80000000, (~u) & 0xffffffff, u | 0x80000000)
    dr = d[r].cpu().numpy().astype(np.int64) & 0xffffffff
    cols, pos, klo = dr & 255, (dr >> 8) & 255, dr >> 16
    order = np.argsort(-key, kind="stable")
    true_rank = {int(c): n for n, c in enumerate(order[:k])}
    print(f"row {r}: slot col rank(true) keylo(true)")
    for p in range(k):
        c = int(cols[p])
        print(f"  {p:2d} {c:3d} {int(pos[p]):2d}({true_rank.get(c, -1):2d}) {int(klo[p]):04x}({int(key[c]) & 0xffff:04x})")
    np.save(os.path.join(ROOT, "gpurun_out", f"topk_diag2_row{r}.npy"), xr)
