"""Probe (tools build, MAXK_TOPK_DIAG=3, MAXK_TOPK_ROWS4_KMAX=64): the failing row's LDS winner
region right after compaction (keys, values, columns), and each lane's slot start, winner
count, region offsets and final slot, from the dense-output channel of
maxk_topk_cbsr_dense."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

k = 48
g = torch.Generator(device="cuda").manual_seed(0)
V = 2_449_029
x = torch.randn(V, 256, generator=g, device="cuda")
dense, v, i = mk.topk_cbsr_dense(x, k)
ref = torch.topk(x, k, dim=1).values
bad = torch.nonzero((v != ref).any(1)).flatten().tolist()
print("bad rows", bad)
for r in bad[:2] + [bad[0] + 1, bad[0] - 1]:
    d = dense[r].view(torch.int32).cpu().numpy().astype(np.int64) & 0xffffffff
    xr = x[r].cpu().numpy()
    u = xr.view(np.uint32).astype(np.int64)
    key = np.where(u & 0x80000000, (~u) & 0xffffffff, u | 0x80000000)
    print(f"row {r}: lane slot_start {d[160:176].tolist()}")
    print(f"   nw {d[176:192].tolist()}")
    print(f"   wkey offset {d[192:208].tolist()}")
    print(f"   wcol offset {d[208:224].tolist()}")
    print(f"   slot end {d[224:240].tolist()}")
    kk, vv, cc = d[0:48], d[48:96], d[96:144]
    okk = [int(kk[p]) == int(key[int(cc[p])]) if cc[p] < 256 else False for p in range(48)]
    print(f"   key matches its column: {okk}")
    print(f"   cols {cc.tolist()}")
    print(f"   keys {[hex(int(a)) for a in kk]}")
