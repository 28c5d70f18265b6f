"""Probe: run the four-row top-k (variant library, MAXK_HIP_LIB) on slices of the rows
around the k=48 mismatch (gpurun_out/topk_diag_k48.npz: rows bad-64 .. bad+63 of the seed-0
Gaussian input), to see whether the failure is a function of the row alone, of its wave's
four rows, or of more."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

z = np.load(os.path.join(ROOT, "tools", "_probe", "topk_diag_k48.npz"))
X = torch.from_numpy(z["x"]).cuda()
k = 48
b = 64  # the bad row's index in X


def check(name, x):
    v, i = mk.topk_cbsr(x.contiguous(), k)
    ref = torch.topk(x, k, dim=1).values
    bad = torch.nonzero((v != ref).any(1)).flatten().tolist()
    print(f"{name}: rows {x.shape[0]}, differing {bad}", flush=True)


check("all 128", X)
check("bad row alone", X[b:b + 1])
check("bad row's wave (4 rows)", X[b:b + 4])
check("bad row as sub 1", X[b - 1:b + 3])
check("bad row as sub 3", X[b - 3:b + 1])
check("bad row x4", X[b:b + 1].repeat(4, 1))
check("bad row x64", X[b:b + 1].repeat(64, 1))
for D in (256,):
    xs = X[b:b + 1].clone()
    # perturb: negate, scale
    check("bad row * 2", xs * 2)
    check("bad row + 1", xs + 1)
    check("bad row reversed columns", xs.flip(1))
