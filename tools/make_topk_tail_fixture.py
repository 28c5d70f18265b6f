"""Writes tests/golden/topk/topk_tail_overflow.npz (run on the GPU box; needs torch's HIP generator):
the two rows of the seed-0 [2449029, 256] Gaussian input (tools/topk_gauss.py) behind r02's
four-row top-k mismatch at k = 48 -- row 2186888, whose LDS winners were overwritten, and row
2449028, the last row, whose clamped copy the dead sub-rows of the final row group compacted
past their LDS region -- with their oracle top-k for k in {16, 32, 48, 64}, and the recipe to
rebuild the whole input (tests/test_fullsize_gpu.py::test_topk_tail_rows_fixture)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

V, D = 2_449_029, 256
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(V, D, generator=g, device="cuda")
rows = np.array([2186888, V - 1])
xr = x[torch.from_numpy(rows).cuda()].cpu().numpy()
out = {"rows": rows, "x": xr, "V": np.int64(V), "D": np.int64(D), "seed": np.int64(0)}
for k in (16, 32, 48, 64):
    v, i = O.topk(xr, k)
    out[f"val_k{k}"], out[f"idx_k{k}"] = v, i
os.makedirs(os.path.join(ROOT, "tests", "golden", "topk"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "topk", "topk_tail_overflow.npz"), **out)
print("wrote", {k: a.shape for k, a in out.items()})
