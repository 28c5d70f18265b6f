"""Probe, not product: CBSR encode (top-k) time on [V, 256] for several k, the library picked by
MAXK_HIP_LIB, checked against torch.topk.   python tools/topk_ab.py [--rows 2449029]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2449029)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
for dist in ("normal", "uniform"):
    x = (torch.randn if dist == "normal" else torch.rand)(a.rows, 256, device="cuda", generator=g)
    for k in (8, 16, 32):
        v, i = mk.topk_cbsr(x, k)
        tv, ti = torch.topk(x, k, dim=1)
        # values exact; indices point at them (GPU torch.topk orders ties arbitrarily, the
        # kernel takes the lowest column, as CPU torch does)
        assert torch.equal(v, tv) and torch.equal(x.gather(1, i.long()), v), (dist, k)
        for _ in range(3):
            mk.topk_cbsr(x, k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            mk.topk_cbsr(x, k)
        e.record()
        torch.cuda.synchronize()
        print(f"{dist:8s} [{a.rows}, 256] k={k:2d}: {s.elapsed_time(e) / a.iters:.3f} ms", flush=True)
