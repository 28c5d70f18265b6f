"""Probe, not product: maxk_cbsr_scatter_dense on an ogbn-products-sized [2.45M, 256] output
(k = 32) and a Reddit-sized one, HIP events per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

dev = torch.device("cuda")
for V, k in ((2449029, 32), (2449029, 16), (232965, 16)):
    x = torch.randn(V, 256, device=dev)
    cv, ci = mk.topk_cbsr(x, k)
    out = mk.cbsr_scatter_dense(cv, ci, 256)
    ref = torch.zeros(V, 256, device=dev).scatter_(1, ci.long(), cv)
    assert torch.equal(out, ref)
    for _ in range(3):
        mk.cbsr_scatter_dense(cv, ci, 256)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        mk.cbsr_scatter_dense(cv, ci, 256)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"V={V} k={k}: {ms:.3f} ms  ({V * 256 * 4 / ms / 1e6:.0f} GB/s of output)")
