"""Probe: top-k (maxk_topk_cbsr) time on Gaussian rows, the shape a Linear layer's output
has, for the products and Reddit sizes at k = 16 and 32 (median of 20 launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
for V in (2_449_029, 232_965):
    x = torch.randn(V, 256, generator=g, device="cuda")
    for k in (16, 32, 48, 64):
        for _ in range(3):
            mk.topk_cbsr(x, k)
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            mk.topk_cbsr(x, k)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        v, i = mk.topk_cbsr(x, k)
        ref = torch.topk(x, k, dim=1)
        # values bit-exact; indices point at them (torch's order among equal values differs:
        # ours takes the lower column first, as the oracle and the reference's CPU path do)
        same = torch.equal(v, ref.values) and torch.equal(x.gather(1, i.long()), v)
        print(f"gauss V={V} k={k}: {sorted(ts)[10]:.4f} ms, values match torch.topk: {same}")
