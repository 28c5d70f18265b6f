"""Probe: every row of the top-k on the Gaussian input of tools/topk_gauss.py (seed 0,
[2449029, 256], the first tensor of that generator) against the OpenMP oracle, bit-exact
(values and selectors), for the library MAXK_HIP_LIB points at (a tools/tune.sh variant,
e.g. MAXK_TOPK_ROWS4_KMAX=64) or the product library.  Prints the differing rows and saves
their inputs to gpurun_out/topk_bad_<tag>_k<k>.npz (the r02 four-row k=48 mismatch hunt,
VERDICT r02 item 1).  Usage: python tools/topk_rows_probe.py TAG [k ...]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import maxk_cuda_kernels as mk  # noqa: E402
import oracle as O  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
ks = [int(a) for a in sys.argv[2:]] or [16, 32, 48, 64]
g = torch.Generator(device="cuda").manual_seed(0)
V = 2_449_029
x = torch.randn(V, 256, generator=g, device="cuda")
xh = x.cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
CH = 1 << 18
for k in ks:
    for _ in range(3):
        mk.topk_cbsr(x, k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mk.topk_cbsr(x, k)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    v, i = mk.topk_cbsr(x, k)
    vh, ih = v.cpu().numpy(), i.cpu().numpy()
    t0 = time.time()
    bad = []
    for r0 in range(0, V, CH):
        ov, oi = O.topk(xh[r0:r0 + CH], k)
        d = np.nonzero((ov.view(np.uint32) != vh[r0:r0 + CH].view(np.uint32)).any(1) |
                       (oi != ih[r0:r0 + CH]).any(1))[0]
        bad.extend((d + r0).tolist())
    tv = torch.topk(x, k, dim=1).values
    same_torch = bool(torch.equal(tv, v))
    print(f"{tag} k={k}: {sorted(ts)[5]:.4f} ms; rows differing from the oracle: {len(bad)} "
          f"of {V} (oracle {time.time() - t0:.1f} s); values equal torch.topk: {same_torch}",
          flush=True)
    if bad:
        print(f"  first rows: {bad[:20]}")
        rows = np.array(bad[:256])
        ov, oi = O.topk(xh[rows], k)
        np.savez(os.path.join(ROOT, "gpurun_out", f"topk_bad_{tag}_k{k}.npz"), rows=rows,
                 x=xh[rows], got_val=vh[rows], got_idx=ih[rows], ref_val=ov, ref_idx=oi)
        for r in rows[:3]:
            o_v, o_i = O.topk(xh[r:r + 1], k)
            diff = np.nonzero(o_i[0] != ih[r])[0]
            print(f"  row {r}: first differing slot {diff[:5]}, got idx {ih[r][diff[:5]]} "
                  f"ref idx {o_i[0][diff[:5]]}; got set == ref set: "
                  f"{set(ih[r].tolist()) == set(o_i[0].tolist())}")
