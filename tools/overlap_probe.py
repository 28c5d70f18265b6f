"""Probe, not product: does the csc backward's phase 2 of one call overlap usefully with the
phase 1 of another on a second stream?  (VERDICT r04 item 2's "interleave phase 1 of one column
half with phase 2 of the other".)  Two csc backward calls on the products-sized graph at k = 32:
  serial    A then B on one stream;
  together  A on stream 1 and B on stream 2 at once (phase 1 beside phase 1, then 2 beside 2);
  staggered B delayed on stream 2 by a sleep of about A's phase 1 (A's phase 2 beside B's phase
            1, the pattern a split-phase backward would produce).
If `staggered` beats `serial` by well more than `together` does, the mixed pair shares the
memory system better than two copies of one phase.
    python tools/overlap_probe.py [--graph products] [--k 32] [--sleep-ms 5.0]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
import maxk_cuda_kernels as mk  # noqa: E402
import maxk_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="products")
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--sleep-ms", type=float, default=5.0)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda")
D = maxk_graph.PRESETS[a.graph]["D"]
row_ptr, col = maxk_graph.synthetic_graph(a.graph, device="cuda")
V, E = row_ptr.numel() - 1, col.numel()
g = torch.Generator(device=dev).manual_seed(1)
val = torch.rand(E, generator=g, device=dev)
G = torch.rand(V, D, generator=g, device=dev)
_, ci = mk.topk_cbsr(torch.rand(V, D, generator=g, device=dev), a.k)
plan = mk.transpose_plan(col, V)
outs = [torch.empty(V, a.k, device=dev) for _ in range(2)]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def call(i, stream):
    with torch.cuda.stream(stream):
        mk.sspmm_backward(row_ptr, col, val, G, ci, out=outs[i], mode="csc", plan=plan,
                          validate=False)


# cycles per ms for torch.cuda._sleep: calibrate on this box
def sleep_cycles_per_ms():
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    torch.cuda._sleep(10_000_000)
    ev1.record()
    torch.cuda.synchronize()
    return 10_000_000 / ev0.elapsed_time(ev1)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(torch.cuda.current_stream())
        fn()
        ev1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    return sorted(ts)[len(ts) // 2]


cpm = sleep_cycles_per_ms()
main = torch.cuda.current_stream()


def serial():
    call(0, main)
    call(1, main)


def two(delay_ms):
    s1.wait_stream(main)
    s2.wait_stream(main)
    call(0, s1)
    if delay_ms > 0:
        with torch.cuda.stream(s2):
            torch.cuda._sleep(int(delay_ms * cpm))
    call(1, s2)
    main.wait_stream(s1)
    main.wait_stream(s2)


def sleep_only(delay_ms):
    with torch.cuda.stream(main):
        torch.cuda._sleep(int(delay_ms * cpm))


t_one = timed(lambda: call(0, main))
t_serial = timed(serial)
t_together = timed(lambda: two(0.0))
t_stag = timed(lambda: two(a.sleep_ms))
t_sleep = timed(lambda: sleep_only(a.sleep_ms))
print(f"{a.graph} V={V} E={E} D={D} k={a.k}: one csc backward {t_one:.3f} ms; two calls: "
      f"serial {t_serial:.3f}, together {t_together:.3f}, staggered by {a.sleep_ms} ms "
      f"{t_stag:.3f} (the sleep alone {t_sleep:.3f}; staggered minus the delay "
      f"{t_stag - t_sleep:.3f})")
torch.testing.assert_close(outs[0], outs[1])
