"""Probe, not product: P processes generating the synthetic graph on ONE shared GPU at
once (the N-rank rehearsal's first stage), each timing make_graph and dumping its stack if
it runs past --stacks seconds.  Diagnoses the r01 N=4 rehearsal stall.
    python tools/share_probe.py --procs 4 [--graph reddit] [--stacks 90]"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    import faulthandler
    faulthandler.dump_traceback_later(a.stacks, exit=False)
    sys.path.insert(0, os.path.join(ROOT, "spgemm-prunning_amd"))
    import torch
    import maxk_graph
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    torch.ones(1, device=dev)
    torch.cuda.synchronize()
    t1 = time.time()
    P = maxk_graph.PRESETS[a.graph]
    E = P["E"] - ((P["E"] - P["V"]) % 2)
    steps = []
    rp, col = maxk_graph.make_graph(P["V"], E, P["alpha"], P["i0"], 1, dev, trace=steps)
    torch.cuda.synchronize()
    t2 = time.time()
    print(f"[child {os.getpid()}] init {t1 - t0:.1f}s make_graph {t2 - t1:.1f}s "
          f"E={col.numel()} stages {steps}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--graph", default="reddit")
    ap.add_argument("--stacks", type=float, default=90)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    t0 = time.time()
    ps = [subprocess.Popen([sys.executable, __file__, "--child", "--graph", a.graph,
                            "--stacks", str(a.stacks)]) for _ in range(a.procs)]
    rc = [p.wait() for p in ps]
    print(f"[parent] {a.procs} procs done in {time.time() - t0:.1f}s rc={rc}", flush=True)
    return max(abs(r) for r in rc)


if __name__ == "__main__":
    sys.exit(main())
