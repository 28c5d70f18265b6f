#!/usr/bin/env python3
"""Per-op summary of a rocprofv3 --kernel-trace --stats run of bench.py.

  stats_summary.py RUN_kernel_stats.csv [bench.json]

Sums the average durations of each op's kernels (bench.OP_KERNELS) so they can be set
beside the bench line's live HIP-event fwd_ms / bwd_ms."""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import OP_KERNELS  # noqa: E402


def base(n):
    """Kernel name without namespace; template arguments dropped except where they tell
    two ops apart (slab_fixup_kernel<0> forward, <1> backward)."""
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    n = n.split("(")[0].replace("maxk::", "")
    return n if n.startswith("slab_fixup_kernel<") else n.split("<")[0]


def main(stats, bench=None):
    rows = list(csv.DictReader(open(stats)))
    avg, calls = {}, {}
    print(f"{'kernel':64s} {'calls':>5s} {'avg_ms':>9s} {'min_ms':>9s} {'max_ms':>9s}")
    for r in rows:
        if "maxk::" not in r["Name"]:
            continue
        b = base(r["Name"])
        if int(r["Calls"]) > calls.get(b, 0):  # template variants: the most-called one
            avg[b], calls[b] = float(r["AverageNs"]) / 1e6, int(r["Calls"])
        nm = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{nm[:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e6:9.4f}"
              f" {float(r['MinNs']) / 1e6:9.4f} {float(r['MaxNs']) / 1e6:9.4f}")
    line = json.load(open(bench)) if bench else None
    print()
    for op, ks in OP_KERNELS.items():
        if not all(k in avg for k in ks[:2]):
            continue
        if op.startswith("sspmm_backward_") and line and \
                line["extra"]["bwd_mode"] != op.rsplit("_", 1)[1]:
            continue
        t = sum(avg.get(k, 0.0) for k in ks)
        live = ""
        if line:
            live = f"   bench live HIP events: {line['extra']['fwd_ms' if 'forward' in op else 'bwd_ms']} ms"
        print(f"op {op:24s} = {' + '.join(ks)}: {t:.4f} ms per launch{live}")


if __name__ == "__main__":
    main(*sys.argv[1:])
