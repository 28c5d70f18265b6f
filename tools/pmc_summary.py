#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

FETCH_SIZE/WRITE_SIZE are KB; on gfx950 FETCH_SIZE reads 1/2 of wide streaming
bytes (MI355X_MICROARCH.md, HBM) -- the corrected column doubles it.  r06 validated the
doubling for every product kernel, sub-line gathers included: their fabric reads are all
128-B requests (TCC_EA0_RDREQ_128B_sum / TCC_EA0_RDREQ_sum >= 0.999), tallied at 64 B each
(tools/fetch_probe.hip, profiles/r06/fetch_calibration/).

  pmc_summary.py CSV... [--traffic-out profiles/rNN/traffic.json --key WORKLOAD]

With --traffic-out, per-op HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE summed over
the op's kernels, bench.OP_KERNELS) are merged into that JSON under WORKLOAD (bench.py's
traffic_key, e.g. reddit-D256-k16-csc-n1), where bench.py reads them as roofline.traffic.
When the CSVs also hold a TCP_TOTAL_CACHE_ACCESSES_sum pass (the texture path's tag
accesses, r05), the op's tag accesses per launch go beside them ("tag_accesses"), and
GRBM_GUI_ACTIVE ("gui_active", summed over the 8 XCDs): bench.py's roofline.binding.
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def base(n):
    """Kernel name without namespace; template arguments dropped except where they tell
    two ops apart (slab_fixup_kernel<0> forward, <1> backward)."""
    n = short(n).replace("maxk::", "")
    return n if n.startswith("slab_fixup_kernel<") else n.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--traffic-out")
    ap.add_argument("--key")
    a = ap.parse_args()
    d = collections.defaultdict(list)
    for p in a.csv:
        for r in csv.DictReader(open(p)):
            if "maxk" not in r["Kernel_Name"]:
                continue
            d[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    per_kernel = collections.defaultdict(dict)  # base name -> counter -> mean bytes
    n_disp = {}
    for (k, c), v in sorted(d.items()):
        m = sum(v) / len(v)
        extra = ""
        if c == "FETCH_SIZE":
            extra = f"  -> {m * 1024 / 1e9:.3f} GB raw, {2 * m * 1024 / 1e9:.3f} GB x2-corrected"
        elif c == "WRITE_SIZE":
            extra = f"  -> {m * 1024 / 1e9:.3f} GB"
        if c in ("TCP_TOTAL_CACHE_ACCESSES_sum", "GRBM_GUI_ACTIVE"):
            prev = per_kernel[base(k)].get(c)
            if prev is None or len(v) > n_disp[(base(k), c)]:
                per_kernel[base(k)][c] = m
                n_disp[(base(k), c)] = len(v)
        if c in ("FETCH_SIZE", "WRITE_SIZE"):
            # template variants of one kernel (e.g. a validating call's plain forward beside
            # the timed emitting one): the variant with the most dispatches stands for it
            prev = per_kernel[base(k)].get(c)
            if prev is None or len(v) > n_disp[(base(k), c)]:
                per_kernel[base(k)][c] = m * 1024
                n_disp[(base(k), c)] = len(v)
        print(f"{k[:48]:48s} {c:14s} n={len(v):3d} mean={m:.5g}{extra}")
    if a.traffic_out:
        from bench import OP_KERNELS
        out = {}
        if os.path.exists(a.traffic_out):
            out = json.load(open(a.traffic_out))
        ops = {}
        for op, ks in OP_KERNELS.items():
            # the op ran if one of its own kernels did (the shared fixups alone do not count:
            # the forward's record route and dense route share slab_fixup_kernel<0>)
            if not any(k in per_kernel for k in ks if not k.startswith("slab_fixup")):
                continue
            if op.startswith("sspmm_backward_") and f"-{op.rsplit('_', 1)[1]}-" not in a.key:
                continue  # the key names the backward mode the counters were taken in
            f = sum(per_kernel.get(k, {}).get("FETCH_SIZE", 0.0) for k in ks)
            w = sum(per_kernel.get(k, {}).get("WRITE_SIZE", 0.0) for k in ks)
            ops[op] = {"bytes": int(2 * f + w), "fetch_raw": int(f), "write": int(w),
                       "kernels": {k: per_kernel.get(k, {}) for k in ks}}
            tags = [per_kernel.get(k, {}).get("TCP_TOTAL_CACHE_ACCESSES_sum") for k in ks]
            if any(t is not None for t in tags):
                ops[op]["tag_accesses"] = int(sum(t or 0.0 for t in tags))
                ops[op]["gui_active"] = int(sum(per_kernel.get(k, {}).get("GRBM_GUI_ACTIVE", 0.0)
                                                for k in ks))
        out[a.key] = ops
        with open(a.traffic_out, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
        print(f"wrote {a.traffic_out} [{a.key}]: " +
              ", ".join(f"{op} {v['bytes'] / 1e9:.3f} GB" for op, v in ops.items()))


if __name__ == "__main__":
    main()
