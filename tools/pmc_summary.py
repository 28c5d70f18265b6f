#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).
FETCH_SIZE/WRITE_SIZE are KB; on gfx950 FETCH_SIZE reads 1/2 of wide streaming
bytes (MI355X_MICROARCH.md, HBM) -- the corrected column doubles it."""
import collections
import csv
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(paths):
    d = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if "maxk" not in r["Kernel_Name"]:
                continue
            d[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(d.items()):
        m = sum(v) / len(v)
        extra = ""
        if c == "FETCH_SIZE":
            extra = f"  -> {m * 1024 / 1e9:.3f} GB raw, {2 * m * 1024 / 1e9:.3f} GB x2-corrected"
        elif c == "WRITE_SIZE":
            extra = f"  -> {m * 1024 / 1e9:.3f} GB"
        print(f"{k[:48]:48s} {c:14s} n={len(v):3d} mean={m:.5g}{extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
