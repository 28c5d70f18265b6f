#!/usr/bin/env python3
"""Summarise tools/fetch_probe.hip's rocprofv3 --pmc passes.

For every probe kernel: the bytes it requested, the fabric read requests split by size
(TCC_EA0_RDREQ_sum, _32B_sum, _128B_sum; the rest are 64-B requests), the bytes those requests
carry (32 n32 + 64 n64 + 128 n128), and rocprofv3's FETCH_SIZE beside them: the ratio is the
correction FETCH_SIZE needs for that access pattern (the guide's x2 is the all-128-B case).
Also the analytic distinct 128-B lines and 64-B sectors per record at stride R.

  fetch_probe_summary.py PROBE_LOG CSV...
"""
import collections
import csv
import re
import sys


def per_record(R):
    """(128-B lines, 64-B sectors) one R-byte record at stride R touches, averaged over the
    offsets the stride cycles through."""
    lines = sectors = 0
    for i in range(128):
        o = (i * R) % 128
        lines += (o + R - 1) // 128 + 1
        sectors += (o + R - 1) // 64 - o // 64 + 1
    return lines / 128, sectors / 128


def main():
    log, csvs = sys.argv[1], sys.argv[2:]
    req = {}
    for ln in open(log):
        m = re.match(r"(\S+) table (\d+) MiB.*?bytes_requested (\d+) ms ([\d.]+)", ln)
        if m:
            req[m.group(1)] = (int(m.group(2)), int(m.group(3)), float(m.group(4)))
    d = collections.defaultdict(list)
    for p in csvs:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("void ", "").split("(")[0].replace(" ", "")
            d[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in d.items()}
    print(f"{'kernel':24s} {'MiB':>5s} {'req GB':>7s} {'ms':>7s} {'RDREQ':>10s} {'32B':>6s} "
          f"{'128B %':>6s} {'by-size GB':>10s} {'FETCH GB':>9s} {'factor':>6s} "
          f"{'lines/rec':>9s} {'sect/rec':>8s}")
    for name, (mib, nbytes, ms) in req.items():
        key = name.replace(" ", "")
        n = mean.get((key, "TCC_EA0_RDREQ_sum"))
        n32 = mean.get((key, "TCC_EA0_RDREQ_32B_sum"), 0.0)
        n128 = mean.get((key, "TCC_EA0_RDREQ_128B_sum"), 0.0)
        fetch = mean.get((key, "FETCH_SIZE"))
        by_size = None if n is None else 32 * n32 + 128 * n128 + 64 * (n - n32 - n128)
        m = re.match(r"gather_rec<(\d+)", name)
        lr, sr = per_record(int(m.group(1))) if m else (float("nan"), float("nan"))
        f = lambda x, s=1e9, w=9, p=3: (f"{x / s:{w}.{p}f}" if x is not None else " " * (w - 1) + "-")  # noqa
        print(f"{name:24s} {mib:5d} {nbytes / 1e9:7.3f} {ms:7.4f} "
              f"{(n or 0):10.4g} {n32:6.2g} {100 * n128 / n if n else 0:6.1f} "
              f"{f(by_size, w=10)} {f(None if fetch is None else fetch * 1024, w=9)} "
              f"{(by_size / (fetch * 1024)) if (by_size and fetch) else float('nan'):6.3f} "
              f"{lr:9.3f} {sr:8.3f}")


if __name__ == "__main__":
    main()
