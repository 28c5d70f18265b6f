"""Per-kernel averages of every PMC counter in the rocprofv3 passes under a directory
(<dir>/p*/run_counter_collection.csv), maxk:: kernels only, with each kernel's dispatch count,
and the bench line the first pass printed (its fwd / bwd medians).
    python tools/pmc_kernels.py gpurun_out/r04/pmc_set/reddit_k8"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if "maxk::" not in n:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(acc.items()):
    calls = max(len(v) for v in cs.values())
    print(f"{n}  (dispatches per counter: {calls})")
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v) / len(v):16.6g}")
for j in sorted(glob.glob(os.path.join(d, "p*.json")))[:1]:
    try:
        b = json.loads(open(j).read().strip().splitlines()[-1])
        e = b["extra"]
        print(f"bench: {b['config']['workload']}: fwd {e['fwd_ms']} ms, bwd {e['bwd_ms']} ms "
              f"({e['bwd_mode']}), {b['value']} GTEPS")
    except (ValueError, KeyError, IndexError):
        pass
