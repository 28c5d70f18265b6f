#!/bin/bash
# Kernel times of the N=8 shards (all ranks, tools/shard_probe.py) on the community products
# graph: csc randomly labelled vs csc and hybrid in locality order.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/shard_prof; mkdir -p $O
p() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 tools/shard_probe.py --graph products_comm --worlds 8 --iters 5 "$@" > $O/$name.txt 2>&1
  echo "== $name"; tail -1 $O/$name.txt
  python3 - "$O/$name" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "maxk::" in r["Name"]:
            n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            print(f"  {n[:50]:50s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e6:8.4f} ms")
PY
}
MAXK_BWD_MODE=csc p random_csc
MAXK_BWD_MODE=csc p ordered_csc --reorder
p ordered_auto --reorder
echo shard prof done
