#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, no trace domains) over one command; prints the
# per-kernel mean of every counter for kernels matching $MATCH.
#   gpurun -- 'MATCH=pull_q bash tools/pmc_sets.sh OUT "SET1" "SET2" ... -- python3 tools/pull_ab.py --k 16 --slices 0 --iters 3'
set -o pipefail
O=$1; shift
sets=()
while [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- "$@" > $O/p$i.out 2> $O/p$i.err || { echo "pass $i ($set) failed rc=$?"; tail -3 $O/p$i.err; exit 1; }
done
python3 - $O "${MATCH:-pull}" <<'PY'
import csv, glob, sys, collections
o, match = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if match not in n:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(acc.items()):
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.4g}")
PY
