#!/bin/bash
# r03: pull backward work order (MAXK_PULL_ORDER) x row-slice count, Reddit-sized graph, per k;
# then the L2 counters of the default build at k = 16 and 8.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/pull_order; mkdir -p $O
V=$PWD/spgemm-prunning_amd/lib/variants
for v in ${VARIANTS:-base ord1}; do
  for k in ${KS:-16 32 8}; do
    echo "## $v k=$k" | tee -a $O/times.txt
    MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 150 python -u tools/pull_ab.py --graph reddit --k $k \
      --slices ${SLICES:-0 24 44 66} --iters 20 2>&1 | grep -v amdgpu.ids | tee -a $O/times.txt || exit 1
  done
done
[ -n "$NOPMC" ] && exit 0
export TMPDIR=/tmp
for k in 16 8; do
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCC_EA0_RDREQ_sum" \
             "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE"; do
    i=$((i+1))
    MAXK_HIP_LIB=$V/${PMCV:-base}/libmaxk_hip.so timeout -s KILL 90 rocprofv3 --pmc $set -d $O/k${k}_p$i -o run --output-format csv -- \
      python3 tools/pull_ab.py --graph reddit --k $k --slices 0 --iters 3 > $O/k${k}_p$i.out 2> $O/k${k}_p$i.err \
      || { echo "pass $i ($set) failed"; tail -3 $O/k${k}_p$i.err; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for k in (16, 8):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{o}/k{k}_p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if "pull_q" not in n:
                continue
            acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in sorted(acc.items()):
        print(f"k={k} {n}")
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v)/len(v):16.4g}  (n={len(v)})")
PY
