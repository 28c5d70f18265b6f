#!/bin/bash
# PMC passes (one rocprofv3 run each, no trace domains) over tools/pull_ab.py at one k:
# texture addresser / L1 / L2 traffic and SQ instruction mix of the pull backward kernels.
#   gpurun -- 'bash tools/pmc_pull.sh r02 16'   (MAXK_HIP_LIB selects a variant)
set -o pipefail
R=${1:-r02}; K=${2:-16}; O=gpurun_out/$R/pmc_pull_k$K; mkdir -p $O
export TMPDIR=/tmp
PROG="tools/pull_ab.py --graph ${GRAPH:-reddit} --k $K --slices 0 --iters 3"
i=0
for set in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_TA_BUSY_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 $PROG > $O/p$i.out 2> $O/p$i.err || { echo "pass $i ($set) failed rc=$?"; tail -3 $O/p$i.err; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if "pull" not in n and "bucket_sum" not in n:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(acc.items()):
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.4g}")
PY
