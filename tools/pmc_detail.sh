#!/bin/bash
# Detail PMC passes (one rocprofv3 run each) over the default bench: L2 hit/miss and
# fabric credit stalls, SQ wave/instruction cycles, TCP/TA latency and busy.
#   gpurun -- 'bash tools/pmc_detail.sh r01'
set -eo pipefail
R=${1:-r01}; O=gpurun_out/$R/pmc_detail; mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm ${BENCH_ARGS:-}"
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 $BENCH > $O/p$i.json 2> $O/p$i.err
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if "maxk::" not in n:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(acc.items()):
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.4g}")
PY
