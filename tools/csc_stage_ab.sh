#!/bin/bash
# A/B of csc phase 2 with and without LDS-staged eid slots (lib/variants stage / nostage),
# products at k = 8 / 16 / 32: rocprofv3 kernel averages of csc_sum_kernel and phase 1
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for k in 8 16 32; do
  for v in stage nostage; do
    MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/csab/$v$k -o run --output-format csv -- python3 bench.py --graph products --k $k --bwd-mode csc --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse > /dev/null 2>&1 || { echo "$v $k FAILED"; exit 1; }
    python3 - "$v$k" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/csab/{sys.argv[1]}/run_kernel_stats.csv")):
    n = r["Name"]
    if "csc_sum_kernel" in n or "sspmm_bwd_kernel" in n:
        n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{sys.argv[1]:10s} {n[:50]:50s} {float(r['AverageNs'])/1e6:8.4f} ms")
PY
  done
done
