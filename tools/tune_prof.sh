#!/bin/bash
# per-kernel average durations (rocprofv3 --stats) of the bench for every library variant
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in $(ls spgemm-prunning_amd/lib/variants); do
  MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp/$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse "$@" > /dev/null 2>&1 || { echo "$v FAILED"; exit 1; }
  echo "== $v"; python3 - "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/tp/{sys.argv[1]}/run_kernel_stats.csv")):
    if "maxk::" in r["Name"]:
        n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"  {n[:50]:50s} {float(r['AverageNs'])/1e6:8.4f} ms")
PY
done
