#!/bin/bash
# pull_sel4_kernel (four selectors per thread) vs pull_sel_kernel: parity and kernel times.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/sel4; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -k "pull_selector_kernels or backward_golden or pull_backward" > $O/test.log 2>&1
tail -1 $O/test.log
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse --steps 10 --warmup 3"
prof() { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$1 -o run --output-format csv -- python3 bench.py $B "${@:2}" > $O/$1.json 2> $O/$1.err
  python3 - "$O/$1" "$1" <<'PY'
import csv, glob, sys, json
d = json.load(open(sys.argv[1] + ".json")); e = d["extra"]
print(sys.argv[2], "bwd", e["bwd_ms"], e["bwd_mode"], e.get("hybrid_pull_edges_frac"), e.get("hybrid_pull_tiles"))
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "maxk::" in r["Name"]:
            n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            print(f"  {n[:50]:50s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e6:8.4f} ms")
PY
}
prof comm_ordered --graph products_comm --reorder
prof reddit
echo sel4 done
