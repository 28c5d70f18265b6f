#!/bin/bash
# Forward record pack, four l per thread (default build) vs one (variant nopack4): parity
# tests, then per-kernel times on products (k=32), Reddit (k=16) and the N=8 ordered shards.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/pack4; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "forward or duplicate or past_D or random_graphs or fused" > $O/test.log 2>&1
tail -1 $O/test.log
B="--steps 10 --warmup 3 --no-cpu-baseline --no-cpu-spmm --no-rocsparse"
for v in default nopack4; do
  if [ $v = default ]; then unset MAXK_HIP_LIB; else export MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; fi
  for cfg in "reddit" "products --graph products"; do
    set -- $cfg; n=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${v}_$n -o run --output-format csv -- python3 bench.py $B "$@" > $O/${v}_$n.json 2> $O/${v}_$n.err
    python3 - "$O/${v}_$n" "$v $n" <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[1] + ".json")); e = d["extra"]
out = [sys.argv[2], "fwd", e["fwd_ms"]]
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pack" in r["Name"]:
            out += [r["Name"].split("(")[0].split("::")[-1], round(float(r["AverageNs"]) / 1e6, 4)]
print(*out)
PY
  done
done
echo pack4 done
