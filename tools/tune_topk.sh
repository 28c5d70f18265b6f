#!/bin/bash
# top-k encode time per library variant and graph: tools/tune_topk.sh "reddit products"
cd "$(dirname "$0")/.."
for v in $(ls spgemm-prunning_amd/lib/variants); do
  for g in ${1:-reddit products}; do
    r=$(MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rocsparse --graph $g 2>/dev/null) || { echo "$v $g FAILED"; exit 1; }
    echo "$v $g topk_ms=$(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["topk_ms"], d["config"]["k"])')"
  done
done
