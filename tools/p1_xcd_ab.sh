#!/bin/bash
# backward phase-1 item order A/B (lib/variants base / p1xcd): products (csc), the ordered
# planted-community graph (csc) and Reddit with --bwd-mode csc
cd "$(dirname "$0")/.."
for v in base p1xcd; do
  for g in "--graph products" "--graph products_comm --reorder" "--graph reddit --bwd-mode csc"; do
    r=$(MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-spmm --no-rocsparse $g 2>/dev/null) || { echo "$v $g FAILED"; exit 1; }
    echo "$v $g fwd/bwd ms $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["fwd_ms"], d["extra"]["bwd_ms"], d["extra"]["bwd_mode"])')"
  done
done
