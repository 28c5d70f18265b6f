#!/bin/bash
# forward item order A/B (lib/variants base / fxcd): bench lines on Reddit, products and the
# planted-community products graph in its locality order
cd "$(dirname "$0")/.."
for v in ${VARIANTS:-base fxcd}; do
  for g in ${GRAPHS:-"--graph reddit" "--graph products" "--graph products_comm --reorder"}; do
    r=$(MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-spmm --no-rocsparse $g 2>/dev/null) || { echo "$v $g FAILED"; exit 1; }
    echo "$v $g fwd_ms=$(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["fwd_ms"], d["extra"]["bwd_ms"])')"
  done
done
