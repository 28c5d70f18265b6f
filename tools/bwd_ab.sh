#!/bin/bash
# A/B of backward variants (lib/variants/*): bench live bwd_ms on GRAPH at each k (BWD mode auto).
set -o pipefail
V=$PWD/spgemm-prunning_amd/lib/variants
G=${GRAPH:-products}; KS=$1; shift
for v in "$@"; do
  for k in $KS; do
    r=$(MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python bench.py --graph $G --k $k --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse ${BWD:+--bwd-mode $BWD} 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['extra']['bwd_ms'], d['extra']['bwd_mode'])") || exit 1
    echo "$v $G k=$k bwd_ms $r"
  done
done
