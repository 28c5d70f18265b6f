#!/bin/bash
# A/B of forward variants (lib/variants/*): bench live fwd ms on GRAPH at each k.
set -o pipefail
V=$PWD/spgemm-prunning_amd/lib/variants
G=${GRAPH:-products}; KS=$1; shift
for v in "$@"; do
  for k in $KS; do
    r=$(MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python bench.py --graph $G --k $k --steps 20 --no-cpu-baseline --no-rocsparse 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['extra']['fwd_ms'])") || exit 1
    echo "$v $G k=$k fwd_ms $r"
  done
done
