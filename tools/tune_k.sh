#!/bin/bash
# bench every library variant at several k: tools/tune_k.sh "8 16 32 64" [bench args]
cd "$(dirname "$0")/.."
KS=${1:-"8 16 32 64"}; shift
for v in $(ls spgemm-prunning_amd/lib/variants); do
  for k in $KS; do
    r=$(MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse --k $k "$@" 2>/dev/null) || { echo "$v k=$k FAILED"; exit 1; }
    echo "$v k=$k $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e["fwd_ms"], e["bwd_ms"])')"
  done
done
