#!/bin/bash
# Run bench.py once per library variant (and a few chunk sizes on the base build).
# Output: one line per run to stdout. Used under gpurun.
cd "$(dirname "$0")/.."
for v in $(ls spgemm-prunning_amd/lib/variants); do
  r=$(MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse "$@" 2>/dev/null) || { echo "$v FAILED"; exit 1; }
  echo "$v $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e["fwd_ms"], e["bwd_ms"])')"
done
for c in ${CHUNKS:-}; do
  r=$(timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse --chunk $c "$@" 2>/dev/null) || { echo "chunk $c FAILED"; exit 1; }
  echo "chunk$c $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e["fwd_ms"], e["bwd_ms"])')"
done
