#!/bin/bash
# A/B of library variants (tools/tune.sh builds them under lib/variants/NAME) on bench
# configurations: the bench's live fwd / bwd medians and GTEPS, variants interleaved per
# configuration and repeated R times (box-to-box noise is larger than run-to-run).
#   bash tools/ab_bench.sh "base snt" "--graph products --k 8" "--graph products --k 32"
# "base" is the product library (spgemm-prunning_amd/lib).  R=2 by default.
set -o pipefail
cd "$(dirname "$0")/.."
VARS=$1; shift
V=$PWD/spgemm-prunning_amd/lib/variants
for a in "$@"; do
  for rep in $(seq ${R:-2}); do
    for v in $VARS; do
      lib=$V/$v/libmaxk_hip.so
      [ "$v" = base ] && lib=$PWD/spgemm-prunning_amd/lib/libmaxk_hip.so
      r=$(MAXK_HIP_LIB=$lib timeout -k 10 300 python bench.py $a --steps 10 --warmup 3 \
          --no-cpu-baseline --no-rocsparse --no-cpu-spmm 2>/dev/null | python -c "
import json, sys
d = json.load(sys.stdin); e = d['extra']
print(e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], e['edge_sel_stream'], d['value'])") || exit 1
      echo "$a | $v | fwd bwd mode stream GTEPS: $r"
    done
  done
done
