#!/bin/bash
# A/B of forward variants (lib/variants/*) on every preset graph: the bench's live fwd_ms.
set -o pipefail
V=$PWD/spgemm-prunning_amd/lib/variants
for v in "$@"; do
  for g in flickr products reddit proteins; do
    r=$(MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python bench.py --graph $g --steps 20 --no-cpu-baseline --no-rocsparse 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); e=d['extra']; print(e['fwd_ms'], e['bwd_ms'], d['value'])") || exit 1
    echo "$v $g fwd/bwd/GTEPS $r"
  done
done
