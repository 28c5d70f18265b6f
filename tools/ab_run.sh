#!/bin/bash
# A/B of library variants (tools/tune.sh): GPU parity subset per variant, then
# rocprofv3 kernel averages per bench configuration.  ARGS: one bench-arg string per config.
set -o pipefail
cd "$(dirname "$0")/.."
V=$PWD/spgemm-prunning_amd/lib/variants
for v in $(ls $V); do
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/ab_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 gpurun_out/ab_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab_$v.log)"
done
for a in "$@"; do echo "== $a"; bash tools/tune_prof.sh $a | grep -v "cbsr_pack\|slab_fixup\|iota\|bucket_ptr\|topk\|transpose\|radix\|Radix\|csc_ptr" || exit 1; done
