#!/bin/bash
# r03: pull backward row-slice count per k (two repeats), and 4-slot parts at k = 8
# (MAXK_PULL_MIN_KP=4: two parts of 4 slots, 4096-destination buckets)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/pull_slices; mkdir -p $O
V=$PWD/spgemm-prunning_amd/lib/variants
run() {  # variant k slices...
  local v=$1 k=$2; shift 2
  echo "## $v k=$k" | tee -a $O/times.txt
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python -u tools/pull_ab.py --graph reddit --k $k \
    --slices "$@" --iters 30 2>&1 | grep -v amdgpu.ids | tee -a $O/times.txt || exit 1
}
for rep in 1 2; do
  run base 16 20 24 28 33 20 24 28 33
  run base 8 36 44 52 66 36 44 52 66
  run base 32 24 28 33 40 24 28 33 40
  run minkp4 8 0 22 33 44
done
