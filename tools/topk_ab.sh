#!/bin/bash
# A/B of top-k library variants on the same box: tools/topk_rows_probe.py per variant, ks
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
V=$PWD/spgemm-prunning_amd/lib/variants
KS=${KS:-16 32 48}
for rep in 1 2; do
for v in $(ls $V); do
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python -u tools/topk_rows_probe.py $v $KS > gpurun_out/r03/topk_ab_$v.txt 2>&1 || { cat gpurun_out/r03/topk_ab_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r03/topk_ab_$v.txt
done
done
