#!/bin/bash
# r03: four-row top-k k=48 mismatch, hypothesis variants on the seed-0 Gaussian input
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
V=$PWD/spgemm-prunning_amd/lib/variants
for v in "$@"; do
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 200 python -u tools/topk_rows_probe.py $v 48 > gpurun_out/r03/topk_hyp_$v.txt 2>&1 || { cat gpurun_out/r03/topk_hyp_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r03/topk_hyp_$v.txt
done
