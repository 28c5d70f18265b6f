#!/bin/bash
# r04 GPU call D: the forward summing long rows with fp64 LDS atomics (MAXK_FWD_F64) -- GPU
# parity of that build, then its bench A/B against the product build.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/fwd_f64
mkdir -p $O gpurun_out/r04/topk
# the top-k with its bad-row check inside the ties branch: tests, then A/B against r03's kernel
if [ "${TOPK:-1}" = 1 ]; then
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k "topk" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r04/topk/pytest_topk3.log 2>&1
tail -1 gpurun_out/r04/topk/pytest_topk3.log
for rep in 1 2; do for v in base topk_r03; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so
  [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  for rows in 232965 2449029; do
    echo "== $v rows=$rows rep=$rep"
    MAXK_HIP_LIB=$lib timeout -k 10 120 python tools/topk_ab.py --rows $rows
  done
done; done > gpurun_out/r04/topk/topk_ab3.txt 2>&1
fi
for v in f64pf pf; do
  MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so timeout -k 10 600 \
    python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
R=1 timeout -k 10 900 bash tools/ab_bench.sh "base f64 f64p pf f64pf" "--k 16" "--k 8" \
  "--graph products --k 8" "--graph products --k 32" > $O/ab.txt 2>&1
cat $O/ab.txt
