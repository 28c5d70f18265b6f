#!/bin/bash
# r04 GPU call D: the forward summing long rows with fp64 LDS atomics (MAXK_FWD_F64) -- GPU
# parity of that build, then its bench A/B against the product build.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/fwd_f64
mkdir -p $O
MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/f64/libmaxk_hip.so timeout -k 10 600 \
  python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $O/pytest_f64.log 2>&1
tail -1 $O/pytest_f64.log
R=2 timeout -k 10 900 bash tools/ab_bench.sh "base f64" "--k 16" "--k 8" "--k 32" \
  "--graph products --k 8" "--graph products --k 32" "--graph proteins" "--graph flickr" \
  > $O/ab.txt 2>&1
cat $O/ab.txt
