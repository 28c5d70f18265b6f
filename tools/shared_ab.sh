#!/bin/bash
# r04: the 8-lane forward with two edge groups per LDS copy (MAXK_FWD_SHARED) -- parity of the
# product build's new dense small-k test and of the variant, then an order-controlled A/B on
# the dense graphs that take 8 lanes at k <= 8.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/fwd_shared
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "dense_small_k" -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_base_dense.log 2>&1
echo "base dense: $(tail -n 1 $O/pytest_base_dense.log)"
MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/shared/libmaxk_hip.so timeout -k 10 600 \
  python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_shared.log 2>&1
echo "shared: $(tail -n 1 $O/pytest_shared.log)"
R=3 timeout -k 10 800 bash tools/ab_bench.sh "shared base" "--k 8" "--k 4 --no-rocsparse" \
  "--graph proteins --k 8 --no-rocsparse" 2>&1 | tee $O/ab.txt
