set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/b2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket or backward or all_k or high_degree or empty or zero_rows or overwritten or rectangular" > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for k in 16 8 4; do echo "== k=$k"; bash tools/tune_prof.sh --k $k --bwd-mode bucket 2>&1 | grep -E "==|bucket|FAILED"; done
