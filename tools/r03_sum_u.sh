#!/bin/bash
# r03: csc phase-2 depth (MAXK_SUM_U) on the products-sized graph at k = 32 / 16 (kernel times)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/sum_u; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/spgemm-prunning_amd/lib/variants
for k in 32 16; do
  for v in base sumu8 sumu2; do
    MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${v}_k$k -o run --output-format csv -- \
      python3 bench.py --graph products --k $k --bwd-mode csc --steps 8 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > /dev/null 2> $O/${v}_k$k.err \
      || { tail -5 $O/${v}_k$k.err; exit 1; }
    echo "== $v k=$k: $(python3 tools/stats_summary.py $O/${v}_k$k/run_kernel_stats.csv | grep -E '^maxk::csc_sum' | head -1)"
  done
done
