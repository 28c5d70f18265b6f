#!/bin/bash
# r03: bound the gain of a destination-ordered contribution layout on ogbn-products-sized
# graphs at small k: phase 1 with scattered row stores (MAXK_BWD_ABL=8) and phase 2 reading
# rows in order (MAXK_BWD_ABL=4), per-kernel times under rocprofv3 --stats (wrong results:
# tuning builds only).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/products_layout; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/spgemm-prunning_amd/lib/variants
for k in ${KS:-8 16 32}; do
  for v in ${VARIANTS:-base abl4 abl8}; do
    MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${v}_k$k -o run --output-format csv -- \
      python3 bench.py --graph products --k $k --bwd-mode csc --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > /dev/null 2> $O/${v}_k$k.err \
      || { tail -5 $O/${v}_k$k.err; exit 1; }
    echo "== $v k=$k"
    python3 tools/stats_summary.py $O/${v}_k$k/run_kernel_stats.csv | grep -E "sspmm_bwd_kernel|csc_sum_kernel"
  done
done
