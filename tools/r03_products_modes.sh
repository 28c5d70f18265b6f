#!/bin/bash
# r03: ogbn-products-sized backward, every mode at k = 8 / 16 / 32 (bench lines), and the
# per-kernel split of csc under rocprofv3 --stats.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/products_modes; mkdir -p $O
export TMPDIR=/tmp
for k in ${KS:-8 16 32}; do
  for m in ${MODES:-csc bucket atomic}; do
    timeout -k 10 300 python -u bench.py --graph products --k $k --bwd-mode $m --steps 10 --warmup 3 \
      --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/k${k}_$m.json 2> $O/k${k}_$m.err || { tail -5 $O/k${k}_$m.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/k${k}_$m.json')); x=d['extra']; print('k=$k $m fwd %.3f bwd %.3f' % (x['fwd_ms'], x['bwd_ms']))"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k$k -o run --output-format csv -- \
    python3 bench.py --graph products --k $k --bwd-mode csc --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > /dev/null 2> $O/prof_k$k.err \
    || { tail -5 $O/prof_k$k.err; exit 1; }
  python3 tools/stats_summary.py $O/prof_k$k/run_kernel_stats.csv | grep -v "^ *$" | head -30
done
