#!/bin/bash
# r03: destination-sorted backward (mode "sorted") against csc / bucket on the ogbn-products-
# and Reddit-sized graphs at k = 8 / 16: parity subset, then per-kernel times (rocprofv3 --stats)
# per library variant (plain / nt positional stores).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/sorted; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "backward_golden" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=$PWD/spgemm-prunning_amd/lib/variants
for g in ${GRAPHS:-products reddit}; do
for k in ${KS:-8 16}; do
  for v in ${VARIANTS:-base posnt}; do
    for m in ${MODES:-sorted csc}; do
      [ "$v" != base ] && [ "$m" != sorted ] && continue
      MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${g}_${v}_${m}_k$k -o run --output-format csv -- \
        python3 bench.py --graph $g --k $k --bwd-mode $m --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/${g}_${v}_${m}_k$k.json 2> $O/${g}_${v}_${m}_k$k.err \
        || { tail -5 $O/${g}_${v}_${m}_k$k.err; exit 1; }
      echo "== $g $v $m k=$k: $(python3 -c "import json; x=json.load(open('$O/${g}_${v}_${m}_k$k.json'))['extra']; print('bwd', x['bwd_ms'], 'adjoint', x.get('adjoint_rel_err'))")"
      python3 tools/stats_summary.py $O/${g}_${v}_${m}_k$k/run_kernel_stats.csv | grep -E "sspmm_bwd_kernel|csc_sum_kernel|bucket_sum|bucket_fixup"
    done
  done
done
done
