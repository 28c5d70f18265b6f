#!/bin/bash
# Pull entries pre-divided by row_div (MAXK_PULL_PRESCALE=1) vs the per-call G / row_div copy:
# parity tests, then the 3-layer SAGE epoch on the ordered community products graph and Reddit.
set -eo pipefail
O=gpurun_out/prescale; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_hybrid_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
tail -1 $O/test.log
for pre in 1 0; do
  MAXK_PULL_PRESCALE=$pre timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products_comm --reorder --no-library > $O/comm_p$pre.json 2> $O/comm_p$pre.err
  echo "products_comm ordered prescale=$pre $(cat $O/comm_p$pre.json)"
  MAXK_PULL_PRESCALE=$pre timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py reddit --no-library > $O/reddit_p$pre.json 2> $O/reddit_p$pre.err
  echo "reddit prescale=$pre $(cat $O/reddit_p$pre.json)"
done
echo prescale done
