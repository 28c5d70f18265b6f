#!/bin/bash
# r03: sharded GPU tests + a 2-rank bench rehearsal on one GPU (gloo-staged collectives, the
# pipelined gather mode and its unsharded self-check)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/dist; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_parity_gpu.py -x -q -m gpu -k "accumulate or dist" --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
for g in ${GRAPHS:-products reddit}; do
  MAXK_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --graph $g --steps 5 --warmup 2 \
    --no-cpu-baseline --no-rocsparse --no-cpu-spmm --dist-mode gather > $O/n2_$g.json 2> $O/n2_$g.err || { tail -20 $O/n2_$g.err; exit 1; }
  tail -1 $O/n2_$g.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['extra']; print('$g', d['value'], d['ms_per_step'], {k: x[k] for k in ('dist_check_fwd_max_rel_err','dist_check_bwd_max_rel_err','dist_mode','dist_pipeline','adjoint_rel_err')})"
done
