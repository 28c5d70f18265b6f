#!/bin/bash
# The sharded path with the window-sorted backward: dist GPU tests (incl. forced bsort / csc at
# world 2), per-rank shard times at N = 8 for products k = 8, and a 2-rank bench rehearsal on
# the one GPU (gloo-staged collectives) that checks itself against the unsharded result.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/dist_bsort; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_dist_gpu.py tests/test_parity_gpu.py -x -q -m gpu -k "dist or accumulate" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log

MAXK_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --graph products --k 8 --steps 5 --warmup 2 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/n2_products_k8.json 2> $O/n2_products_k8.err || { tail -20 $O/n2_products_k8.err; exit 1; }
python -c "import json; d=json.loads(open('$O/n2_products_k8.json').read().splitlines()[-1]); e=d['extra']; print('n2 products k8', d['value'], e['bwd_mode'], e.get('dist_check_fwd_max_rel_err'), e.get('dist_check_bwd_max_rel_err'))"
