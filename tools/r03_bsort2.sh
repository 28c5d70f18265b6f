#!/bin/bash
# After the bsort auto rule: the whole GPU suite, then products k=4/8 benches (bsort + stream)
# and a kernel-stats profile of the k=8 bench.
set -eo pipefail
O=gpurun_out/bsort2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for k in 4 8; do
  timeout -k 10 300 python bench.py --graph products --k $k --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/products_k$k.json 2> $O/products_k$k.err
  python -c "import json; d=json.load(open('$O/products_k$k.json')); e=d['extra']; print('products k=$k', d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], e.get('edge_sel_stream'), d['roofline']['frac'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_k8 -o run --output-format csv -- python3 bench.py --graph products --k 8 --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/stats_k8.json 2> $O/stats_k8.err
echo done
