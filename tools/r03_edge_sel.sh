#!/bin/bash
# r03: edge-selector stream (forward emits, csc backward reads): parity subset, the probe, and
# the products bench lines (csc, stream on / off)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/edge_sel; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_layers_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/edge_sel_probe.py --graph products 2>&1 | grep -v amdgpu.ids | tee $O/probe_products.txt || exit 1
timeout -k 10 200 python -u tools/edge_sel_probe.py --graph reddit --k 16 2>&1 | grep -v amdgpu.ids | tee $O/probe_reddit.txt || exit 1
for k in 8 16 32; do
  for es in auto 0; do
    MAXK_EDGE_SEL=$es timeout -k 10 300 python -u bench.py --graph products --k $k --steps 10 --warmup 3 \
      --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/products_k${k}_es$es.json 2> $O/products_k${k}_es$es.err || { tail -5 $O/products_k${k}_es$es.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/products_k${k}_es$es.json')); x=d['extra']; print('products k=$k es=$es', d['value'], 'fwd', x['fwd_ms'], 'bwd', x['bwd_ms'], x['bwd_mode'], x['edge_sel_stream'], 'frac', d['roofline']['frac'])"
  done
done
