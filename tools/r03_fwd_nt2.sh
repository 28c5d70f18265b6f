#!/bin/bash
# Size-based non-temporal forward output stores: parity (forward golden + full-size products),
# products k = 8 / 16 / 32 benches (k = 32 also with the edge-selector stream forced on), Reddit.
set -eo pipefail
O=gpurun_out/fwdnt2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forward or products" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--no-cpu-baseline --no-rocsparse --no-cpu-spmm"
run() { local n=$1; shift; timeout -k 10 300 env "$@" > $O/$n.json 2> $O/$n.err; python -c "import json; d=json.load(open('$O/$n.json')); e=d['extra']; print('$n', d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], e.get('edge_sel_stream'))"; }
run reddit python bench.py $B
for k in 8 16 32; do run products_k$k python bench.py --graph products --k $k $B; done
run products_k32_es1 MAXK_EDGE_SEL=1 python bench.py --graph products --k 32 $B
run products_k64_es1 MAXK_EDGE_SEL=1 python bench.py --graph products --k 64 $B
