#!/bin/bash
# Hybrid backward: tile kernels on a side stream beside the csc (MAXK_HYBRID_STREAMS=1) vs in line.
set -eo pipefail
O=gpurun_out/hybrid_streams; mkdir -p $O
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse"
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']; print(sys.argv[2], d['value'], 'fwd', e['fwd_ms'], 'bwd', e['bwd_ms'], e['bwd_mode'], 'frac', d['roofline']['frac'], 'loc', e.get('pull_locality'))" "$@"; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py $B "$@" > $O/$name.json 2> $O/$name.err; line $O/$name.json $name; }
timeout -k 10 400 python3 -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
tail -1 $O/test.log
for st in 1 0; do
  MAXK_HYBRID_STREAMS=$st run ordered_s$st --graph products_comm --reorder
  MAXK_HYBRID_STREAMS=$st run p50_s$st --graph products_comm_p50 --reorder
done
echo streams probe done
