#!/bin/bash
# r03: bench every preset (one JSON line each) into gpurun_out/r03/presets/; every GPU step
# under its own limit, the first failure ends the script.
set -o pipefail
O=gpurun_out/r03/presets; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; echo "$name $(python -c "import json,sys; d=json.load(open('$O/$name.json')); e=d['extra']; print(d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], e.get('edge_sel_stream'), d['roofline']['frac'])")"; }
run reddit --no-cpu-baseline --no-cpu-spmm
for g in products proteins flickr; do run $g --graph $g --no-cpu-baseline --no-cpu-spmm; done
for k in 8 32 64; do run reddit_k$k --k $k --no-cpu-baseline --no-rocsparse --no-cpu-spmm; done
for m in bucket csc atomic; do run reddit_$m --bwd-mode $m --no-cpu-baseline --no-rocsparse --no-cpu-spmm; done
for k in 8 16 64; do run products_k$k --graph products --k $k --no-cpu-baseline --no-rocsparse --no-cpu-spmm; done
run products_comm_ordered --graph products_comm --reorder --no-cpu-baseline --no-rocsparse --no-cpu-spmm
echo presets done
