#!/bin/bash
# products presets (csc backward) and the products epoch after the csc phase-2 change
set -eo pipefail
O=gpurun_out/presets; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name $(python -c "import json,sys; d=json.load(open('$O/$name.json')); e=d['extra']; print(d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], d['roofline']['frac'])")"; }
run products --graph products --no-cpu-baseline --no-cpu-spmm
for k in 8 16 64; do run products_k$k --graph products --k $k --no-cpu-baseline --no-rocsparse; done
run reddit_csc --bwd-mode csc --no-cpu-baseline --no-rocsparse
timeout -k 10 600 python spgemm-prunning_amd/maxk_train_bench.py products > $O/train_products.json 2> $O/train_products.err; cat $O/train_products.json
echo presets done
