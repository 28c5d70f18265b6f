#!/bin/bash
# Bench every preset (one JSON line each) and the two training epochs into gpurun_out/presets/;
# every GPU step under its own limit, the first failure ends the script.
set -eo pipefail
O=gpurun_out/presets; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name $(python -c "import json,sys; d=json.load(open('$O/$name.json')); e=d['extra']; print(d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], d['roofline']['frac'])")"; }
run reddit --no-cpu-baseline --no-cpu-spmm
for g in products proteins flickr; do run $g --graph $g --no-cpu-baseline --no-cpu-spmm; done
for k in 8 32 64; do run reddit_k$k --k $k --no-cpu-baseline --no-rocsparse; done
for m in bucket csc atomic; do run reddit_$m --bwd-mode $m --no-cpu-baseline --no-rocsparse; done
for k in 8 16 64; do run products_k$k --graph products --k $k --no-cpu-baseline --no-rocsparse; done
echo presets done
