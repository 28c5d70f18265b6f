#!/bin/bash
# Planted-community products-sized graph (maxk_graph PRESETS products_comm), randomly labelled
# and after maxk_graph.locality_order: bench lines per backward mode, halo bytes at N = 2/4/8.
set -eo pipefail
O=gpurun_out/locality; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py --graph products_comm --no-cpu-baseline --no-cpu-spmm "$@" > $O/$name.json 2> $O/$name.err; echo "$name $(python -c "import json; d=json.load(open('$O/$name.json')); e=d['extra']; print(d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], d['roofline']['frac'], e.get('pull_locality'), e.get('reorder_s'), e.get('rocsparse_spmm_ms'))")"; }
run random
run random_pull --bwd-mode pull --no-rocsparse
run ordered --reorder
run ordered_csc --reorder --bwd-mode csc --no-rocsparse
run ordered_hybrid --reorder --bwd-mode hybrid --no-rocsparse
run random_hybrid --bwd-mode hybrid --no-rocsparse
timeout -k 10 300 python tools/halo_bytes.py --graph products_comm --device cuda > $O/halo_random.txt 2>&1
timeout -k 10 300 python tools/halo_bytes.py --graph products_comm --device cuda --reorder > $O/halo_ordered.txt 2>&1
cat $O/halo_random.txt $O/halo_ordered.txt
echo locality done
