#!/bin/bash
# Reddit-sized graph relabelled by decreasing degree: does the pull backward gain when heavy
# destinations share buckets (more entries per (row, tile))?
set -eo pipefail
O=gpurun_out/degree; mkdir -p $O
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse"
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']; print(sys.argv[2], d['value'], 'fwd', e['fwd_ms'], 'bwd', e['bwd_ms'], e['bwd_mode'], 'loc', e.get('pull_locality'))" "$@"; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py $B "$@" > $O/$name.json 2> $O/$name.err; line $O/$name.json $name; }
run reddit_base
MAXK_BENCH_ORDER=degree run reddit_degree --reorder
run reddit_k32_base --k 32
MAXK_BENCH_ORDER=degree run reddit_k32_degree --reorder --k 32
run proteins_base --graph proteins
MAXK_BENCH_ORDER=degree run proteins_degree --graph proteins --reorder
echo degree probe done
