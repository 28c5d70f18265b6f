#!/bin/bash
# Hybrid backward on the planted-community products graphs: per-kernel times (rocprofv3
# --stats), the tile-density threshold, a weaker-locality graph (p_in 0.5) and what "auto" picks.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/hybrid; mkdir -p $O
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse"
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']; print(sys.argv[2], d['value'], 'fwd', e['fwd_ms'], 'bwd', e['bwd_ms'], e['bwd_mode'], 'frac', d['roofline']['frac'], 'loc', e.get('pull_locality'))" "$@"; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py $B "$@" > $O/$name.json 2> $O/$name.err; line $O/$name.json $name; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $B --graph products_comm --reorder --bwd-mode hybrid --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/hybrid/prof/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"  {n[:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.4f} ms")
PY
for d in 0.25 1 2; do MAXK_HYBRID_DENSITY=$d run ordered_d$d --graph products_comm --reorder --bwd-mode hybrid; done
run p50_auto --graph products_comm_p50 --reorder
run p50_csc --graph products_comm_p50 --reorder --bwd-mode csc
run p50_hybrid --graph products_comm_p50 --reorder --bwd-mode hybrid
run comm_random_auto --graph products_comm
echo hybrid probe done
