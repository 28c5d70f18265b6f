#!/bin/bash
# r03: Flickr (small graph, launch/latency bound): forward work-item size sweep + kernel split
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/flickr; mkdir -p $O
export TMPDIR=/tmp
for c in 0 64 128 256; do
  timeout -k 10 200 python -u bench.py --graph flickr --chunk $c --steps 50 --warmup 10 --no-cpu-baseline --no-cpu-spmm > $O/chunk$c.json 2> $O/chunk$c.err || { tail -3 $O/chunk$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/chunk$c.json')); x=d['extra']; print('chunk $c', d['value'], 'fwd', x['fwd_ms'], 'bwd', x['bwd_ms'], 'rocsparse best', x.get('rocsparse_spmm_ms_best'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --graph flickr --steps 50 --warmup 10 --no-cpu-baseline --no-cpu-spmm --no-rocsparse > /dev/null 2>&1 && python3 tools/stats_summary.py $O/prof/run_kernel_stats.csv | grep -E "maxk::|^op"
