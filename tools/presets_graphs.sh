set -eo pipefail
O=gpurun_out/presets; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name $(python -c "import json,sys; d=json.load(open('$O/$name.json')); e=d['extra']; print(d['value'], e['fwd_ms'], e['bwd_ms'], e['bwd_mode'], d['roofline']['frac'], e.get('rocsparse_spmm_ms'), e.get('rocsparse_spmm_ms_best'))")"; }
for g in products proteins flickr; do run $g --graph $g --no-cpu-baseline --no-cpu-spmm; done
