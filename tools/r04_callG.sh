#!/bin/bash
# r04 GPU call G: products k = 32 with and without the edge-selector stream, alternating on one
# box (the bench line and the 3-layer epoch), to settle the k = 32 default.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/es32
mkdir -p $O
for rep in 1 2 3; do for es in 0 1; do
  timeout -k 10 300 python bench.py --graph products --k 32 --edge-sel $es --steps 20 \
    --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/bench_es${es}_$rep.json 2> $O/bench_es${es}_$rep.err
  python -c "import json,sys; d=json.load(open('$O/bench_es${es}_$rep.json')); e=d['extra']; print('es=$es rep=$rep', e['fwd_ms'], e['bwd_ms'], d['ms_per_step'], d['value'])"
done; done
for rep in 1 2; do for es in 0 1; do
  MAXK_EDGE_SEL=$es timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products \
    > $O/epoch_es${es}_$rep.json 2> $O/epoch_es${es}_$rep.err
  python -c "import json; d=json.load(open('$O/epoch_es${es}_$rep.json')); print('epoch es=$es rep=$rep', d['maxk_epoch_ms'])"
done; done
