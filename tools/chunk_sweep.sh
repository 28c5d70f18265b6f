#!/bin/bash
# Work-item size (tokens per wave) sweep of the bench: forward / backward medians per chunk,
# two rounds.  CHUNKS: the chunk values (default 0 1024 2048 3072 4096); CHUNK_ARGS: extra bench
# arguments (default: the Reddit-sized default config); CHUNK_NAME: the summary's name.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${ROUND:-r04}/chunk
mkdir -p $O
for rep in 1 2; do for c in ${CHUNKS:-0 1024 2048 3072 4096}; do
  timeout -k 10 300 python bench.py ${CHUNK_ARGS:-} --chunk $c --steps 20 --no-cpu-baseline \
    --no-rocsparse --no-cpu-spmm > $O/${CHUNK_NAME:-reddit}_c${c}_$rep.json 2>/dev/null
  python -c "import json; d=json.load(open('$O/${CHUNK_NAME:-reddit}_c${c}_$rep.json')); e=d['extra']; print('chunk=$c rep=$rep', e['fwd_ms'], e['bwd_ms'], d['value'])"
done; done 2>&1 | tee $O/summary_${CHUNK_NAME:-reddit}.txt
