#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE (separate rocprofv3 runs, no trace domains) of the bench on the
# non-default configurations; merged into profiles/$R/traffic.json on the CPU side with
#   python tools/pmc_summary.py gpurun_out/$R/pmc_cfg/<name>_FETCH_SIZE/run_counter_collection.csv \
#       gpurun_out/$R/pmc_cfg/<name>_WRITE_SIZE/run_counter_collection.csv \
#       --traffic-out profiles/$R/traffic.json --key <bench traffic_key>
#   gpurun -- 'bash tools/r03_pmc_configs.sh r03'
set -o pipefail
R=${1:-r03}
cd "$(dirname "$0")/.."
O=gpurun_out/$R/pmc_cfg; mkdir -p $O
export TMPDIR=/tmp
B="--steps 5 --warmup 2 --no-cpu-baseline --no-cpu-spmm --no-rocsparse"
CFGS=${CFGS:-"products_k8:--graph products --k 8 products_k16:--graph products --k 16 products_k32:--graph products --k 32 reddit_k8:--k 8"}
IFS=' ' read -r -a items <<< "$CFGS"
name=""; args=""
flush() {
  [ -z "$name" ] && return 0
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $O/${name}_$c -o run --output-format csv -- \
      python3 bench.py $B $args > $O/${name}_$c.json 2> $O/${name}_$c.err \
      || { echo "$name $c failed"; tail -3 $O/${name}_$c.err; return 1; }
  done
  echo "$name done: $(python3 -c "import json; print(json.load(open('$O/${name}_FETCH_SIZE.json'))['roofline']['traffic_key'])")"
}
for w in "${items[@]}"; do
  if [[ "$w" == *:* ]]; then
    flush || exit 1
    name=${w%%:*}; args=${w#*:}
  else
    args="$args $w"
  fi
done
flush || exit 1
