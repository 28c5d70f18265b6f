#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, separate passes) of the products-sized backward:
# csc on the randomly labelled graph and the hybrid on the community graph in locality order.
# Merged into profiles/$R/traffic.json by tools/pmc_summary.py afterwards (on the CPU side).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_products; mkdir -p $O
B="--steps 5 --warmup 2 --no-cpu-baseline --no-cpu-spmm --no-rocsparse"
for cfg in "products --graph products" "comm_ordered --graph products_comm --reorder"; do
  set -- $cfg; n=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $O/${n}_$c -o run --output-format csv -- python3 bench.py $B "$@" > $O/${n}_$c.json 2> $O/${n}_$c.err
  done
  echo "$n done"
done
