#!/bin/bash
# 3-layer MaxK-SAGE epochs (BASELINE configs[2] shape) against the rocSPARSE model: products,
# Reddit, and the community products graph randomly labelled and in locality order.
set -eo pipefail
O=gpurun_out/epochs; mkdir -p $O
for cfg in "products products" "reddit reddit" "products_comm_random products_comm" "products_comm_ordered products_comm --reorder"; do
  set -- $cfg; n=$1; shift
  timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py "$@" > $O/$n.json 2> $O/$n.err
  echo "$n $(cat $O/$n.json)"
done
