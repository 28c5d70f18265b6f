#!/bin/bash
# 3-layer MaxK-SAGE epochs (BASELINE configs[2] shape) against the rocSPARSE model: products,
# Reddit, and the community products graph randomly labelled and in locality order.
set -eo pipefail
O=gpurun_out/epochs_r03; mkdir -p $O
for cfg in "products products" "reddit reddit" "products_comm_random products_comm" "products_comm_ordered products_comm --reorder"; do
  set -- $cfg; n=$1; shift
  timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py "$@" > $O/$n.json 2> $O/$n.err
  echo "$n $(cat $O/$n.json)"
done
# products with the edge-selector stream off (the k = 32 stream's effect on the epoch)
MAXK_EDGE_SEL=0 timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products > $O/products_es0.json 2> $O/products_es0.err
echo "products_es0 $(cat $O/products_es0.json)"
