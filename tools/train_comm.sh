#!/bin/bash
# 3-layer MaxK-SAGE epoch (BASELINE configs[2] shape) on the planted-community products graph,
# randomly labelled (backward auto -> csc) and in locality order (auto -> hybrid).
set -eo pipefail
O=gpurun_out/train_comm; mkdir -p $O
timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products_comm > $O/random.json 2> $O/random.err
cat $O/random.json
timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products_comm --reorder > $O/ordered.json 2> $O/ordered.err
cat $O/ordered.json
MAXK_HYBRID_STREAMS=0 timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products_comm --reorder --no-library > $O/ordered_s0.json 2> $O/ordered_s0.err
cat $O/ordered_s0.json
