#!/bin/bash
# r04: forward batch depth (MAXK_FWD_U: 4 / 8 (product) / 16 wave steps of loads per batch)
# on the sparse products graph and the dense Reddit graph, order-controlled A/B.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/fwd_u
mkdir -p $O
R=2 timeout -k 10 900 bash tools/ab_bench.sh "base u16" "--k 8" "--k 32" "--k 64" \
  "--graph proteins" "--k 16" 2>&1 | tee $O/ab2.txt
