#!/bin/bash
# r04: forward at k <= 8 with 16 lanes per edge (kg16: 4 LDS copies per wave instead of 8, so
# LDS no longer caps the waves per CU) against the product build, with a byte-identical copy
# of the product build in another slot to expose run-order effects.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/fwd_occ
mkdir -p $O
R=3 timeout -k 10 800 bash tools/ab_bench.sh "kg16 basecopy base" "--graph products --k 8" \
  "--graph products --k 16" 2>&1 | tee $O/ab2.txt
