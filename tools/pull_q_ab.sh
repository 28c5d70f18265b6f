#!/bin/bash
# A/B of the pull backward variants built by tools/tune.sh (lib/variants/*): pull time and
# agreement with the two-phase form per variant and k (tools/pull_ab.py), Reddit-sized graph.
# Usage: tools/pull_q_ab.sh "16 8 32 64" base q ...
set -o pipefail
cd "$(dirname "$0")/.."
KS=$1; shift
V=$PWD/spgemm-prunning_amd/lib/variants
for v in "$@"; do
  for k in $KS; do
    echo "## $v k=$k"
    MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 120 python -u tools/pull_ab.py --graph ${GRAPH:-reddit} --k $k --slices 0 --iters 20 || exit 1
  done
done
