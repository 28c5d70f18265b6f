#!/bin/bash
# Build libmaxk_hip variants for tuning: tools/tune.sh NAME "FLAGS" ...
# Each goes to spgemm-prunning_amd/lib/variants/NAME/libmaxk_hip.so; select with MAXK_HIP_LIB.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  out=$ROOT/spgemm-prunning_amd/lib/variants/$name
  mkdir -p $out /tmp/maxk_build_$name
  make -s -C $ROOT/spgemm-prunning_amd OBJDIR=/tmp/maxk_build_$name OUTDIR=$out EXTRA_HIPFLAGS="$flags" -j8
done
