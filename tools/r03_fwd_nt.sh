#!/bin/bash
# Forward output stores plain vs non-temporal (variant library): forward times per graph / k.
set -eo pipefail
O=gpurun_out/fwdnt; mkdir -p $O
for lib in default fwdnt; do
  L=spgemm-prunning_amd/lib/libmaxk_hip.so; [ $lib = fwdnt ] && L=spgemm-prunning_amd/lib/variants/fwdnt/libmaxk_hip.so
  MAXK_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/edge_sel_probe.py --graph products --k 8 16 32 > $O/products_$lib.txt 2>&1
  MAXK_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/edge_sel_probe.py --graph reddit --k 16 > $O/reddit_$lib.txt 2>&1
  echo "== $lib"; cat $O/products_$lib.txt $O/reddit_$lib.txt | grep -o "k=[0-9]*:.*forward [0-9.]* ms, forward emitting the stream [0-9.]* ms" | sed 's/csc.*forward \([0-9.]*\) ms, forward emitting/fwd \1, emit/'
done
