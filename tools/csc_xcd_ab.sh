#!/bin/bash
# csc phase 2 work order on random and community-ordered graphs: the default build (XCD runs of
# MAXK_XCD_SUM_RUN = 64 blocks per window) against variants built by tools/tune.sh
# (run16: -DMAXK_XCD_SUM_RUN=16; run0: one contiguous eighth per XCD, the earlier order;
# noxcd: -DMAXK_XCD_SUM=0, round-robin).  tools/csc_xcd_ab.sh VARIANT...
set -eo pipefail
O=gpurun_out/csc_xcd; mkdir -p $O
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse"
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']; print(sys.argv[2], 'fwd', e['fwd_ms'], 'bwd', e['bwd_ms'], e['bwd_mode'])" "$@"; }
for v in default "$@"; do
  if [ $v = default ]; then unset MAXK_HIP_LIB; else export MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; fi
  for cfg in "reddit_csc --bwd-mode csc" "products_csc --graph products" "comm_ordered_hybrid --graph products_comm --reorder" "proteins_csc --graph proteins --bwd-mode csc"; do
    set -- $cfg; n=$1; shift
    timeout -k 10 300 python3 bench.py $B "$@" > $O/${v}_$n.json 2> $O/${v}_$n.err
    line $O/${v}_$n.json "$v $n"
  done
  MAXK_BWD_MODE=csc timeout -k 10 300 python3 tools/shard_probe.py --graph products_comm --worlds 8 > $O/${v}_shard_random.txt 2>&1
  echo "$v shard random csc: $(tail -1 $O/${v}_shard_random.txt)"
  MAXK_BWD_MODE=csc timeout -k 10 300 python3 tools/shard_probe.py --graph products_comm --reorder --worlds 8 > $O/${v}_shard_ordered.txt 2>&1
  echo "$v shard ordered csc: $(tail -1 $O/${v}_shard_ordered.txt)"
  timeout -k 10 300 python3 tools/shard_probe.py --graph products_comm --reorder --worlds 8 > $O/${v}_shard_ordered_auto.txt 2>&1
  echo "$v shard ordered auto: $(tail -1 $O/${v}_shard_ordered_auto.txt)"
done
echo csc xcd done
