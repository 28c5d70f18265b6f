# r05 session: phase-1 item size at N = 8 (items floor at 256 tokens there): base (16 items per
# slot), q4 / q2 (4 / 2 per slot: ~480 / ~960 tokens); shard probe at N = 1 and 8
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s18
mkdir -p $O
for rep in 1 2; do
for v in base q4 q2; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  MAXK_HIP_LIB=$lib timeout -k 10 300 python tools/shard_probe.py --graph products --k 32 --worlds 1 8 > $O/shard_${v}_$rep.txt 2>&1
done
done
