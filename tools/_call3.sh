# r05 session: grouped csc phase 2 (U = 4, on below an average in-degree of 16) -- parity of the
# csc paths, then phase-2 items of 256 (base), ~512 (p8) and ~1024 (p4) tokens at N = 8, and g0
# (grouping off); shard probe at N = 1 and 8
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s17
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for v in base p8 p4 g0; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  MAXK_HIP_LIB=$lib timeout -k 10 300 python tools/shard_probe.py --graph products --k 32 --worlds 1 8 > $O/shard_${v}_$rep.txt 2>&1
done
done
