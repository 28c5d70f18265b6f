# r05 session: dense route with the selecting store -- parity, then Flickr A/B (base vs dr0 =
# no dense route) and a kernel trace of base
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s8
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_harness.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in base dr0; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  MAXK_HIP_LIB=$lib timeout -k 10 200 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 32 64 > $O/kt_${v}_$rep.txt 2>&1
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 32 64 > $O/prof.log 2>&1
