# r05 session: dense route with whole rows (hub rows only split), fixup launches kept
# -- parity, Flickr kernel test, kernel trace
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s11
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_harness.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 32 64 > $O/kt_base_$rep.txt 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 32 64 > $O/prof.log 2>&1
