# r05 session: the dense backward's selected-column form (pick_rows_kernel, k < D / 2) --
# parity, then kernel tests with --bwd-mode dense against auto (pull) on Flickr and Reddit
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s12
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_harness.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for m in auto dense; do
  timeout -k 10 200 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 32 --bwd-mode $m > $O/kt_flickr_${m}_$rep.txt 2>&1
done
done
for m in auto dense; do
  timeout -k 10 300 python spgemm-prunning_amd/maxk_kernel_test.py reddit --k 8 16 --bwd-mode $m > $O/kt_reddit_${m}.txt 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 --bwd-mode dense > $O/prof.log 2>&1
