# r05 session: LDS-free record pack (cbsr_pack_regs_kernel) -- parity, then kernel traces of the
# Flickr kernel test (k = 8 / 16) and bench A/B on products k = 32 / 8: base vs pr0 (LDS pack)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s21
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in base pr0; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  MAXK_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 > $O/kt_$v.txt 2>&1
done
R=2 timeout -k 10 900 bash tools/ab_bench.sh "base pr0" "--graph products --k 32" "--graph products --k 8" "--graph flickr" > $O/ab.txt 2>&1
cat $O/ab.txt
