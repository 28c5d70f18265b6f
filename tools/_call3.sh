# r05 session: record stride in 32-B multiples once 128-B records outgrow the Infinity Cache
# (products k = 16: 96-B records, 235 MB instead of 313 MB) -- parity on the variant, then the
# bench forward A/B on products k = 16 / 8 / 12
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s19
mkdir -p $O
MAXK_HIP_LIB=spgemm-prunning_amd/lib/variants/rs/libmaxk_hip.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_rs.log 2>&1 || { tail -40 $O/pytest_rs.log; exit 1; }
tail -1 $O/pytest_rs.log
R=2 timeout -k 10 900 bash tools/ab_bench.sh "base rs" "--graph products --k 16" "--graph products --k 12" > $O/ab.txt 2>&1
cat $O/ab.txt
