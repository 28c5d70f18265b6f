# r05 session: GPU suite, then A/B of the small-graph forward (s0 = r04 batches, r0 = streaming
# rows over packed records, base = pack-free streaming) and the direct pull (pd0 = three
# launches, pw1 / pw4 = MAXK_PULL_DIRECT_WGS) -- variants built by tools/tune.sh
set -eo pipefail
O=gpurun_out/r05/s3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_fuzz_gpu.py tests/test_parity_gpu.py tests/test_hybrid_gpu.py tests/test_layers_gpu.py tests/test_harness.py tests/test_fullsize_gpu.py tests/test_dist_gpu.py tests/test_dist_cpu.py -m gpu -x -q --timeout 300 --timeout-method thread --durations=30 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in base s0 r0 pd0 pw1 pw4; do
  lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  MAXK_HIP_LIB=$lib timeout -k 10 200 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 32 64 > $O/kt_${v}_$rep.txt 2>&1
done
done
R=2 timeout -k 10 900 bash tools/ab_bench.sh "base s0 r0 rbig s128" "--graph flickr" "--graph products --k 32" "--graph products --k 64" "--graph products --k 16 --edge-sel 0" > $O/ab.txt 2>&1
