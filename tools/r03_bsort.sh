set -eo pipefail
mkdir -p gpurun_out/bsort
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bsort or fuzz or all_k or high_degree or empty or zero_rows or overwritten or past_D or rectangular or capture_default" > gpurun_out/bsort/pytest.log 2>&1
tail -3 gpurun_out/bsort/pytest.log
timeout -k 10 400 python -u tools/bsort_probe.py > gpurun_out/bsort/probe.txt 2>&1
cat gpurun_out/bsort/probe.txt
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bsort/stats -o run --output-format csv -- python3 tools/bsort_probe.py --k 8 --iters 5 > gpurun_out/bsort/probe_prof.txt 2>&1
echo done
