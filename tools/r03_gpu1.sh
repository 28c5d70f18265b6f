#!/bin/bash
# r03 first GPU pass: GPU tests, top-k every-row probe (product lib and the four-row k<=64
# variant), default bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/topk_rows_probe.py product 16 32 48 64 > gpurun_out/r03/topk_rows_product.txt 2>&1 || exit 1
cat gpurun_out/r03/topk_rows_product.txt | grep -v amdgpu.ids
MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/rows4k64/libmaxk_hip.so timeout -k 10 300 python -u tools/topk_rows_probe.py rows4k64 16 32 48 64 > gpurun_out/r03/topk_rows_rows4k64.txt 2>&1 || exit 1
cat gpurun_out/r03/topk_rows_rows4k64.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py > gpurun_out/r03/bench.json 2> gpurun_out/r03/bench.err || { tail -20 gpurun_out/r03/bench.err; exit 1; }
cat gpurun_out/r03/bench.json
