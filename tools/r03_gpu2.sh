#!/bin/bash
# r03: top-k tail-overflow fix check: fixture, full-input probe (product KMAX=48, variant 64)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
timeout -k 10 200 python -u tools/make_topk_tail_fixture.py || exit 1
cp tests/golden/topk/topk_tail_overflow.npz gpurun_out/r03/ || exit 1
timeout -k 10 300 python -u tools/topk_rows_probe.py product 16 32 40 48 64 > gpurun_out/r03/topk_rows_product_fixed.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03/topk_rows_product_fixed.txt
MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/rows4k64/libmaxk_hip.so timeout -k 10 300 python -u tools/topk_rows_probe.py rows4k64 48 56 64 > gpurun_out/r03/topk_rows_rows4k64_fixed.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03/topk_rows_rows4k64_fixed.txt
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -k gaussian > gpurun_out/r03/pytest_gauss.log 2>&1; rc=$?; tail -3 gpurun_out/r03/pytest_gauss.log; exit $rc
