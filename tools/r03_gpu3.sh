#!/bin/bash
# r03: GPU suite + default bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03/bench.json 2> gpurun_out/r03/bench.err || { tail -20 gpurun_out/r03/bench.err; exit 1; }
cat gpurun_out/r03/bench.json
