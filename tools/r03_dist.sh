#!/bin/bash
# r03: forward accumulate parity, the sharded path's GPU tests (pipelined gather mode), and the
# per-rank part times + step model at N = 8 (tools/shard_probe.py --pipelines).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/dist; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py tests/test_dist_cpu.py -x -q -m gpu -k "accumulate or dist" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u tools/shard_probe.py --graph products --k 32 --worlds 1 8 --pipelines 1 2 4 2>&1 | grep -v amdgpu.ids | tee $O/shard_products_k32.txt || exit 1
timeout -k 10 300 python -u tools/shard_probe.py --graph reddit --k 16 --worlds 1 8 --pipelines 1 2 4 2>&1 | grep -v amdgpu.ids | tee $O/shard_reddit_k16.txt || exit 1
