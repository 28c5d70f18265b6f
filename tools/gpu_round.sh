#!/bin/bash
# One GPU-box session: parity tests, smoke, default bench, kernel-trace stats and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE -- separate runs, no trace domains).  Every GPU step
# has its own time limit; the first failure ends the script.
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh r01'
set -eo pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse"
STEPS=${STEPS:-tests,smoke,bench,stats,pmc}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -2 $O/smoke.log
fi
if has bench; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
  cat $O/bench.json
fi
if has stats; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv \
    -- python3 $BENCH > $O/stats_bench.json 2> $O/stats_bench.err
fi
if has pmc; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv \
    -- python3 $BENCH > $O/pmc_fetch.json 2> $O/pmc_fetch.err
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv \
    -- python3 $BENCH > $O/pmc_write.json 2> $O/pmc_write.err
fi
echo done
