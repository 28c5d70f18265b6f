#!/bin/bash
# Copy one gpu_round.sh run (gpurun_out/rNN) into profiles/rNN and regenerate the summaries.
set -e
R=${1:-r01}; KEY=${2:-reddit-D256-k16-pull-n1}
cd "$(dirname "$0")/.."
O=gpurun_out/$R; P=profiles/$R
mkdir -p $P/stats_bench
cp $O/stats/run_kernel_stats.csv $P/stats_bench/kernel_stats.csv
cp $O/stats_bench.json $P/stats_bench/bench.json
cp $O/bench.json $P/bench_default.json
cp $O/pmc_fetch/run_counter_collection.csv $P/pmc_fetch_size.csv
cp $O/pmc_write/run_counter_collection.csv $P/pmc_write_size.csv
[ -f $O/pytest_gpu.log ] && cp $O/pytest_gpu.log $P/pytest_gpu.log
# keys of other workloads (tools/pmc_products.sh) stay; this one is replaced
python tools/pmc_summary.py $P/pmc_fetch_size.csv $P/pmc_write_size.csv --traffic-out $P/traffic.json --key $KEY > $P/pmc_summary.txt
python tools/stats_summary.py $P/stats_bench/kernel_stats.csv $P/stats_bench/bench.json > $P/kernel_stats_summary.txt
cat $P/kernel_stats_summary.txt; tail -1 $P/pmc_summary.txt
