#!/bin/bash
# Destination-grouped pull probe (Reddit, then proteins-sized at k = 16), plus kernel stats.
set -o pipefail
O=gpurun_out/pulld; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pulld_probe.py > $O/probe_reddit.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/probe_reddit.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 tools/pulld_probe.py --iters 5 > $O/probe_prof.txt 2>&1 || exit 1
python3 tools/stats_summary.py $O/stats/run_kernel_stats.csv | grep -E "pull|kernel " | head -8
