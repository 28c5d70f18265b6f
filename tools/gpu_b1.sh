# scratch GPU session: tests, then bucket vs csc backward across graphs and k
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/b1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # graph k mode
  timeout -k 10 300 python bench.py --graph $1 --k $2 --steps 8 --warmup 3 --no-cpu-baseline --no-rocsparse --no-cpu-spmm --bwd-mode $3 > $O/bench_$1_$2_$3.json 2> $O/bench_$1_$2_$3.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_$1_$2_$3.json'));e=d['extra'];print('$1 k=$2 $3', e['bwd_mode'], d['value'], e['fwd_ms'], e['bwd_ms'], e['adjoint_rel_err'])"
}
for k in 16 8 4 12; do for m in bucket csc; do run reddit $k $m; done; done
for m in bucket csc; do run proteins 16 $m; run products 16 $m; done
run reddit 16 auto
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/stats_bench.json 2> $O/stats_bench.err
python tools/stats_summary.py $O/stats/run_kernel_stats.csv $O/stats_bench.json | head -20
