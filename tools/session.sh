#!/bin/bash
# The one driver for GPU-box sessions (replaces r01-r03's one-off scripts, which are in git
# history: gpu_round.sh, collect_round.sh, presets_r0*.sh, epochs_r0*.sh, kt_r02.sh,
# r03_*.sh).  Every GPU step runs under its own time limit and the first failure ends the
# script (set -e); outputs go to gpurun_out/<round>/<step>/.  Run on the box as
#   gpurun --timeout 1200 -- 'bash tools/session.sh <round> <step> [<step> ...]'
# and copy what is judged into profiles/<round>/ with `bash tools/session.sh <round> collect`
# here.  Steps:
#   tests     pytest -m gpu (the whole GPU suite)
#   smoke     __graft_entry__.smoke()
#   bench     the default bench line (BENCH contract), with CPU baselines
#   stats     rocprofv3 --kernel-trace --stats of a short default bench
#   pmc       FETCH_SIZE and WRITE_SIZE of the same short bench, one rocprofv3 --pmc pass each
#   presets   every preset with its denominators (rocSPARSE every algorithm; CPU baselines
#             with PRESET_CPU=1); presets_small: the Flickr-shaped ones alone; presets_products:
#             ogbn-products-sized k = 32 and 64 alone
#   pmccfg    PMC passes of the non-default configurations in $CFGS
#             ("name:--bench --args name2:..."), keyed by each run's traffic_key
#   pmcset    counter sets $SETS ("C1 C2;C3 C4", one pass per set) over the configurations in
#             $CFGS; per-kernel averages in gpurun_out/<round>/pmc_set/<name>.txt
#   statscfg  rocprofv3 --kernel-trace --stats of the configurations in $CFGS (as pmccfg);
#             summaries in gpurun_out/<round>/stats_cfg/<name>.txt
#   topkab    top-k GPU tests, then tools/topk_ab.py alternating the product library and the
#             variants in $VARS (lib/variants/<name>, tools/tune.sh), two repeats
#   ab        tools/ab_bench.sh over the variants in $VARS and the bench argument strings in
#             $ABCFGS (separated by ';'); $REPS repeats (2)
#   window    the products forward with its columns folded into cache-sized windows
#             (tools/fwd_slice_probe.py, k = 8 and 16)
#   rehearse  N-rank rehearsals of the multi-GPU bench on the one GPU (gloo-staged
#             collectives): Reddit k = 16 at N = 8 and 4, products k = 32 at N = 8; each run
#             checks itself against the unsharded result (extra.dist_check_*)
#   rehearsek8  the same for products k = 8 at N = 8 (bsort backward, edge-selector stream)
#   esab      products k = 32 with and without the edge-selector stream, alternating on one
#             box: the bench line (3 repeats) and the 3-layer epoch (2 repeats)
#   kt        the reference's kernel test (maxk_kernel_test.py) on every config graph, k = 8..64
#   epochs    3-layer MaxK-SAGE epochs against the rocSPARSE model
#   fetchcal  tools/fetch_probe (known 64/80/128/160/256-B record gathers and a streaming read,
#             24 MiB and 2 GiB tables) under a FETCH_SIZE pass and a fabric-request-size pass
#             (TCC_EA0_RDREQ_sum / _32B / _128B), summarised by tools/fetch_probe_summary.py
#             (r06: the FETCH_SIZE correction per request size)
#   contention  tools/shard_probe.py at N = 8 (products k = 32, the pipelined record exchange)
#             with each part's kernels also timed beside a paced copy standing in for the
#             overlapping RCCL collective (tools/paced_copy.hip, 32 and 64 channels): the
#             contention-inclusive N = 8 step model (r06)
#   phases    box identity and clocks (rocm-smi), then rocprofv3 --kernel-trace --stats of the
#             ogbn-products k = 32 bench (csc phase 1 / phase 2 per-kernel times) and of the
#             default Reddit bench: run on several boxes to name the phase behind the products
#             backward's box-to-box spread (r06)
#   spread    tools/clock_probe.py (products k = 32 forward + csc backward in a 12-s loop) under
#             rocprofv3 --kernel-trace --stats, with rocm-smi clocks / power / temperature
#             sampled from the shell every second beside it: per-phase times and the clocks
#             they ran at, on whichever box this call got (r06)
#   ktg       the compiled harness on the Flickr- and Reddit-sized graphs, plain and with
#             --graph-replay (each op captured once into a hipGraph and timed as one launch),
#             plus rocprofv3 --kernel-trace --stats of the plain Flickr run (the ops' kernel time
#             beside their wall time: the launch-gap share; r06)
#   collect   (here, not on the box) copy gpurun_out/<round> into profiles/<round> and write
#             the summaries (kernel stats, PMC traffic.json, presets and kernel-test tables)
set -eo pipefail
R=${1:?round, e.g. r04}; shift
cd "$(dirname "$0")/.."
O=gpurun_out/$R
P=profiles/$R
export TMPDIR=/tmp
SHORT="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-rocsparse --no-cpu-spmm"

step_tests() {
  mkdir -p $O
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --durations=25 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -2 $O/pytest_gpu.log
}
step_smoke() {
  mkdir -p $O
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -2 $O/smoke.log
}
step_bench() {
  mkdir -p $O
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
  cut -c1-400 $O/bench.json
}
step_stats() {
  mkdir -p $O
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv \
    -- python3 $SHORT > $O/stats_bench.json 2> $O/stats_bench.err
}
# PMC passes: FETCH_SIZE, WRITE_SIZE, and the texture path's tag accesses with the XCD clocks
# (roofline.binding, r05); one rocprofv3 --pmc run each, named by the first counter
PASSES="FETCH_SIZE WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum:GRBM_GUI_ACTIVE"
step_pmc() {
  mkdir -p $O
  local c
  for c in $PASSES; do
    timeout -k 10 300 rocprofv3 --pmc ${c//:/ } -d $O/pmc_${c%%:*} -o run --output-format csv \
      -- python3 $SHORT > $O/pmc_${c%%:*}.json 2> $O/pmc_${c%%:*}.err
  done
}
preset() {  # preset <name> <bench args...>
  local name=$1; shift
  local cpu="--no-cpu-baseline --no-cpu-spmm"
  [ "${PRESET_CPU:-0}" = 1 ] && cpu="--cpu-seconds 6"
  timeout -k 10 400 python bench.py $cpu "$@" > $O/presets/$name.json 2> $O/presets/$name.err
  python - "$O/presets/$name.json" "$name" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1])); e = d["extra"]
print(sys.argv[2], d["value"], e["fwd_ms"], e["bwd_ms"], e["bwd_mode"], e.get("edge_sel_stream"),
      d["roofline"]["frac"], e.get("rocsparse_spmm_ms"), e.get("rocsparse_spmm_ms_best"))
EOF
}
step_presets() {
  mkdir -p $O/presets
  preset reddit
  for k in 8 32 64; do preset reddit_k$k --k $k; done
  for m in csc atomic; do preset reddit_$m --bwd-mode $m --no-rocsparse; done
  for k in 8 16 32 64; do preset products_k$k --graph products --k $k; done
  preset products_k4 --graph products --k 4 --no-rocsparse
  preset proteins --graph proteins
  step_presets_small
  preset products_comm_ordered --graph products_comm --reorder
}
# the ogbn-products-sized presets whose csc phase 2 reads whole-line rows (k % 32 == 0)
step_presets_products() {
  mkdir -p $O/presets
  for k in 32 64; do preset products_k$k --graph products --k $k; done
}
# the Flickr-shaped graph (configs[0], D = 64) at every k: k >= 32 takes the dense route
step_presets_small() {
  mkdir -p $O/presets
  preset flickr --graph flickr
  for k in 8 32 64; do preset flickr_k$k --graph flickr --k $k; done
}
cfg_loop() {  # cfg_loop <function>: $CFGS "name:--args ..." -> function name "args"
  local fn=$1 name="" args="" w
  for w in ${CFGS:?CFGS=\"name:--args ...\"}; do
    if [[ "$w" == *:* ]]; then
      [ -n "$name" ] && $fn "$name" "$args"
      name=${w%%:*}; args=${w#*:}
    else
      args="$args $w"
    fi
  done
  [ -n "$name" ] && $fn "$name" "$args"
  return 0
}
stats_one() {
  local d=$O/stats_cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/$1 -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-spmm --no-rocsparse \
    $2 > $d/$1.json 2> $d/$1.err
  python tools/stats_summary.py $d/$1/run_kernel_stats.csv $d/$1.json > $d/$1.txt
  echo "$1: $(tail -2 $d/$1.txt | tr '\n' ' ')"
}
pmc_one() {
  local c
  for c in $PASSES; do
    timeout -k 10 300 rocprofv3 --pmc ${c//:/ } -d $O/pmc_cfg/${1}_${c%%:*} -o run \
      --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      --no-cpu-spmm --no-rocsparse $2 > $O/pmc_cfg/${1}_${c%%:*}.json \
      2> $O/pmc_cfg/${1}_${c%%:*}.err
  done
  echo "$1 done"
}
step_pmccfg() {
  mkdir -p $O/pmc_cfg
  cfg_loop pmc_one
}
# pmcset: per configuration of $CFGS, one rocprofv3 --pmc pass per counter set of $SETS
# (sets separated by ';', each within one pass's block limits), then the per-kernel averages
# of every counter: gpurun_out/<round>/pmc_set/<name>.txt
set_one() {
  local d=$O/pmc_set/$1 i=0 s
  mkdir -p $d
  IFS=';' read -ra sets <<< "${SETS:?SETS=\"C1 C2;C3 ...\"}"
  for s in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $s -d $d/p$i -o run --output-format csv \
      -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cpu-spmm --no-rocsparse \
      $2 > $d/p$i.json 2> $d/p$i.err
  done
  python3 tools/pmc_kernels.py $d > $O/pmc_set/$1.txt
  echo "$1 done"
}
step_pmcset() {
  mkdir -p $O/pmc_set
  cfg_loop set_one
}
step_fetchcal() {
  mkdir -p $O/fetch
  timeout -k 10 120 tools/fetch_probe > $O/fetch/probe.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch/p1 -o run --output-format csv \
    -- tools/fetch_probe > $O/fetch/p1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
    TCC_EA0_RDREQ_128B_sum -d $O/fetch/p2 -o run --output-format csv \
    -- tools/fetch_probe > $O/fetch/p2.log 2>&1
  python3 tools/fetch_probe_summary.py $O/fetch/probe.log $(find $O/fetch -name '*counter_collection.csv') \
    > $O/fetch/summary.txt
  cat $O/fetch/summary.txt
}
step_contention() {
  mkdir -p $O/scaling
  local ch
  for ch in 32 64; do
    timeout -k 10 400 python tools/shard_probe.py --graph products --k 32 --worlds 1 8 \
      --pipelines 2 --records --contention --channels $ch \
      > $O/scaling/contention_products_k32_ch$ch.txt 2>&1
    tail -12 $O/scaling/contention_products_k32_ch$ch.txt
  done
}
step_phases() {
  local d=$O/phases/$(date +%H%M%S)
  mkdir -p $d
  { hostname; rocm-smi --showproductname --showclocks --showtemp --showpower 2>&1 || true; } \
    > $d/smi_before.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/products_k32 -o run \
    --output-format csv -- python3 bench.py --graph products --k 32 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-cpu-spmm --no-rocsparse > $d/products_k32.json 2> $d/products_k32.err
  python tools/stats_summary.py $d/products_k32/run_kernel_stats.csv $d/products_k32.json \
    > $d/products_k32.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/reddit -o run \
    --output-format csv -- python3 bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --no-cpu-spmm --no-rocsparse > $d/reddit.json 2> $d/reddit.err
  python tools/stats_summary.py $d/reddit/run_kernel_stats.csv $d/reddit.json > $d/reddit.txt
  { rocm-smi --showclocks --showtemp --showpower 2>&1 || true; } > $d/smi_after.txt
  head -12 $d/products_k32.txt
  grep -i 'sclk\|mclk\|fclk' $d/smi_before.txt | head -6 || true
}
step_spread() {
  local d=$O/spread/$(date +%H%M%S)
  mkdir -p $d
  { rocm-smi --showproductname --showuniqueid 2>&1 || true; } > $d/box.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv \
    -- python3 tools/clock_probe.py --seconds 12 > $d/probe.txt 2> $d/probe.err &
  local pid=$! i
  for i in $(seq 60); do
    kill -0 $pid 2>/dev/null || break
    { date +%s.%N; rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E 'sclk|mclk|fclk|Power|junction|memory' || true; } >> $d/clocks.txt
    sleep 1
  done
  wait $pid
  python tools/stats_summary.py $d/prof/run_kernel_stats.csv > $d/stats.txt
  head -6 $d/stats.txt
  grep -i guid\|unique $d/box.txt | head -2 || true
  tail -3 $d/probe.txt
}
step_ktg() {
  local d=$O/kernel_test_graph g D
  mkdir -p $d
  for g in flickr reddit; do
    D=256; [ $g = flickr ] && D=64
    timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'spgemm-prunning_amd')
import torch, maxk_graph
rp, col = maxk_graph.synthetic_graph('$g', device=torch.device('cuda'))
maxk_graph.save_graph(rp, col, '/tmp/maxk_graphs', '$g')"
    timeout -k 10 300 spgemm-prunning_amd/bin/maxk_kernel_test $g --dir /tmp/maxk_graphs \
      --dim $D --k 8,16,32,64 --runs 20 > $d/$g.txt 2> $d/$g.err
    timeout -k 10 300 spgemm-prunning_amd/bin/maxk_kernel_test $g --dir /tmp/maxk_graphs \
      --dim $D --k 8,16,32,64 --runs 20 --graph-replay > $d/${g}_replay.txt 2> $d/${g}_replay.err
    if [ $g = flickr ]; then
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/prof_flickr -o run \
        --output-format csv -- spgemm-prunning_amd/bin/maxk_kernel_test $g \
        --dir /tmp/maxk_graphs --dim $D --k 16 --runs 20 > $d/flickr_prof.txt 2>&1
    fi
    rm -f /tmp/maxk_graphs/$g.indptr /tmp/maxk_graphs/$g.indices
  done
  paste $d/flickr.txt $d/flickr_replay.txt | head -20
}
step_statscfg() {
  mkdir -p $O/stats_cfg
  cfg_loop stats_one
}
step_topkab() {
  mkdir -p $O/topk
  timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k topk -x -q --timeout 120 \
    --timeout-method thread > $O/topk/pytest_topk.log 2>&1
  tail -1 $O/topk/pytest_topk.log
  local rep v lib rows
  for rep in 1 2; do for v in base ${VARS:?VARS=\"variant ...\"}; do
    lib=spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so
    [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
    for rows in 232965 2449029; do
      echo "== $v rows=$rows rep=$rep"
      MAXK_HIP_LIB=$lib timeout -k 10 120 python tools/topk_ab.py --rows $rows
    done
  done; done > $O/topk/topk_ab.txt 2>&1
}
step_ab() {
  mkdir -p $O/ab
  local cfgs=()
  IFS=';' read -ra cfgs <<< "${ABCFGS:?ABCFGS=\"--k 16;--graph products --k 8\"}"
  R=${REPS:-2} timeout -k 10 900 bash tools/ab_bench.sh "base ${VARS:?}" "${cfgs[@]}" \
    > $O/ab/ab.txt 2>&1
  cat $O/ab/ab.txt
}
step_window() {
  mkdir -p $O/probe
  local k
  for k in 8 16; do
    timeout -k 10 300 python tools/fwd_slice_probe.py --graph products --k $k \
      > $O/probe/fwd_window_products_k$k.txt 2>&1
  done
}
rehearse_one() {  # rehearse_one <name> <ranks> <bench args...>
  local n=$1 w=$2; shift 2
  MAXK_DIST_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29500 + w)) bench.py \
    --gpus $w --steps 5 --warmup 2 "$@" > $O/rehearsal/$n.json 2> $O/rehearsal/$n.err
  python - $O/rehearsal/$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[2], "fwd err", e["dist_check_fwd_max_rel_err"], "bwd err",
      e["dist_check_bwd_max_rel_err"], "mode", e["dist_mode"], "parts", e["dist_pipeline"],
      "bwd", e["bwd_mode"], "stream", e["edge_sel_stream"], "ms/step", d["ms_per_step"])
PY
}
step_rehearse() {
  mkdir -p $O/rehearsal
  rehearse_one n8_reddit 8
  rehearse_one n4_reddit 4
  rehearse_one n8_products_k32 8 --graph products
}
step_rehearsek8() {  # products k = 8 at N = 8: the sharded bsort backward and selector stream
  mkdir -p $O/rehearsal
  rehearse_one n8_products_k8 8 --graph products --k 8
}
step_esab() {
  mkdir -p $O/es32
  local rep es
  for rep in 1 2 3; do for es in 0 1; do
    timeout -k 10 300 python bench.py --graph products --k 32 --edge-sel $es --steps 20 \
      --no-cpu-baseline --no-rocsparse --no-cpu-spmm > $O/es32/bench_es${es}_$rep.json \
      2> $O/es32/bench_es${es}_$rep.err
  done; done
  for rep in 1 2; do for es in 0 1; do
    MAXK_EDGE_SEL=$es timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py \
      products > $O/es32/epoch_es${es}_$rep.json 2> $O/es32/epoch_es${es}_$rep.err
  done; done
}
step_kt() {
  mkdir -p $O/kernel_test
  for g in reddit products proteins; do
    timeout -k 10 400 python spgemm-prunning_amd/maxk_kernel_test.py $g --k 8 16 32 64 --json \
      > $O/kernel_test/$g.txt 2> $O/kernel_test/$g.err
  done
  timeout -k 10 300 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 \
    --k 8 16 32 64 --json > $O/kernel_test/flickr.txt 2> $O/kernel_test/flickr.err
  python tools/kt_table.py $O/kernel_test
}
# the compiled C-ABI consumer (bin/maxk_kernel_test: kernels/main.cu's recipe and wall-clock
# timing, no Python on the timed path) on the synthetic graphs written as .indptr/.indices to
# the box's /tmp (r05: the reference's kernel numbers come from that C++ program)
step_ktc() {
  mkdir -p $O/kernel_test_cpp
  local g D
  for g in flickr reddit products proteins; do
    D=256; [ $g = flickr ] && D=64
    timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'spgemm-prunning_amd')
import torch, maxk_graph
rp, col = maxk_graph.synthetic_graph('$g', device=torch.device('cuda'))
maxk_graph.save_graph(rp, col, '/tmp/maxk_graphs', '$g')"
    timeout -k 10 300 spgemm-prunning_amd/bin/maxk_kernel_test $g --dir /tmp/maxk_graphs \
      --dim $D --k 8,16,32,64 --runs 20 > $O/kernel_test_cpp/$g.txt 2> $O/kernel_test_cpp/$g.err
    rm -f /tmp/maxk_graphs/$g.indptr /tmp/maxk_graphs/$g.indices
  done
  cat $O/kernel_test_cpp/*.txt
}
step_epochs() {
  mkdir -p $O/train
  for cfg in "products products" "reddit reddit" "products_comm_ordered products_comm --reorder"; do
    set -- $cfg; local n=$1; shift
    timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py "$@" > $O/train/$n.json \
      2> $O/train/$n.err
    echo "$n $(cat $O/train/$n.json)"
  done
}
step_collect() {
  mkdir -p $P
  if [ -f $O/stats/run_kernel_stats.csv ]; then
    mkdir -p $P/stats_bench
    cp $O/stats/run_kernel_stats.csv $P/stats_bench/kernel_stats.csv
    cp $O/stats_bench.json $P/stats_bench/bench.json
    python tools/stats_summary.py $P/stats_bench/kernel_stats.csv $P/stats_bench/bench.json \
      > $P/kernel_stats_summary.txt
  fi
  [ -f $O/bench.json ] && cp $O/bench.json $P/bench_default.json
  for f in pytest_gpu.log smoke.log; do [ -f $O/$f ] && cp $O/$f $P/$f; done
  if [ -f $O/pmc_FETCH_SIZE/run_counter_collection.csv ]; then
    cp $O/pmc_FETCH_SIZE/run_counter_collection.csv $P/pmc_fetch_size.csv
    cp $O/pmc_WRITE_SIZE/run_counter_collection.csv $P/pmc_write_size.csv
    local tags=""
    if [ -f $O/pmc_TCP_TOTAL_CACHE_ACCESSES_sum/run_counter_collection.csv ]; then
      cp $O/pmc_TCP_TOTAL_CACHE_ACCESSES_sum/run_counter_collection.csv $P/pmc_tags.csv
      tags=$P/pmc_tags.csv
    fi
    python tools/pmc_summary.py $P/pmc_fetch_size.csv $P/pmc_write_size.csv $tags \
      --traffic-out $P/traffic.json \
      --key "$(python -c "import json; print(json.load(open('$O/pmc_FETCH_SIZE.json'))['roofline']['traffic_key'])")" \
      > $P/pmc_summary.txt
  fi
  if [ -d $O/pmc_cfg ]; then
    for j in $O/pmc_cfg/*_FETCH_SIZE.json; do
      local n=$(basename $j _FETCH_SIZE.json)
      python tools/pmc_summary.py $O/pmc_cfg/${n}_FETCH_SIZE/run_counter_collection.csv \
        $O/pmc_cfg/${n}_WRITE_SIZE/run_counter_collection.csv \
        $(ls $O/pmc_cfg/${n}_TCP_TOTAL_CACHE_ACCESSES_sum/run_counter_collection.csv 2>/dev/null) \
        --traffic-out $P/traffic.json \
        --key "$(python -c "import json; print(json.load(open('$j'))['roofline']['traffic_key'])")" \
        > $P/pmc_summary_$n.txt
    done
  fi
  if [ -d $O/presets ]; then
    mkdir -p $P/presets
    cp $O/presets/*.json $P/presets/
    python tools/presets_table.py $P/presets > $P/presets_table.md
  fi
  if [ -d $O/kernel_test ]; then
    mkdir -p $P/kernel_test
    cp $O/kernel_test/*.txt $P/kernel_test/
    python tools/kt_table.py $P/kernel_test > $P/kernel_test_table.md
  fi
  if [ -d $O/kernel_test_cpp ]; then
    mkdir -p $P/kernel_test_cpp
    cp $O/kernel_test_cpp/*.txt $P/kernel_test_cpp/
  fi
  if [ -d $O/train ]; then
    mkdir -p $P/train
    cp $O/train/*.json $P/train/
  fi
}

for s in "$@"; do
  echo "== $s"
  step_$s
done
echo "session $R done: $*"
