#!/bin/bash
# Four-row top-k threshold search: bisection over [lower bound, max] (default build) vs the bit
# search from the lower bound (variant bits) and from the row minimum (variant lb0):
# parity tests, then bench's top-k time (U(0,1) rows) and Gaussian rows.
set -eo pipefail
O=gpurun_out/topk_lb; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_layers_gpu.py -x -q --timeout 300 --timeout-method thread -k "topk or random_graphs or maxk" > $O/test.log 2>&1
tail -1 $O/test.log
B="--no-cpu-baseline --no-cpu-spmm --no-rocsparse"
for v in default "$@"; do
  if [ $v = default ]; then unset MAXK_HIP_LIB; else export MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so; fi
  for cfg in "reddit" "reddit_k32 --k 32" "products --graph products" "products_k16 --graph products --k 16" "proteins_k32 --graph proteins --k 32"; do
    set -- $cfg; n=$1; shift
    timeout -k 10 300 python3 bench.py $B "$@" > $O/${v}_$n.json 2> $O/${v}_$n.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'topk_ms', d['extra']['topk_ms'])" $O/${v}_$n.json "$v $n"
  done
  timeout -k 10 300 python3 tools/topk_gauss.py > $O/${v}_gauss.txt 2>&1
  sed "s/^/$v /" $O/${v}_gauss.txt | grep gauss
done
echo topk lb done
