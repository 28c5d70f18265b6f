#!/bin/bash
# r04 GPU call C: the deferred top-k error count (tests + A/B against the r03 kernel), the
# products forward with its columns folded into cache-sized windows (what a resident record
# table would cost), tag / L2 counters of the Reddit pull and the products forward, and the
# 3-layer epoch with and without the k = 32 edge-selector stream.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04
mkdir -p $O/topk $O/probe $O/train
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k "topk" -x -q --timeout 120 \
  --timeout-method thread > $O/topk/pytest_topk2.log 2>&1
tail -1 $O/topk/pytest_topk2.log
V=spgemm-prunning_amd/lib/variants
for rep in 1 2; do for v in base topk_r03; do
  lib=$V/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  for rows in 232965 2449029; do
    echo "== $v rows=$rows rep=$rep"
    MAXK_HIP_LIB=$lib timeout -k 10 120 python tools/topk_ab.py --rows $rows
  done
done; done > $O/topk/topk_ab2.txt 2>&1
echo "topk ab done"
for k in 8 16; do
  timeout -k 10 300 python tools/fwd_slice_probe.py --graph products --k $k \
    > $O/probe/fwd_window_products_k$k.txt 2>&1
done
echo "window probe done"
CFGS="reddit_k8:--k 8 reddit_k16:--k 16 products_k8:--graph products --k 8 products_k32s:--graph products --k 32 --edge-sel 1" \
SETS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum" \
  bash tools/session.sh r04 pmcset
i=0
for es in auto 1 auto 1; do
  i=$((i+1))
  MAXK_EDGE_SEL=$es timeout -k 10 400 python3 spgemm-prunning_amd/maxk_train_bench.py products \
    > $O/train/products_es${es}_$i.json 2> $O/train/products_es${es}_$i.err
  echo "epoch products MAXK_EDGE_SEL=$es: $(cut -c1-300 $O/train/products_es${es}_$i.json)"
done
