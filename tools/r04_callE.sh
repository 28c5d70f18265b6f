#!/bin/bash
# r04 GPU call E: N-rank rehearsals of the multi-GPU bench on the one-GPU box -- every rank a
# process on the same MI355X, collectives staged through host memory by gloo
# (MAXK_DIST_BACKEND=gloo; bench.py gives each rank one hardware queue) -- at the rank counts
# the driver's scaling run uses, on its default configuration (Reddit k = 16) and on
# ogbn-products k = 32.  Each bench run checks its sharded result against the unsharded one
# (extra.dist_check_*); the timings are of the shared GPU and host-staged collectives, not of
# N GPUs over RCCL.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04/rehearsal
mkdir -p $O
run() {  # run <name> <ranks> <bench args...>
  local n=$1 w=$2; shift 2
  MAXK_DIST_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29500 + w)) bench.py \
    --gpus $w --steps 5 --warmup 2 "$@" > $O/$n.json 2> $O/$n.err
  python - $O/$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[2], "fwd err", e["dist_check_fwd_max_rel_err"], "bwd err", e["dist_check_bwd_max_rel_err"],
      "mode", e["dist_mode"], "parts", e["dist_pipeline"], "bwd", e["bwd_mode"],
      "stream", e["edge_sel_stream"], "ms/step", d["ms_per_step"])
PY
}
run n8_reddit 8
run n4_reddit 4
run n8_products_k32 8 --graph products
