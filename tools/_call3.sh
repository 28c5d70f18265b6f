# r05 session: smoke (now with the dense route), then the N = 8 step model of the grouped-csc
# build (products k = 32, pipelined parts 1 / 2) and the N = 4 shard probe
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s20
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python tools/shard_probe.py --graph products --k 32 --worlds 1 4 8 --pipelines 1 2 > $O/shard_products_k32_model.txt 2>&1
cat $O/shard_products_k32_model.txt
