#!/bin/bash
# GPU tests + bench of every preset (one JSON line each) into gpurun_out/presets/
set -e
O=gpurun_out/presets; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1; tail -1 $O/pytest.log
timeout -k 10 300 python bench.py > $O/reddit.json 2> $O/reddit.err; cat $O/reddit.json
for g in products proteins flickr; do
  timeout -k 10 300 python bench.py --graph $g --no-cpu-baseline > $O/$g.json 2> $O/$g.err; cat $O/$g.json
done
for k in 8 32 64; do
  timeout -k 10 300 python bench.py --k $k --no-cpu-baseline --no-rocsparse > $O/reddit_k$k.json 2> $O/reddit_k$k.err; cat $O/reddit_k$k.json
done
timeout -k 10 300 python bench.py --bwd-mode bucket --no-cpu-baseline --no-rocsparse > $O/reddit_bucket.json 2> $O/reddit_bucket.err; cat $O/reddit_bucket.json
timeout -k 10 300 python bench.py --bwd-mode csc --no-cpu-baseline --no-rocsparse > $O/reddit_csc.json 2> $O/reddit_csc.err; cat $O/reddit_csc.json
timeout -k 10 300 python bench.py --bwd-mode atomic --no-cpu-baseline --no-rocsparse > $O/reddit_atomic.json 2> $O/reddit_atomic.err; cat $O/reddit_atomic.json
for g in products reddit; do
  timeout -k 10 600 python spgemm-prunning_amd/maxk_train_bench.py $g > $O/train_$g.json 2> $O/train_$g.err; cat $O/train_$g.json
done
for k in 8 16 64; do
  timeout -k 10 300 python bench.py --graph products --k $k --no-cpu-baseline --no-rocsparse > $O/products_k$k.json 2> $O/products_k$k.err; cat $O/products_k$k.json
done
