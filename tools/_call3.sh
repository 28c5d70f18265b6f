# r05 session: forward items of at least two average rows on dense graphs (fwd_long_rows) --
# parity, the Reddit shards at N = 1 / 4 / 8 and the default bench
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s29
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py tests/test_dist_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/shard_probe.py --graph reddit --k 16 --worlds 1 2 4 8 > $O/shard_reddit.txt 2>&1
grep -v amdgpu $O/shard_reddit.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cpu-spmm --no-rocsparse > $O/bench.json 2> $O/bench.err
cut -c1-200 $O/bench.json
