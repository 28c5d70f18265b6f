set -eo pipefail
mkdir -p gpurun_out/r04/chunk
for k in 8 32; do for c in 0 512 1024 4096 0; do
  timeout -k 10 300 python bench.py --graph products --k $k --chunk $c --steps 20 --no-cpu-baseline --no-rocsparse --no-cpu-spmm > gpurun_out/r04/chunk/k${k}_c$c.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/r04/chunk/k${k}_c$c.json')); e=d['extra']; print('k=$k chunk=$c', e['fwd_ms'], e['bwd_ms'], d['value'])"
done; done 2>&1 | tee gpurun_out/r04/chunk/summary.txt
