set -eo pipefail
mkdir -p gpurun_out/r04/topk
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k "topk" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/topk/pytest_topk.log 2>&1
tail -1 gpurun_out/r04/topk/pytest_topk.log
V=spgemm-prunning_amd/lib/variants
for rep in 1 2; do for v in base topk_rowsum topk_r03; do
  lib=$V/$v/libmaxk_hip.so; [ $v = base ] && lib=spgemm-prunning_amd/lib/libmaxk_hip.so
  for rows in 232965 2449029; do
    echo "== $v rows=$rows rep=$rep"
    MAXK_HIP_LIB=$lib timeout -k 10 120 python tools/topk_ab.py --rows $rows
  done
done; done > gpurun_out/r04/topk/topk_ab.txt 2>&1
bash tools/session.sh r04 kt
