#!/bin/bash
# Top-k threshold search with interpolated probes (variant) against plain bisection (base):
# bit-exact tests with the variant, then times on products- and Reddit-sized rows, twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03/topk_interp; mkdir -p $O
V=$PWD/spgemm-prunning_amd/lib/variants
MAXK_HIP_LIB=$V/interp/libmaxk_hip.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "topk or fuzz or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for v in base interp; do
  echo "== $v"
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 python -u tools/topk_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  MAXK_HIP_LIB=$V/$v/libmaxk_hip.so timeout -k 10 300 python -u tools/topk_ab.py --rows 232965 2>&1 | grep -v amdgpu.ids || exit 1
done; done
