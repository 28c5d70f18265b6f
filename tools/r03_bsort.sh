#!/bin/bash
# Window-sorted backward on the GPU box: its parity tests, the probe (bsort against csc /
# bucket, with and without the edge-selector stream) and a kernel-trace profile of it;
# optional variant libraries under spgemm-prunning_amd/lib/variants/ probed after.
set -eo pipefail
O=gpurun_out/bsort
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bsort" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 400 python -u tools/bsort_probe.py --k 4 8 > $O/probe.txt 2>&1
cat $O/probe.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 tools/bsort_probe.py --k 8 --iters 5 > $O/probe_prof.txt 2>&1
V=spgemm-prunning_amd/lib/variants
for v in $(ls $V 2>/dev/null); do
  MAXK_HIP_LIB=$PWD/$V/$v/libmaxk_hip.so timeout -k 10 300 python -u tools/bsort_probe.py --k 8 > $O/probe_$v.txt 2>&1
  echo "$v: $(cat $O/probe_$v.txt | tail -1)"
done
echo done
