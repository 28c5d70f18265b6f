set -o pipefail
for v in ${VARIANTS:-base abl1 abl4 abl8}; do
  MATCH=pull_q MAXK_HIP_LIB=$PWD/spgemm-prunning_amd/lib/variants/$v/libmaxk_hip.so bash tools/pmc_sets.sh gpurun_out/pmcv_$v "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE TA_BUSY_avr SQ_INSTS_VMEM_RD" -- python3 tools/pull_ab.py --k 16 --slices 0 --iters 3 > gpurun_out/pmcv_$v.txt 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/pmcv_$v.txt
done
