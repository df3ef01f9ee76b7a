#!/bin/bash
# Hardware counters for the weight-gradient kernel vs the library GEMM (tools/wgrad_one.py):
# kernel-trace + pmc only, one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcw/$tag -o run --output-format csv -- python3 tools/wgrad_one.py > gpurun_out/pmcw/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
  return 0
}
run mfma SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL
run fetch FETCH_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
exit 0
