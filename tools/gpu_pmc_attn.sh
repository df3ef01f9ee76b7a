#!/bin/bash
# Hardware counters for the attention kernels (tools/attn_only.py): kernel-trace + pmc only,
# one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmca
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmca/$tag -o run --output-format csv -- python3 tools/attn_only.py > gpurun_out/pmca/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
  return 0
}
export P=${P:-0.0}
run mfma SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS
exit 0
