#!/bin/bash
# Per-kernel hardware counters for the memory-bound kernels (tools/mem_only.py) and the
# attention kernels (tools/attn_only.py): kernel-trace + pmc only, one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
run() {  # tag script counters...
  local tag=$1 script=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc2/$tag -o run --output-format csv -- python3 $script > gpurun_out/pmc2/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
  return 0
}
run mem_fetch tools/mem_only.py FETCH_SIZE
run mem_write tools/mem_only.py WRITE_SIZE
run mem_sq tools/mem_only.py SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run attn_mfma tools/attn_only.py SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run attn_fetch tools/attn_only.py FETCH_SIZE
exit 0
