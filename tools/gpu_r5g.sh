#!/bin/bash
# Round 5: fused vs split attention backward -- per-kernel times, then counters (one set per pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r5g
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python3 tools/attn_fused_time.py > $out/stats.log 2>&1
rc=$?; echo "stats rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc "$@" -d $out/$tag -o run --output-format csv -- python3 tools/attn_fused_time.py > $out/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
}
run mfma SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS
exit 0
