#!/bin/bash
# Round 5 final: attention kernel counters at the bench shape (b 32, h 25, s 2048, d 64, causal,
# dropout 0.1): one kernel-trace pass for times, then one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp B=32 P=0.1 ITERS=2
mkdir -p gpurun_out/r5pa
timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/r5pa/stats -o run --output-format csv -- python3 tools/attn_only.py \
  > gpurun_out/r5pa/stats.log 2>&1 || { echo "stats rc=$?"; exit 1; }
run() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/r5pa/$tag -o run --output-format csv -- python3 tools/attn_only.py > gpurun_out/r5pa/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run mfma SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS
run mem FETCH_SIZE
python3 tools/pmc_table.py gpurun_out/r5pa/stats gpurun_out/r5pa/mfma gpurun_out/r5pa/wait gpurun_out/r5pa/lds attn > gpurun_out/r5pa/table.md
cat gpurun_out/r5pa/table.md
