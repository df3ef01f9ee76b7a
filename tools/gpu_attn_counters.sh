#!/bin/bash
# Attention kernel counters at the bench shape (tools/attn_only.py, B 32 / P 0.1 by default):
# one kernel-trace pass for times, then one counter set per rocprofv3 pass (kernel-trace + pmc
# only), summarised by tools/pmc_table.py.  usage: tools/gpu_attn_counters.sh OUT
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp B=${B:-32} P=${P:-0.1} ITERS=${ITERS:-2}
out=gpurun_out/$1
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --kernel-trace -d "$out/time" -o run --output-format csv -- python3 tools/attn_only.py \
  > "$out/time.log" 2>&1 || { echo "time pass failed"; exit 1; }
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$out/$tag" -o run --output-format csv -- \
    python3 tools/attn_only.py > "$out/$tag.log" 2>&1
  local rc=$?; echo "$tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run mfma SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAVES
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS
python3 tools/pmc_table.py "$out/time" "$out/mfma" "$out/wait" "$out/lds" "attn|keep_bits" > "$out/table.md"
cat "$out/table.md"
