#!/bin/bash
# Round 3 session 2 start: GPU tests, smoke, default bench, kernel profile of the default
# bench (dropout 0.1), attention stall counters.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
PROF=0 bash tools/gpu_round.sh || exit $?
mkdir -p gpurun_out/prof_r3s2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3s2/k -o run --output-format csv -- \
  python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_r3s2/bench.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r3s2/k -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 6 45 > gpurun_out/prof_r3s2/summary.md
head -30 gpurun_out/prof_r3s2/summary.md
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/prof_r3s2/$tag -o run --output-format csv -- python3 tools/attn_only.py > gpurun_out/prof_r3s2/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
}
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run inst SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
run lvl SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE
exit 0
