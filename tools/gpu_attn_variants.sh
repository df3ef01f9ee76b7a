#!/bin/bash
# A/B the attention kernel variants built under build_attn/ (tools/attn_bench.cpp), then
# collect per-kernel counters for the baseline.  Every GPU step has its own time limit
# and the script stops at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/attn
mkdir -p $out
stop() { case $1 in 124|137|134|139) echo "stopping after rc=$1"; exit $1;; esac; }
for exe in build_attn/attn_bench_*; do
  tag=$(basename $exe)
  timeout -k 10 120 $exe ${SHAPE:-32 2048 25 64} 20 > $out/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc: $(tail -1 $out/$tag.log)"; stop $rc
done
[ "${PMC:-1}" = 1 ] || exit 0
pmc() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc "$@" -d $out/pmc_$tag -o run --output-format csv -- build_attn/attn_bench_v0 8 2048 25 64 3 > $out/pmc_$tag.log 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"; stop $rc
}
pmc wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pmc inst SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES
exit 0
