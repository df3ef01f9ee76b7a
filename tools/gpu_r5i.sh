#!/bin/bash
# Round 5: ping-pong weight-gradient kernel counters at GPT-2 XL fc1 (dW 6400 x 1600, T 65536,
# 7 splits) and fc2 (1600 x 6400, 4 splits): kernel-trace + pmc only, one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r5i
mkdir -p $out
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $out/$tag -o run --output-format csv -- python3 tools/wgrad_one.py > $out/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
}
for shp in "6400 1600 7" "1600 6400 4"; do
  set -- $shp
  export WG_N=$1 WG_K=$2 WG_SPLITS=$3 WG_ITERS=3
  t=${1}x${2}
  run ${t}_mfma SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
  run ${t}_wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU
  run ${t}_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
  run ${t}_tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
  run ${t}_fetch FETCH_SIZE
done
exit 0
