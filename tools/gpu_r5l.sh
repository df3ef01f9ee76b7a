#!/bin/bash
# Round 5: the fused HIP ops (LayerNorm, residual dropout, bias+GeLU, masked / causal softmax,
# RoPE, vocab cross-entropy) fwd+bwd at training shapes (tools/fused_ops_only.py): a kernel-trace
# pass for times, then counter passes (one set per run, kernel-trace + pmc only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r5l
mkdir -p $out
run() {  # tag rocprof-args...
  local tag=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace "$@" -d $out/$tag -o run --output-format csv -- python3 tools/fused_ops_only.py > $out/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) tail -5 $out/$tag.log; exit $rc;; esac
}
run time --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_table.py $out/time $out/fetch $out/write $out/sq smpk > $out/table.md && cat $out/table.md
