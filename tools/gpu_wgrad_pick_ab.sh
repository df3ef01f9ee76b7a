#!/bin/bash
# Same-box A/B of the weight-gradient algorithm pick (one timing round vs two interleaved
# rounds, SMP_WGRAD_PICK_ROUNDS), alternating, with the per-shape picks logged; then the
# attention counter passes (tools/gpu_pmc_attn.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in 1 2; do
  for r in 1 2; do
    SMP_WGRAD_PICK_ROUNDS=$r SMP_WGRAD_LOG=1 timeout -k 10 300 python bench.py --steps 12 --warmup 3 > gpurun_out/ab/r${r}_$i.log 2>&1
    rc=$?; echo "rounds=$r run=$i rc=$rc"; grep -h "wgrad T=\|metric" gpurun_out/ab/r${r}_$i.log | sed 's/, "config".*//'
    [ $rc -ne 0 ] && exit $rc
  done
done
bash tools/gpu_pmc_attn.sh
