#!/bin/bash
# Round 5: fused attention backward kernel profile (kernel trace + stats) at the bench shape,
# and the GPT-J TP4 bf16 test on the RCCL/gloo TP path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/prof -o attn -- python tools/attn_fused_time.py \
  > gpurun_out/r5f/prof.log 2>&1 || { tail -20 gpurun_out/r5f/prof.log; exit 1; }
grep bwd_us gpurun_out/r5f/prof.log
find gpurun_out/r5f/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {} | cut -c1-220'
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread \
  "tests/test_hybrid_gpu.py::test_gptj6b_width_tp4_bf16_gpu" > gpurun_out/r5f/gptj.log 2>&1
echo "gptj rc=$?"; tail -1 gpurun_out/r5f/gptj.log
