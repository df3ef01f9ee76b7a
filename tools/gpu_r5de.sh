#!/bin/bash
# Round 5: fused attention backward (numerics, timing), LN-backward dropout fusion tests, then the
# GPT-J TP4 bf16 one-shot triage.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r5e.sh
echo "=== dropout / LN"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dropout_gpu.py \
  > gpurun_out/r5e/dropout.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/r5e/dropout.log
echo "=== r5d"
bash tools/gpu_r5d.sh
