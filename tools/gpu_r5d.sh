#!/bin/bash
# Round 5: GPT-J TP4 bf16 one-shot timeout triage -- the test as is (durations), then with the
# one-shot path off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread --durations=0 \
  "tests/test_hybrid_gpu.py::test_gptj6b_width_tp4_bf16_gpu" > gpurun_out/r5d/t1.log 2>&1
echo "rc1=$?"; grep -E "passed|failed|s call" gpurun_out/r5d/t1.log | tail -3
SMP_ONESHOT_TRACE=1 timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread --durations=0 \
  "tests/test_hybrid_gpu.py::test_gptj6b_width_tp4_bf16_gpu" -p no:cacheprovider > gpurun_out/r5d/t2.log 2>&1
echo "rc2=$?"; grep -E "passed|failed|s call" gpurun_out/r5d/t2.log | tail -3
