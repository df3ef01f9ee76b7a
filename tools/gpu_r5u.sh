#!/bin/bash
# Round 5: the full bf16 GPU path trains (40 AdamW steps memorise one batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_runtime_gpu.py::test_full_gpu_path_trains" > gpurun_out/r5u/tests.log 2>&1; rc=$?
grep -E "losses|OK|passed|failed|Error" gpurun_out/r5u/tests.log | cut -c1-600 | head -10
exit $rc
