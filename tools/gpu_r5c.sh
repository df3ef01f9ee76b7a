#!/bin/bash
# Round 5: new / tightened GPU tests -- bf16 / fp16 hybrid equivalence, relative-norm kernel
# bounds, plain-torch bench-shape reference, premul-sum, mixed-device mask decision.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_hybrid_gpu.py tests/test_kernels_gpu.py tests/test_runtime_gpu.py \
  "tests/test_attention_gpu.py::test_gpt2xl_width_step_matches_fp32" > gpurun_out/r5c/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5c/tests.log | grep -v PASSED | head -30
tail -2 gpurun_out/r5c/tests.log
exit $rc
