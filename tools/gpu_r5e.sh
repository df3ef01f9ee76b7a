#!/bin/bash
# Round 5: fused attention backward -- numerics / determinism, then timing at the bench shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_attention_gpu.py::test_fused_bwd_matches_fp32_and_is_deterministic" > gpurun_out/r5e/tests.log 2>&1 \
  || { grep -E "Error|error|assert|FAILED" gpurun_out/r5e/tests.log | head -30; tail -5 gpurun_out/r5e/tests.log; exit 1; }
tail -1 gpurun_out/r5e/tests.log
timeout -k 10 200 python tools/attn_fused_time.py 2>&1 | grep -v "amdgpu.ids" | tail -3
