#!/bin/bash
# Round 5: keep bits regenerated from the hash above the per-layer budget -- equality with the
# stored words and bitwise-equal backward; the attention and dropout GPU suites.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_dropout_gpu.py > gpurun_out/r5n/tests.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/r5n/tests.log | head -20; tail -5 gpurun_out/r5n/tests.log; exit 1; }
tail -1 gpurun_out/r5n/tests.log
