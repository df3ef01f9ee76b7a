#!/bin/bash
# Round 5: LayerNorm backward with two rows of loads in flight -- LN / dropout numerics, then the
# fused-op time + counter passes (ln_bwd_blk was 103 us at T = 32768 before).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_dropout_gpu.py -k "layer or ln or norm or dropout" > gpurun_out/r5o/tests.log 2>&1 \
  || { grep -E "Error|assert|FAILED" gpurun_out/r5o/tests.log | head -20; tail -5 gpurun_out/r5o/tests.log; exit 1; }
tail -1 gpurun_out/r5o/tests.log
bash tools/gpu_r5l.sh | grep -E "rc=|ln_bwd|ln_fwd"
