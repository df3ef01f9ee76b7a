#!/bin/bash
# Round 5: vector RoPE kernel -- numerics (fp32 / bf16 / fp16, vec8 / vec4 / scalar paths), then
# the fused-op counter passes again (tools/gpu_r5l.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k rope \
  > gpurun_out/r5m/tests.log 2>&1 || { tail -30 gpurun_out/r5m/tests.log; exit 1; }
tail -1 gpurun_out/r5m/tests.log
bash tools/gpu_r5l.sh
