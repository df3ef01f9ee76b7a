#!/bin/bash
# Round 4: dropout-path prefetch variants -- attention GPU tests on the in-tree build, then
# per-kernel A/B of abtest/_C_<VARIANTS>.so against it (tools/gpu_r4i.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_gpu.py \
  > gpurun_out/r4m/tests.log 2>&1 || { tail -30 gpurun_out/r4m/tests.log; exit 1; }
tail -2 gpurun_out/r4m/tests.log
bash tools/gpu_r4i.sh
