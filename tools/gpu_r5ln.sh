#!/bin/bash
# Round 5: wide-row LayerNorm backward with a two-row register ring -- LN GPU tests on the
# in-tree build, then the A/B (abtest/_C_lr0 = one row at a time, _C_lr1 = ring), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5ln
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "layernorm or add_layernorm" > gpurun_out/r5ln/tests.log 2>&1 || { tail -30 gpurun_out/r5ln/tests.log; exit 1; }
tail -1 gpurun_out/r5ln/tests.log
for rep in 1 2; do
  for v in lr0 lr1; do
    timeout -k 10 120 python -u tools/ln_wide_time.py abtest/_C_$v.so 2>&1 | grep -v "amdgpu.ids" || exit 1
  done
done
