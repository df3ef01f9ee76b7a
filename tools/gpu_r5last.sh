#!/bin/bash
# Round 5 last call: smoke() and the LayerNorm / rope GPU tests on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5last
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5last/smoke.log 2>&1 \
  || { tail -20 gpurun_out/r5last/smoke.log; exit 1; }
grep "smoke ok" gpurun_out/r5last/smoke.log | head -1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "layernorm or rope or rotary" > gpurun_out/r5last/tests.log 2>&1 || { tail -30 gpurun_out/r5last/tests.log; exit 1; }
tail -1 gpurun_out/r5last/tests.log
