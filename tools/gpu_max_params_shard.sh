#!/bin/bash
# BASELINE config 5 evidence: one rank's shard of GPT-3 175B at PP=4 x TP=2 (embedding + 24
# layers, TP-sliced shapes) trained for 3 steps on one MI355X; AdamW moments in pinned host
# memory (exact-size hipHostRegister'd arrays), master weights in HBM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/maxp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_runtime_gpu.py::test_optimizer_state_offload_matches_resident > gpurun_out/maxp/pytest.log 2>&1 \
  || { tail -30 gpurun_out/maxp/pytest.log; exit 1; }
tail -2 gpurun_out/maxp/pytest.log
free -g | head -2
SMP_OFFLOAD_OPTIMIZER_FIELDS=${FIELDS:-m,v} SMP_LOG_LEVEL=warning timeout -k 10 900 \
  python -u tools/max_params.py shard --layers 24 > gpurun_out/maxp/shard.log 2>&1
rc=$?; grep -v "^\[" gpurun_out/maxp/shard.log | tail -8; exit $rc
