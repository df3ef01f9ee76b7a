#!/bin/bash
# Round-3 GPU tests: hybrid feature matrix on GPU tensors, fast mode over IPC, static
# weight-gradient pick, one-shot failure path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3t
timeout -k 10 900 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_hybrid_gpu.py \
  tests/test_pipeline_gpu.py::test_pp4_fast_mode_ipc tests/test_wgrad_gpu.py::test_wgrad_static_pick_is_deterministic \
  > gpurun_out/r3t/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/r3t/pytest.log; exit $rc
