#!/bin/bash
# New GPU tests of this session (leak, weight-gradient split ladder), then the round-end tiers.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_leak_gpu.py tests/test_wgrad_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -8 gpurun_out/new_tests.log
exit $rc
