#!/bin/bash
# wgrad kernel variants (SMP_WGRAD_PIPE), interleaved twice, then the wgrad GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wgab
for i in 1 2; do
  for P in ${PIPES:-1 6 2 7}; do
    SMP_WGRAD_PIPE=$P timeout -k 10 120 python tools/wgrad_ab.py 2>&1 | grep '^{' || exit 1
  done
done
for P in ${PIPES:-1 6 2 7}; do
  SMP_WGRAD_PIPE=$P timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py > gpurun_out/wgab/pytest_$P.log 2>&1 || { echo "tests failed pipe=$P"; tail -20 gpurun_out/wgab/pytest_$P.log; exit 1; }
  echo "pipe=$P: $(tail -1 gpurun_out/wgab/pytest_$P.log)"
done
