#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_leak_gpu.py -x -q -s --timeout 150 --timeout-method thread > gpurun_out/leak.log 2>&1
rc=$?; echo "leak rc=$rc"; grep -h "LEAKINFO\|passed\|failed" gpurun_out/leak.log | cut -c1-800
exit $rc
