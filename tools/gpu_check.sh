#!/bin/bash
# One gpurun call: kernel numerics, smoke, short bench. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-6}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v INFO gpurun_out/bench.log | tail -5
exit $rc
