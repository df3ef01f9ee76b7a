#!/bin/bash
# One gpurun call rehearsing the driver's round-end tiers: every GPU test, smoke(), the
# default bench, then a rocprofv3 kernel profile of the bench. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_round.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v INFO gpurun_out/bench_round.log | tail -3
[ $rc -ne 0 ] && exit $rc
[ "${PROF:-1}" = "0" ] && exit 0
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 $BENCH_ARGS > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v INFO gpurun_out/prof_bench.log | tail -2
exit $rc
