#!/bin/bash
# Kernel-level profile of the bench (rocprofv3 kernel trace + stats).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps ${STEPS:-3} --warmup 1 $BENCH_ARGS > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v INFO gpurun_out/prof_bench.log | tail -3
find gpurun_out/prof -name "*stats*" | head
exit $rc
