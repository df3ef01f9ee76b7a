#!/bin/bash
# Bench kernel profile: rocprofv3 --kernel-trace --stats over 4 timed + 2 warmup steps,
# summarised per step (tools/prof_summary.py) into gpurun_out/prof_summary.md.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/prof && mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 $BENCH_ARGS > gpurun_out/prof_bench.log 2>&1 || exit $?
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 6 45 > gpurun_out/prof_summary.md
tail -1 gpurun_out/prof_bench.log
head -30 gpurun_out/prof_summary.md
