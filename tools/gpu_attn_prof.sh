#!/bin/bash
# Attention kernel microbench + per-kernel rocprofv3 stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/attnprof
timeout -k 10 300 python tools/bench_kernels.py --attention > gpurun_out/attn_bench.json 2>gpurun_out/attn_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attnprof -o run --output-format csv -- python tools/bench_kernels.py --attention > gpurun_out/attnprof.log 2>&1 || exit $?
f=$(find gpurun_out/attnprof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$f" 1 30 || head -30 "$f"
