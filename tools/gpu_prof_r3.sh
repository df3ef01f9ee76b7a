#!/bin/bash
# Round 3: attention A/B (reverted dropout path vs round start), then bench kernel profiles
# at dropout 0 and 0.1 (rocprofv3 --kernel-trace --stats, 4 timed + 2 warm-up steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof3
SKIP_TESTS=1 bash tools/gpu_attn_ab.sh 2>&1 | tail -4
for DR in 0.0 0.1; do
  rm -rf gpurun_out/prof3/d$DR && mkdir -p gpurun_out/prof3/d$DR
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/d$DR -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 2 --dropout $DR > gpurun_out/prof3/bench_d$DR.log 2>&1 || exit $?
  f=$(find gpurun_out/prof3/d$DR -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 6 45 > gpurun_out/prof3/summary_d$DR.md
  grep '"metric"' gpurun_out/prof3/bench_d$DR.log | cut -c1-200
  head -22 gpurun_out/prof3/summary_d$DR.md
done
