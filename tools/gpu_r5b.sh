#!/bin/bash
# Round 5: bench A/B on one box -- ping-pong weight-gradient kernel (default) vs the round-4
# kernel (SMP_WGRAD_IMPL=glds), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
for arm in pp glds pp glds; do
  if [ $arm = glds ]; then export SMP_WGRAD_IMPL=glds; else unset SMP_WGRAD_IMPL; fi
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5b/bench_$arm.log 2>&1 \
    || { tail -20 gpurun_out/r5b/bench_$arm.log; exit 1; }
  echo "$arm $(grep '"metric"' gpurun_out/r5b/bench_$arm.log | cut -c1-200)"
done
