#!/bin/bash
# Round 5: the default 1-GPU bench with dropout 0 (attention / hidden / embedding), a data point
# for dropout-free training (the bench default is 0.1), plus the default for a same-box reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5nd
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --dropout 0 > gpurun_out/r5nd/d0.log 2>&1 || { tail -20 gpurun_out/r5nd/d0.log; exit 1; }
grep '"metric"' gpurun_out/r5nd/d0.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5nd/d01.log 2>&1 || { tail -20 gpurun_out/r5nd/d01.log; exit 1; }
grep '"metric"' gpurun_out/r5nd/d01.log | cut -c1-200
