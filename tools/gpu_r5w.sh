#!/bin/bash
# Round 5: padded LM head (aligned logits rows; weight gradient on the ping-pong kernel) vs the
# unpadded hipBLASLt LM head, same box, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
for i in 1 2; do
  for f in 1 0; do
    SMP_PADDED_LM_HEAD=$f timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5w/bench_${f}_${i}.log 2>&1 \
      || { tail -20 gpurun_out/r5w/bench_${f}_${i}.log; exit 1; }
    echo "padded=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5w/bench_${f}_${i}.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r5w/bench_${f}_${i}.log)"
  done
done
