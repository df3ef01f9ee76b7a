#!/bin/bash
# Round 5: BASELINE config 3 / 4 heaviest-rank shards on one MI355X with the round-5 kernels
# (timing run + a kernel trace of the last step each), compare profiles/r4/shards_configs34.md.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5sh
for S in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 400 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 > gpurun_out/r5sh/$S.log 2>&1 \
    || { tail -20 gpurun_out/r5sh/$S.log; exit 1; }
  grep SHARD gpurun_out/r5sh/$S.log
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5sh/trace_$S -o t -- python3 tools/shard_bench.py $S --mbs 8 \
    --steps 3 --warmup 2 > gpurun_out/r5sh/trace_$S.log 2>&1 || { tail -20 gpurun_out/r5sh/trace_$S.log; exit 1; }
  f=$(find gpurun_out/r5sh/trace_$S -name "*.db" | head -1)
  python3 tools/step_kernels.py "$f" > gpurun_out/r5sh/kernels_$S.txt && head -24 gpurun_out/r5sh/kernels_$S.txt
  rm -f "$f"
done
