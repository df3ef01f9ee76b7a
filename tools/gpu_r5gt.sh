#!/bin/bash
# Round 5: kernel traces of the config 3 / 4 shards at the final defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5gt
for S in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5gt/trace_$S -o t -- python3 tools/shard_bench.py $S --mbs 8 \
    --steps 3 --warmup 2 > gpurun_out/r5gt/trace_$S.log 2>&1 || { tail -20 gpurun_out/r5gt/trace_$S.log; exit 1; }
  f=$(find gpurun_out/r5gt/trace_$S -name "*.db" | head -1)
  python3 tools/step_kernels.py "$f" > gpurun_out/r5gt/kernels_$S.txt && head -40 gpurun_out/r5gt/kernels_$S.txt
  rm -f "$f"
done
