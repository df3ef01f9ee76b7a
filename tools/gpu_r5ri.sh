#!/bin/bash
# Round 5: in-place packed-QKV rotary (rotary channels only) -- rope / rotary-layer / GPT-J +
# NeoX hybrid GPU tests, then a same-box shard A/B against the per-view path (two passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5ri
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_hybrid_gpu.py -k "rope or rotary or gptj or neox" > gpurun_out/r5ri/tests.log 2>&1 \
  || { tail -40 gpurun_out/r5ri/tests.log; exit 1; }
tail -1 gpurun_out/r5ri/tests.log
for rep in 1 2; do
  for S in gptj_tp4 neox_pp2tp4; do
    for cfg in "default" "SMP_ROPE_PACKED=0"; do
      envs=""; [ "$cfg" != default ] && envs="$cfg"
      env $envs timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 \
        > gpurun_out/r5ri/$S.log 2>&1 || { tail -20 gpurun_out/r5ri/$S.log; exit 1; }
      echo "$S [$cfg] $(grep SHARD gpurun_out/r5ri/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"])')"
    done
  done
done
