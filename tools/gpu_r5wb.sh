#!/bin/bash
# Round 5: weight-gradient policy on the config 3 / 4 shard shapes (K = 4096 / 6144, where the
# ping-pong kernel has no fused bias mode): default (bias fused into the round-4 kernel) vs
# SMP_WGRAD_DBIAS=0 (table pick, separate column sums) vs SMP_WGRAD_KERNEL=1 SMP_WGRAD_DBIAS=0
# (ping-pong kernel on every shape, separate column sums).  Two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5wb
for rep in 1 2; do
  for S in gptj_tp4 neox_pp2tp4; do
    for cfg in "default" "SMP_WGRAD_DBIAS=0" "SMP_WGRAD_KERNEL=1 SMP_WGRAD_DBIAS=0"; do
      envs=""; [ "$cfg" != default ] && envs="$cfg"
      env $envs timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 \
        > gpurun_out/r5wb/$S.log 2>&1 || { tail -20 gpurun_out/r5wb/$S.log; exit 1; }
      echo "$S [$cfg] $(grep SHARD gpurun_out/r5wb/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"])')"
    done
  done
done
