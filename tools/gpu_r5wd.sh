#!/bin/bash
# Round 5: same-box A/B on the config 3 / 4 shards of the packed-QKV rotary (SMP_ROPE_PACKED=0:
# per-view rotation) and of the weight-gradient bias policy (SMP_WGRAD_DBIAS=wide: round-4 LDS
# mode for wide dY) against the new defaults.  Two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5wd
for rep in 1 2; do
  for S in gptj_tp4 neox_pp2tp4; do
    for cfg in "default" "SMP_ROPE_PACKED=0" "SMP_WGRAD_DBIAS=wide"; do
      envs=""; [ "$cfg" != default ] && envs="$cfg"
      env $envs timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 \
        > gpurun_out/r5wd/$S.log 2>&1 || { tail -20 gpurun_out/r5wd/$S.log; exit 1; }
      echo "$S [$cfg] $(grep SHARD gpurun_out/r5wd/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"])')"
    done
  done
done
