#!/bin/bash
# Round 5: TunableOp GEMM selection for the config 3 / 4 shard shapes -- tune (writes
# configs/tunableop/<shard>_mbs8_s2048.csv), then the same-box A/B: heuristic vs tuned, two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5tu configs/tunableop
for S in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 1200 python -u tools/shard_bench.py $S --mbs 8 --steps 2 --warmup 3 --tunableop tune \
    > gpurun_out/r5tu/tune_$S.log 2>&1 || { tail -20 gpurun_out/r5tu/tune_$S.log; exit 1; }
  cp configs/tunableop/${S}_mbs8_s2048.csv gpurun_out/r5tu/
  echo "tuned $S: $(grep -c Tunable configs/tunableop/${S}_mbs8_s2048.csv) entries"
done
for rep in 1 2; do
  for S in gptj_tp4 neox_pp2tp4; do
    for m in off use; do
      timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 --tunableop $m \
        > gpurun_out/r5tu/$S.log 2>&1 || { tail -20 gpurun_out/r5tu/$S.log; exit 1; }
      echo "$S [$m] $(grep SHARD gpurun_out/r5tu/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"], r["gemm_selection"])')"
    done
  done
done
