#!/bin/bash
# Round 5: after the weight-gradient bias policy change -- wgrad / linear GPU tests, both
# config 3 / 4 shards at the new default, and the default GPT-2 XL bench (unaffected shapes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5wc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py \
  > gpurun_out/r5wc/tests.log 2>&1 || { tail -30 gpurun_out/r5wc/tests.log; exit 1; }
tail -1 gpurun_out/r5wc/tests.log
for S in gptj_tp4 neox_pp2tp4 gptj_tp4 neox_pp2tp4; do
  timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 > gpurun_out/r5wc/$S.log 2>&1 \
    || { tail -20 gpurun_out/r5wc/$S.log; exit 1; }
  echo "$S $(grep SHARD gpurun_out/r5wc/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"], r["tokens_per_s"], r.get("model_tflops_shard"))')"
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5wc/bench.log 2>&1 || { tail -20 gpurun_out/r5wc/bench.log; exit 1; }
grep '"metric"' gpurun_out/r5wc/bench.log
