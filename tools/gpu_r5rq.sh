#!/bin/bash
# Round 5: packed-QKV rotary (one dqkv buffer) + the weight-gradient bias policy --
# rope / wgrad / GPT-J + NeoX hybrid GPU tests, both config 3 / 4 shards (x2), kernel trace of
# the GPT-J shard, and the default GPT-2 XL bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5rq
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_wgrad_gpu.py tests/test_hybrid_gpu.py -k "rope or wgrad or gptj or neox or GPTJ or NeoX" \
  > gpurun_out/r5rq/tests.log 2>&1 || { tail -30 gpurun_out/r5rq/tests.log; exit 1; }
tail -1 gpurun_out/r5rq/tests.log
for S in gptj_tp4 neox_pp2tp4 gptj_tp4 neox_pp2tp4; do
  timeout -k 10 300 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 > gpurun_out/r5rq/$S.log 2>&1 \
    || { tail -20 gpurun_out/r5rq/$S.log; exit 1; }
  echo "$S $(grep SHARD gpurun_out/r5rq/$S.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"], r["tokens_per_s"], r.get("model_tflops_shard"), r.get("peak_mem_gb"))')"
done
for S in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5rq/trace_$S -o t -- python3 tools/shard_bench.py $S --mbs 8 \
    --steps 3 --warmup 2 > gpurun_out/r5rq/trace_$S.log 2>&1 || { tail -20 gpurun_out/r5rq/trace_$S.log; exit 1; }
  f=$(find gpurun_out/r5rq/trace_$S -name "*.db" | head -1)
  python3 tools/step_kernels.py "$f" > gpurun_out/r5rq/kernels_$S.txt && head -3 gpurun_out/r5rq/kernels_$S.txt
  rm -f "$f"
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5rq/bench.log 2>&1 || { tail -20 gpurun_out/r5rq/bench.log; exit 1; }
grep '"metric"' gpurun_out/r5rq/bench.log
