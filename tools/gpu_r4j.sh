#!/bin/bash
# Round 4: parallel-attention residual fusion (add3 + LN passthrough) -- numerics, GPT-J / NeoX
# width hybrid tests, and the config-3/4 shard timings after the change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "add3 or add_layernorm" tests/test_hybrid_gpu.py -k "add3 or add_layernorm or gptj or neox" \
  > gpurun_out/r4j/tests.log 2>&1 || { tail -30 gpurun_out/r4j/tests.log; exit 1; }
tail -3 gpurun_out/r4j/tests.log
for s in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 300 python -u tools/shard_bench.py $s --mbs 8 --steps 5 --warmup 3 > gpurun_out/r4j/$s.log 2>&1 \
    || { tail -20 gpurun_out/r4j/$s.log; exit 1; }
  grep SHARD gpurun_out/r4j/$s.log
done
