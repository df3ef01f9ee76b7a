#!/bin/bash
# Round 5: cross-layer residual fusion (MLP dropout + residual add deferred into the next
# layer's LayerNorm kernel) -- bitwise check against the separate kernels, the bench-shape model
# test, then the bench with it on and off (same box, alternating).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_dropout_gpu.py::test_cross_layer_residual_fusion_is_bitwise_neutral" \
  "tests/test_attention_gpu.py::test_gpt2xl_width_step_matches_fp32" > gpurun_out/r5p/tests.log 2>&1 \
  || { grep -E "Error|assert|FAILED|OK|loss" gpurun_out/r5p/tests.log | head -30; tail -5 gpurun_out/r5p/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5p/tests.log | tail -2
for i in 1 2; do
  for f in 1 0; do
    SMP_FUSE_CROSS_LAYER_RESIDUAL=$f timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5p/bench_${f}_${i}.log 2>&1 \
      || { tail -20 gpurun_out/r5p/bench_${f}_${i}.log; exit 1; }
    echo "fuse=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5p/bench_${f}_${i}.log)"
  done
done
