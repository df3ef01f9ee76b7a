#!/bin/bash
# Attention kernel A/B: correctness tests of the in-tree build, then interleaved timings of
# abtest/_C_base.so (previous build) vs the in-tree build on the GPT-2 XL shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/attnab
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_dropout_gpu.py ${EXTRA_TESTS} \
  > gpurun_out/attnab/pytest.log 2>&1 || { tail -30 gpurun_out/attnab/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/attnab/pytest.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_time.py abtest/_C_base.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
  timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
done
