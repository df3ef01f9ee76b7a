#!/bin/bash
# Round 4, first GPU pass: kernel/optimizer/one-shot GPU tests of the in-tree build, then the
# attention A/B against abtest/_C_base.so (round-3 build) and a short default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_dropout_gpu.py tests/test_optimizers_gpu.py tests/test_oneshot_gpu.py tests/test_wgrad_gpu.py tests/test_kernels_gpu.py > gpurun_out/r4a/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r4a/pytest.log; exit 1; }
tail -3 gpurun_out/r4a/pytest.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_time.py abtest/_C_base.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
  timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
done
timeout -k 10 300 python bench.py --steps 6 --warmup 3 > gpurun_out/r4a/bench.log 2>&1 || { tail -20 gpurun_out/r4a/bench.log; exit 1; }
tail -1 gpurun_out/r4a/bench.log
timeout -k 10 300 python tools/wgrad_table.py > gpurun_out/r4a/wgrad_table.jsonl 2>&1 || { tail -5 gpurun_out/r4a/wgrad_table.jsonl; exit 1; }
tail -1 gpurun_out/r4a/wgrad_table.jsonl
timeout -k 10 300 python tools/kvariant_time.py intree abtest/_C_wg_prio.so abtest/_C_wg_tk32ns4.so abtest/_C_wg_tk32ns3.so abtest/_C_wg_tk32ns4prio.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
