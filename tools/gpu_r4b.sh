#!/bin/bash
# Round 4, second GPU pass: optimizer diagnosis, the full kernel GPU test files (no -x: every
# failure listed; a crash / timeout still stops the script), attention A/B vs the round-3
# build, a short bench, the wgrad table and the wgrad compile-time variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4b
timeout -k 10 100 python tools/opt_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_dropout_gpu.py tests/test_optimizers_gpu.py tests/test_oneshot_gpu.py tests/test_wgrad_gpu.py \
  tests/test_kernels_gpu.py > gpurun_out/r4b/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r4b/pytest.log | tail -15
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/attn_time.py abtest/_C_base.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
  timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
done
timeout -k 10 300 python bench.py --steps 6 --warmup 3 > gpurun_out/r4b/bench.log 2>&1 || { tail -20 gpurun_out/r4b/bench.log; exit 1; }
tail -1 gpurun_out/r4b/bench.log
timeout -k 10 300 python tools/wgrad_table.py > gpurun_out/r4b/wgrad_table.jsonl 2>&1 || { tail -5 gpurun_out/r4b/wgrad_table.jsonl; exit 1; }
tail -1 gpurun_out/r4b/wgrad_table.jsonl
timeout -k 10 300 python tools/kvariant_time.py intree abtest/_C_wg_prio.so abtest/_C_wg_tk32ns4.so abtest/_C_wg_tk32ns3.so abtest/_C_wg_tk32ns4prio.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
