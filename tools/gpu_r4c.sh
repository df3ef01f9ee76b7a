#!/bin/bash
# Round 4, third GPU pass: per-kernel attention traces (round-3 build vs in-tree), the wgrad
# compile-time variants, the config 3/4 width equivalence tests, the optimizer tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_dropout_gpu.py > gpurun_out/r4c/attn_tests.log 2>&1 || { tail -30 gpurun_out/r4c/attn_tests.log; exit 1; }
tail -1 gpurun_out/r4c/attn_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c/prof_base -o base -- python3 tools/attn_time.py abtest/_C_base.so > gpurun_out/r4c/prof_base.log 2>&1 || { tail -5 gpurun_out/r4c/prof_base.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c/prof_intree -o intree -- python3 tools/attn_time.py > gpurun_out/r4c/prof_intree.log 2>&1 || { tail -5 gpurun_out/r4c/prof_intree.log; exit 1; }
echo profiles done
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_optimizers_gpu.py \
  tests/test_hybrid_gpu.py -k "adam or lamb or novo or gptj or neox" > gpurun_out/r4c/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r4c/pytest.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/kvariant_time.py intree abtest/_C_wg_prio.so abtest/_C_wg_tk32ns4.so abtest/_C_wg_tk32ns3.so abtest/_C_wg_tk32ns4prio.so 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
