#!/bin/bash
# Pipelined-forward A/B: attention/dropout GPU tests (pipelined kernel is the default), then
# interleaved timings with SMP_ATTN_FWD_PIPE=0 (in-turn loop) and =1 on the GPT-2 XL shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pipeab
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_dropout_gpu.py \
  > gpurun_out/pipeab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pipeab/pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" gpurun_out/pipeab/pytest.log | head -80; exit $rc; }
for i in 1 2; do
  for P in 0 1; do
    SMP_ATTN_FWD_PIPE=$P timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" | sed "s/^/pipe=$P /" || exit 1
  done
done
