#!/bin/bash
# Full-size GPT-J 6B (28 x h4096, head dim 256, RoPE 64, parallel attn/MLP) training step on ONE
# MI355X: bf16 + fp32 master + AdamW, seq 2048, synthetic data.  One bench per micro-batch size.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mbs in ${MBS_LIST:-4 8}; do
  timeout -k 10 420 python bench.py --model gptj-6b --mbs $mbs --steps 5 --warmup 2 --tunableop ${TUNE:-off} \
    > gpurun_out/gptj_mbs$mbs.log 2>&1
  rc=$?; echo "gptj mbs $mbs rc=$rc"; grep "\"metric\"" gpurun_out/gptj_mbs$mbs.log | tail -1
  [ $rc -ne 0 ] && { grep -v INFO gpurun_out/gptj_mbs$mbs.log | tail -5; exit $rc; }
done
exit 0
