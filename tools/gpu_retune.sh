#!/bin/bash
# Re-tune the bench's GEMM selections (TunableOp, rotating buffers over the 256 MB MALL) into a
# scratch file, then A/B the bench with the committed file vs the fresh one on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tune
( while sleep 50; do echo "heartbeat $(date +%T)" >> gpurun_out/tune/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
SMP_TUNABLEOP_FILE=gpurun_out/tune/gpt2-xl_mbs32_s2048_pp1_tp1.csv SMP_TUNABLEOP_ROTATING_MB=512 \
  timeout -k 10 1500 python bench.py --tunableop tune --steps 2 --warmup 2 > gpurun_out/tune/tune.log 2>&1 \
  || { tail -20 gpurun_out/tune/tune.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/committed /"
  SMP_TUNABLEOP_FILE=gpurun_out/tune/gpt2-xl_mbs32_s2048_pp1_tp1.csv timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 \
    | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/retuned /"
done
