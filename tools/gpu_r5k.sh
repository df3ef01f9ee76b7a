#!/bin/bash
# Round 5: BASELINE config-2 flow (GPT-2 XL PP=4 interleaved, micro-batch 16) rehearsed on ONE GPU
# -- 4 ranks time-share cuda:0, gloo process groups, IPC pipeline transport -- for 3 warmup + 4
# timed steps, so the record-and-replay scheduler (on by default for PP > 1 since this round;
# 5 recorded steps) replays the last two.  Flow check, not a performance measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/r5k
( while sleep 50; do echo "heartbeat $(date +%T)" >> gpurun_out/r5k/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_BENCH_ACTIVE_MB=2 SMP_STEP_TIMEOUT_S=300 \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29523 bench.py --gpus 4 --microbatches 8 --steps 4 --warmup 3 --tunableop off \
  > gpurun_out/r5k/pp4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r5k/pp4.log | cut -c1-900 || tail -30 gpurun_out/r5k/pp4.log
[ $rc -ne 0 ] && { tail -30 gpurun_out/r5k/pp4.log; exit $rc; }
grep -i "replay" gpurun_out/r5k/pp4.log | head -5
exit 0
