#!/bin/bash
# PP engine overhead on one MI355X: N pipeline ranks share the GPU (IpcP2P transport,
# gloo object/process groups).  Total GPU work per step equals the PP=1 run, so the
# step-time difference is the pipeline runtime's cost (scheduling, transport, bubbles
# are absent since the stages time-share one device).
set -o pipefail
export SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_LOG_LEVEL=warning
mkdir -p gpurun_out
PP=${PP:-4}; MB=${MB:-8}; MBS=${MBS:-4}; STEPS=${STEPS:-5}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $PP --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus $PP --pp $PP --microbatches $MB --mbs $MBS --steps $STEPS --warmup 2 \
  ${EXTRA} > gpurun_out/pp_bench_pp${PP}.log 2>&1
rc=$?
grep '"metric"' gpurun_out/pp_bench_pp${PP}.log || tail -30 gpurun_out/pp_bench_pp${PP}.log
exit $rc
