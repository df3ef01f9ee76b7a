#!/bin/bash
# BASELINE config 2 shape (GPT-2 XL, PP=4 interleaved, 8 microbatches of 4) on ONE MI355X:
# the 4 pipeline ranks time-share the GPU (IpcP2P transport, gloo object groups), so the
# step-time gap to the PP=1 run of the same microbatches is the pipeline runtime's own
# cost.  Writes per-rank Chrome-trace timelines (SMP_TIMELINE_FILE) of the PP=4 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export SMP_DEVICE_INDEX=0 SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/pptrace
MB=${MB:-8}; MBS=${MBS:-4}; STEPS=${STEPS:-5}
timeout -k 10 300 python bench.py --microbatches $MB --mbs $MBS --steps $STEPS --warmup 2 --tunableop off > gpurun_out/pptrace/pp1.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pptrace/pp1.log || tail -20 gpurun_out/pptrace/pp1.log
[ $rc -ne 0 ] && exit $rc
SMP_DIST_BACKEND=gloo SMP_TIMELINE_FILE=gpurun_out/pptrace/timeline_rank{rank}.json \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 4 --pp 4 --microbatches $MB --mbs $MBS --steps $STEPS --warmup 2 --tunableop off \
  > gpurun_out/pptrace/pp4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pptrace/pp4.log || tail -30 gpurun_out/pptrace/pp4.log
exit $rc
