#!/bin/bash
# Config-2 bench layout at its new default (PP=4, 32 microbatches of 8) rehearsed on ONE
# MI355X (4 ranks time-share it) against PP=1 on the same microbatches: same final loss,
# memory headroom.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/pp8
timeout -k 10 500 python bench.py --layout dp --microbatches 32 --mbs 8 --steps 2 --warmup 1 > gpurun_out/pp8/pp1.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pp8/pp1.log | cut -c1-600 || tail -20 gpurun_out/pp8/pp1.log
[ $rc -ne 0 ] && exit $rc
SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 2 --warmup 1 > gpurun_out/pp8/pp4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pp8/pp4.log | cut -c1-700 || tail -30 gpurun_out/pp8/pp4.log
exit $rc
