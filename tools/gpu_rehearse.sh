#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks share cuda:0 over gloo (RCCL needs distinct
# GPUs).  Exercises bench.py's distributed flow (DP reducer with device tensors, barriers,
# max-over-ranks timing, rank-0 JSON) -- not a performance measurement.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_DIST_BACKEND=gloo SMP_DEVICE_INDEX=0
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --model gpt2-small --mbs 2 --seq 512 --tunableop off \
  > gpurun_out/rehearse_dp2.log 2>&1
rc=$?; echo "dp2 rc=$rc"; grep -v INFO gpurun_out/rehearse_dp2.log | grep metric | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 1 --model gpt2-small --mbs 2 --seq 512 --tp 2 \
  --tunableop off > gpurun_out/rehearse_tp2.log 2>&1
rc=$?; echo "tp2 rc=$rc"; grep -v INFO gpurun_out/rehearse_tp2.log | grep metric | tail -2
exit $rc
