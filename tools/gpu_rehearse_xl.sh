#!/bin/bash
# 2 ranks share cuda:0 over gloo: GPT-2 XL data parallel at mbs 8 (T = 16384 tokens per rank,
# so the weight-gradient autotune runs inside the DP backward next to the bucketed reducer).
# Flow check, not a performance measurement.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_DIST_BACKEND=gloo SMP_DEVICE_INDEX=0 SMP_WGRAD_LOG=1
mkdir -p gpurun_out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29621 bench.py --gpus 2 --steps 2 --warmup 1 --mbs 8 > gpurun_out/rehearse_xl_dp2.log 2>&1
rc=$?; echo "xl dp2 rc=$rc"; grep -v INFO gpurun_out/rehearse_xl_dp2.log | tail -12
exit $rc
