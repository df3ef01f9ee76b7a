#!/bin/bash
# the measured max-params ceiling of the config-5 rank layout -- embedding +
# 37 TP-sliced GPT-3 175B layers (33.8 B params: bf16 param + grad + fp32 master in HBM, AdamW
# moments in pinned host memory = 270 GB, under the 270 GiB per-command host cap), 3 steps.
# An HBM out-of-memory is a Python exception: then the 35-layer size (32.0 B) runs instead.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/maxp
( while sleep 50; do echo "heartbeat $(date +%T) $(free -g | awk '/Mem/{print $3}') GB used" >> gpurun_out/maxp/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
free -g | head -2
for L in 37 35; do
  SMP_OFFLOAD_OPTIMIZER_FIELDS=m,v SMP_LOG_LEVEL=warning timeout -k 10 900 \
    python -u tools/max_params.py shard --layers $L > gpurun_out/maxp/shard_L$L.log 2>&1
  rc=$?
  grep -v "^\[" gpurun_out/maxp/shard_L$L.log | tail -6
  [ $rc -eq 0 ] && exit 0
  grep -q "OutOfMemoryError\|out of memory" gpurun_out/maxp/shard_L$L.log || exit $rc
done
exit 1
