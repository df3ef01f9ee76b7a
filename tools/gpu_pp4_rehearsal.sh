#!/bin/bash
# BASELINE config-2 flow (GPT-2 XL PP=4 interleaved, micro-batch 16) rehearsed on ONE GPU: 4 ranks
# time-share cuda:0 over gloo process groups with the IPC pipeline transport, 3 warmup + 4 timed
# steps, so the record-and-replay scheduler (bench.py marks the PP layout static_mode; 5 recorded
# steps) replays the last two.  A flow check of the multi-rank bench path, not a performance number.
# usage: tools/gpu_pp4_rehearsal.sh OUT [VAR=value ...]   (extra environment for the run, e.g.
# SMP_BENCH_STATIC=0 to keep the dynamic scheduler, SMP_BENCH_STEP_TIMES=1 for per-step times)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
out=gpurun_out/$1
shift
mkdir -p "$out"
# (model construction and partitioning of 4 GPT-2 XL ranks run minutes without output)
( while sleep 50; do echo "heartbeat $(date +%T)" >> "$out/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
env "$@" SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_BENCH_ACTIVE_MB=2 SMP_STEP_TIMEOUT_S=300 \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29523 bench.py --gpus 4 --microbatches 8 --steps 4 --warmup 3 --tunableop off > "$out/pp4.log" 2>&1
rc=$?
grep '"metric"' "$out/pp4.log" | cut -c1-1200 || tail -30 "$out/pp4.log"
[ $rc -ne 0 ] && { tail -30 "$out/pp4.log"; exit $rc; }
grep -i "frozen" "$out/pp4.log" | head -4
exit 0
