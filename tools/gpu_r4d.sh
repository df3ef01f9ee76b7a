#!/bin/bash
# Round 4: BASELINE config 3 / 4 heaviest-rank shards (tools/shard_bench.py, timing run + a
# kernel-traced run each) and the config-2 PP=4 rehearsal on one GPU with 2 in-flight
# microbatches (attention_calls in the JSON: key-bias variant launches must be 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/r4d
for S in gptj_tp4 neox_pp2tp4; do
  timeout -k 10 400 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 > gpurun_out/r4d/$S.log 2>&1 \
    || { tail -20 gpurun_out/r4d/$S.log; exit 1; }
  grep '^SHARD' gpurun_out/r4d/$S.log
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r4d/trace_$S -o t -- python3 tools/shard_bench.py $S --mbs 8 \
    --steps 2 --warmup 2 > gpurun_out/r4d/trace_$S.log 2>&1 || { tail -20 gpurun_out/r4d/trace_$S.log; exit 1; }
  f=$(find gpurun_out/r4d/trace_$S -name "*.db" | head -1)
  python3 tools/step_kernels.py "$f" > gpurun_out/r4d/kernels_$S.txt && head -25 gpurun_out/r4d/kernels_$S.txt
  rm -f "$f"
done
SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_BENCH_ACTIVE_MB=2 \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 4 --microbatches 8 --steps 2 --warmup 2 --tunableop off \
  > gpurun_out/r4d/pp4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r4d/pp4.log || tail -30 gpurun_out/r4d/pp4.log
[ $rc -ne 0 ] && exit $rc
# the 1-GPU default bench step, kernel-traced (3 steps; the table is the last full step)
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r4d/trace_bench -o t -- python3 bench.py --steps 3 --warmup 2 \
  > gpurun_out/r4d/trace_bench.log 2>&1 || { tail -20 gpurun_out/r4d/trace_bench.log; exit 1; }
f=$(find gpurun_out/r4d/trace_bench -name "*.db" | head -1)
python3 tools/step_kernels.py "$f" > gpurun_out/r4d/kernels_bench.txt && head -30 gpurun_out/r4d/kernels_bench.txt
rm -f "$f"
