#!/bin/bash
# Round 4: wide-row LayerNorm kernels + the measured attention defaults (scalar forward
# exponent code, no V prefetch): kernel GPU tests, attention timing, the NeoX shard (LN at
# 6144) with its kernel table, the PP=4 one-GPU rehearsal (heartbeat: the 4-rank run prints
# nothing for minutes) and the bench step kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/r4f
( while sleep 50; do echo "heartbeat $(date +%T)" >> gpurun_out/r4f/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_attention_gpu.py tests/test_dropout_gpu.py "tests/test_pipeline_gpu.py::test_pp2_ipc_bounded_mappings" \
  "tests/test_pipeline_gpu.py::test_pp2_ipc_matches_unpartitioned" > gpurun_out/r4f/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r4f/pytest.log | tail -12; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
S=neox_pp2tp4
timeout -k 10 400 python -u tools/shard_bench.py $S --mbs 8 --steps 5 --warmup 3 > gpurun_out/r4f/$S.log 2>&1 \
  || { tail -20 gpurun_out/r4f/$S.log; exit 1; }
grep '^SHARD' gpurun_out/r4f/$S.log
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r4f/trace_$S -o t -- python3 tools/shard_bench.py $S --mbs 8 \
  --steps 2 --warmup 2 > gpurun_out/r4f/trace_$S.log 2>&1 || { tail -20 gpurun_out/r4f/trace_$S.log; exit 1; }
f=$(find gpurun_out/r4f/trace_$S -name "*.db" | head -1)
python3 tools/step_kernels.py "$f" > gpurun_out/r4f/kernels_$S.txt && head -16 gpurun_out/r4f/kernels_$S.txt
rm -f "$f"
SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_BENCH_ACTIVE_MB=2 \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 4 --microbatches 8 --steps 2 --warmup 1 --tunableop off \
  > gpurun_out/r4f/pp4.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r4f/pp4.log || tail -30 gpurun_out/r4f/pp4.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r4f/trace_bench -o t -- python3 bench.py --steps 3 --warmup 2 \
  > gpurun_out/r4f/trace_bench.log 2>&1 || { tail -20 gpurun_out/r4f/trace_bench.log; exit 1; }
grep '"metric"' gpurun_out/r4f/trace_bench.log
f=$(find gpurun_out/r4f/trace_bench -name "*.db" | head -1)
python3 tools/step_kernels.py "$f" > gpurun_out/r4f/kernels_bench.txt && head -30 gpurun_out/r4f/kernels_bench.txt
rm -f "$f"
