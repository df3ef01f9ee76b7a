#!/bin/bash
# Round 3: pipeline transport on a dedicated comm stream, IPC self-check + forced fallback,
# and the BASELINE config-2 bench layout (GPT-2 XL PP=4 interleaved, 32 microbatches of 4)
# rehearsed on ONE MI355X (4 ranks time-share the GPU) against PP=1 on the same microbatches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pp3
export SMP_LOG_LEVEL=warning
bash tools/gpu_ipc_stress.sh || exit 1
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pipeline_gpu.py \
  > gpurun_out/pp3/pytest.log 2>&1 || { tail -40 gpurun_out/pp3/pytest.log; exit 1; }
tail -3 gpurun_out/pp3/pytest.log
MB=${MB:-32}; MBS=${MBS:-4}; STEPS=${STEPS:-3}
timeout -k 10 400 python bench.py --layout dp --microbatches $MB --mbs $MBS --steps $STEPS --warmup 2 --tunableop off \
  > gpurun_out/pp3/pp1.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pp3/pp1.log || tail -20 gpurun_out/pp3/pp1.log
[ $rc -ne 0 ] && exit $rc
for CS in 1 0; do
SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_P2P_COMM_STREAM=$CS SMP_TIMELINE_FILE=gpurun_out/pp3/tl_cs${CS}_rank{rank}.json \
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 4 --steps $STEPS --warmup 2 --tunableop off \
  > gpurun_out/pp3/pp4_cs${CS}.log 2>&1
rc=$?; grep '"metric"' gpurun_out/pp3/pp4_cs${CS}.log || tail -30 gpurun_out/pp3/pp4_cs${CS}.log
[ $rc -ne 0 ] && exit $rc
done
exit 0
