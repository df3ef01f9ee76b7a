#!/bin/bash
# PP=4 one-GPU hang triage: in-flight microbatch cap 2 vs default, IPC vs host transport,
# 8 GPT-2 XL layers, 8 microbatches of 4; a 100 s step watchdog dumps the stacks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pph
export SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo SMP_STEP_TIMEOUT_S=100 SMP_LOG_LEVEL=warning
run() {  # tag layers mbs env...
  local tag=$1 L=$2 M=$3; shift 3
  env "$@" timeout -k 10 260 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29515 bench.py --gpus 4 --layers $L --mbs $M --microbatches 8 --steps 1 --warmup 1 --tunableop off \
    > gpurun_out/pph/$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc"; grep '"metric"' gpurun_out/pph/$tag.log | cut -c1-200
  grep -h "watchdog\|RuntimeError" gpurun_out/pph/$tag.log | head -4
  return 0
}
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_pipeline_gpu.py::test_ipc_pull_from_multi_gb_segment" > gpurun_out/pph/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|rep |OK" gpurun_out/pph/pytest.log | head; [ $rc -eq 0 ] || exit $rc
export SMP_STEP_TIMEOUT_S=120 SMP_ABORT_GRACE_S=100
run L8_mbs16_staged 8 16 SMP_P2P=ipc SMP_BENCH_ACTIVE_MB=2
grep -h "state:" gpurun_out/pph/L8_mbs16_staged.log | cut -c1-600
grep -q '"metric"' gpurun_out/pph/L8_mbs16_staged.log || exit 1
run L48_mbs16_staged 48 16 SMP_P2P=ipc SMP_BENCH_ACTIVE_MB=2
grep -o '"attention_calls": {[^}]*}' gpurun_out/pph/L48_mbs16_staged.log
