#!/bin/bash
# Config-2 rehearsal on ONE GPU at mbs 8 with fewer in-flight microbatches (4 ranks x 66 GB at
# the default pp + 2 = 6 oversubscribe one 288 GB GPU), and at mbs 4 (the round's earlier
# rehearsal shape), to separate memory oversubscription from pipeline cost.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp SMP_LOG_LEVEL=warning
mkdir -p gpurun_out/ppm
for v in "8 2" "4 6"; do
  set -- $v
  SMP_BENCH_ACTIVE_MB=$2 SMP_DEVICE_INDEX=0 SMP_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --mbs $1 --steps 2 --warmup 1 \
    > gpurun_out/ppm/pp4_mbs$1_a$2.log 2>&1
  rc=$?; echo "mbs=$1 active=$2 rc=$rc $(grep '"metric"' gpurun_out/ppm/pp4_mbs$1_a$2.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"], r["final_loss"], r["peak_mem_gb"], r["config"]["gemm_selection"])')"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ppm/pp4_mbs$1_a$2.log; exit $rc; }
done
exit 0
