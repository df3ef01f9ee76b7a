#!/bin/bash
# (1) host-boundness of one PP=4 stage's work on one GPU (12 layers, 32 microbatches of 4,
# PP=1): kernel-busy fraction of the step; (2) same-box A/B of the padded LM head at mbs 32.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/host
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/host/k -o run --output-format csv -- python3 bench.py --layout dp \
  --mbs 4 --microbatches 32 --layers 12 --steps 3 --warmup 2 > gpurun_out/host/bench.log 2>&1 || { tail gpurun_out/host/bench.log; exit 1; }
grep '"metric"' gpurun_out/host/bench.log | cut -c1-200
python3 tools/busy_fraction.py $(find gpurun_out/host/k -name "*kernel_trace.csv") || exit 1
AB_VARIANTS="SMP_PADDED_LM_HEAD=0;SMP_PADDED_LM_HEAD=1" ROUNDS=2 bash tools/gpu_ab_multi.sh
