#!/bin/bash
# Round 5: partial-sum reduce kernels with their loads in flight together (LN dgamma/dbeta stage 2,
# bias-GeLU dbias stage 2, weight-gradient bias column sums) -- kernel tests, then the fused-op
# timing pass and the bench step table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_wgrad_gpu.py tests/test_dropout_gpu.py > gpurun_out/r5v/tests.log 2>&1 \
  || { grep -E "Error|assert|FAILED" gpurun_out/r5v/tests.log | head -20; tail -5 gpurun_out/r5v/tests.log; exit 1; }
tail -1 gpurun_out/r5v/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5v/trace_bench -o t -- python3 bench.py --steps 3 --warmup 2 \
  > gpurun_out/r5v/trace_bench.log 2>&1 || { tail -20 gpurun_out/r5v/trace_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5v/trace_bench.log
f=$(find gpurun_out/r5v/trace_bench -name "*.db" | head -1)
python3 tools/step_kernels.py "$f" > gpurun_out/r5v/kernels_bench.txt && grep -E "step |reduce|col_sum" gpurun_out/r5v/kernels_bench.txt
rm -f "$f"
