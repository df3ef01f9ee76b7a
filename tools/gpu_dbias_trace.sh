#!/bin/bash
# In-step kernel traces with a switch off / on (same box; default SMP_WGRAD_DBIAS, the fused
# bias gradient; DBT_VAR names another): per-kernel steady-state times.  Runs the weight-gradient
# GPU tests first (the fused column sums are checked there against fp32 references).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dbt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py \
  > gpurun_out/dbt/tests.log 2>&1 || { tail -30 gpurun_out/dbt/tests.log; exit 1; }
tail -2 gpurun_out/dbt/tests.log
VAR=${DBT_VAR:-SMP_WGRAD_DBIAS}
for v in ${DBT_VARIANTS:-0 1}; do
  rm -rf gpurun_out/dbt/k$v
  env $VAR=$v timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/dbt/k$v -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 > gpurun_out/dbt/b$v.log 2>&1 || exit $?
  echo "$VAR=$v $(grep '"metric"' gpurun_out/dbt/b$v.log | cut -c1-160)"
  python3 tools/step_kernels.py $(find gpurun_out/dbt/k$v -name '*kernel_trace.csv') > gpurun_out/dbt/t$v.txt
  sed -n '1,24p' gpurun_out/dbt/t$v.txt
done
