#!/bin/bash
# GeLU row-streaming A/B + its numerics tests, then a same-box bench A/B (SMP_GELU_ROWS=0 / 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gelu or col_sum" --timeout 120 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gelu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/gelu_ab.py > gpurun_out/gelu_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/gelu_ab.log
[ $rc -ne 0 ] && exit $rc
for m in 0 1 0 1; do
  SMP_GELU_ROWS=$m timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_gelu_$m.log 2>&1
  rc=$?; echo "bench rows=$m rc=$rc"; grep metric gpurun_out/bench_gelu_$m.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['value'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
