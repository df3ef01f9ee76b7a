#!/bin/bash
# Session-2 check: targeted GPU tests (weight gradient + fused bias, elementwise kernels,
# hybrid TP/PP feature matrix), the default bench, and a kernel profile of it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py \
  tests/test_kernels_gpu.py tests/test_tp_kernels_gpu.py tests/test_hybrid_gpu.py ${EXTRA_TESTS} > gpurun_out/s2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s2/pytest.log
[ $rc -ne 0 ] && { grep -B2 -A25 "Error\|FAILED\|assert" gpurun_out/s2/pytest.log | head -80; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/s2/bench.log 2>&1 || { tail -20 gpurun_out/s2/bench.log; exit 1; }
grep '"metric"' gpurun_out/s2/bench.log | cut -c1-300
[ "${PROF:-1}" = "0" ] && exit 0
rm -rf gpurun_out/s2/k
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/k -o run --output-format csv -- \
  python3 bench.py --steps 4 --warmup 2 > gpurun_out/s2/prof_bench.log 2>&1 || exit $?
f=$(find gpurun_out/s2/k -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 6 45 > gpurun_out/s2/summary.md
head -32 gpurun_out/s2/summary.md
