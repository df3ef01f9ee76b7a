#!/bin/bash
# Measure the per-shape GEMM winners for the headline bench (TunableOp) and re-bench with them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out configs/tunableop
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 1100 python bench.py --steps 4 --warmup 2 --tunableop tune $BENCH_ARGS > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; grep -v INFO gpurun_out/tune.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/tunableop && cp configs/tunableop/*.csv gpurun_out/tunableop/
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --tunableop use $BENCH_ARGS > gpurun_out/bench_tuned.log 2>&1
rc=$?; echo "bench tuned rc=$rc"; grep -v INFO gpurun_out/bench_tuned.log | tail -2
exit $rc
