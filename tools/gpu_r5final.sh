#!/bin/bash
# Round 5 final check 2: the whole GPU test suite, the default 1-GPU bench, and its step kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5final
( while sleep 50; do echo "heartbeat $(date +%T)" >> gpurun_out/r5final/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final/smoke.log 2>&1 || { tail -20 gpurun_out/r5final/smoke.log; exit 1; }
tail -1 gpurun_out/r5final/smoke.log
timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/ > gpurun_out/r5final/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r5final/pytest.log | tail -12; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5final/bench.log 2>&1 || { tail -20 gpurun_out/r5final/bench.log; exit 1; }
grep '"metric"' gpurun_out/r5final/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5final/trace_bench -o t -- python3 bench.py --steps 3 --warmup 2 \
  > gpurun_out/r5final/trace_bench.log 2>&1 || { tail -20 gpurun_out/r5final/trace_bench.log; exit 1; }
f=$(find gpurun_out/r5final/trace_bench -name "*.db" | head -1)
python3 tools/step_kernels.py "$f" > gpurun_out/r5final/kernels_bench.txt && head -32 gpurun_out/r5final/kernels_bench.txt
rm -f "$f"
