#!/bin/bash
# Round 4 final check: build is in-tree (no compile here); smoke(), the whole GPU suite, the
# default bench twice, and attention timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final
( while sleep 50; do echo "heartbeat $(date +%T)" >> gpurun_out/final/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 \
  || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/ > gpurun_out/final/pytest.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/final/pytest.log | tail -12; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/attn_time.py 2>&1 | grep -v "^\[\|amdgpu.ids" || exit 1
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/final/bench$i.log 2>&1 || { tail -20 gpurun_out/final/bench$i.log; exit 1; }
  grep '"metric"' gpurun_out/final/bench$i.log | cut -c1-260
done
