#!/bin/bash
# Round 4: dQ keep bits one tile ahead -- attention + dropout GPU tests on the in-tree build,
# smoke, then the default bench once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_dropout_gpu.py tests/test_attention_chunking.py > gpurun_out/r4n/tests.log 2>&1 \
  || { tail -30 gpurun_out/r4n/tests.log; exit 1; }
tail -1 gpurun_out/r4n/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4n/smoke.log 2>&1 \
  || { tail -20 gpurun_out/r4n/smoke.log; exit 1; }
tail -1 gpurun_out/r4n/smoke.log
timeout -k 10 120 python tools/attn_time.py 2>&1 | grep "drop" || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r4n/bench.log 2>&1 || { tail -20 gpurun_out/r4n/bench.log; exit 1; }
grep '"metric"' gpurun_out/r4n/bench.log | cut -c1-240
