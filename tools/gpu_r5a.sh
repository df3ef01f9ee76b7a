#!/bin/bash
# Round 5: ping-pong weight-gradient kernel -- numerics, then the in-process A/B table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py \
  > gpurun_out/r5a/tests.log 2>&1 || { tail -40 gpurun_out/r5a/tests.log; exit 1; }
tail -1 gpurun_out/r5a/tests.log
timeout -k 10 400 python tools/wgrad_pp_ab.py > gpurun_out/r5a/ab.jsonl 2> gpurun_out/r5a/ab.err \
  || { tail -20 gpurun_out/r5a/ab.err; exit 1; }
cut -c1-200 gpurun_out/r5a/ab.jsonl
