#!/bin/bash
# Round 5: ping-pong weight gradient with the next tile's B half 0 read in phase 3 (balanced
# 16/8/16/8 transposed reads per phase) vs reading it in phase 0 (impl 2) -- correctness, then
# same-process A/B at the GPT-2 XL shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py > gpurun_out/r5j/tests.log 2>&1 \
  || { tail -30 gpurun_out/r5j/tests.log; exit 1; }
tail -1 gpurun_out/r5j/tests.log
WG_IMPLS=1,2 WG_SPLITS=3,4,5,7 timeout -k 10 400 python tools/wgrad_pp_ab.py 2>&1 | grep -v amdgpu.ids | python3 -c "
import json,sys
for l in sys.stdin:
    if not l.startswith('{'): print(l, end=''); continue
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.startswith('best') or k=='library_us'}, {k:v[0] for k,v in d['all_us_tflops'].items()})
"
