#!/bin/bash
# Round 5: ping-pong weight gradient with the whole next tile's LDS-DMA issued in phase 0 (impl 2)
# vs one half-tile per phase (impl 1): bitwise equality, then same-process A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 200 python tools/wgrad_impl_eq.py 2>&1 | grep -v amdgpu.ids || exit 1
WG_IMPLS=1,2 WG_SPLITS=4,5,7 timeout -k 10 400 python tools/wgrad_pp_ab.py 2>&1 | grep -v amdgpu.ids | python3 -c "
import json,sys
for l in sys.stdin:
    if not l.startswith('{'): print(l, end=''); continue
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.startswith('best')}, {k:v[0] for k,v in d['all_us_tflops'].items() if k!='library'})
"
