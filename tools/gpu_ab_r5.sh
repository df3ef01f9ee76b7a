#!/bin/bash
# Same-box A/B of the headline bench: the round-5 package (abtest/r5, built from 8215c3a) against
# the working tree, alternating.  usage: tools/gpu_ab_r5.sh OUT [rounds]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; n=${2:-2}
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  (cd abtest/r5 && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "../../$out/r5_$i.log" 2>&1) || exit 1
  echo "r5   $(grep -o '"ms_per_step": [0-9.]*' "$out/r5_$i.log")"
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$out/new_$i.log" 2>&1 || exit 1
  echo "new  $(grep -o '"ms_per_step": [0-9.]*' "$out/new_$i.log")"
done
