#!/bin/bash
# Same-box A/B of the headline bench over environment settings, alternating.
# usage: tools/gpu_ab_env.sh OUT ROUNDS "VAR=a [VAR2=b]" "VAR=c" ...   ("r5" = the round-5 package)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; n=$2; shift 2
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  j=0
  for v in "$@"; do
    j=$((j + 1))
    if [ "$v" = r5 ]; then
      (cd abtest/r5 && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "../../$out/b${j}_$i.log" 2>&1) || exit 1
    else
      env $v timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$out/b${j}_$i.log" 2>&1 || exit 1
    fi
    echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' "$out/b${j}_$i.log")"
  done
done
