#!/bin/bash
# Same-box A/B of the headline bench: the round-5 package (abtest/r5, built from 8215c3a) against
# the working tree, alternating; then (TRACE=1) a kernel trace of the working tree's step.
# usage: tools/gpu_ab_r5.sh OUT [rounds]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; n=${2:-2}
mkdir -p "$out"
if [ -n "$ATTN" ]; then timeout -k 10 300 python tools/attn_time.py > "$out/attn_time.log" 2>&1 || exit 1; grep in-tree "$out/attn_time.log"; fi
for i in $(seq 1 "$n"); do
  (cd abtest/r5 && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "../../$out/r5_$i.log" 2>&1) || exit 1
  echo "r5   $(grep -o '"ms_per_step": [0-9.]*' "$out/r5_$i.log")"
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$out/new_$i.log" 2>&1 || exit 1
  echo "new  $(grep -o '"ms_per_step": [0-9.]*' "$out/new_$i.log")"
done
if [ -n "$TRACE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace -d "$out/trace" -o t -- python3 bench.py --steps 3 --warmup 2 > "$out/trace.log" 2>&1 || exit 1
  f=$(find "$out/trace" -name "*.db" | head -1)
  python3 tools/step_kernels.py "$f" > "$out/kernels.txt" && head -40 "$out/kernels.txt"
  rm -f "$f"
fi
