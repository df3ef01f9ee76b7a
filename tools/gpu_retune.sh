#!/bin/bash
# Re-tune the bench's GEMM selections (TunableOp, rotating operand buffers so picks reflect
# HBM-cold operands as in the step) into OUT/new.csv, then same-box A/B of the committed file vs
# the new one, alternating.  usage: tools/gpu_retune.sh OUT [ROTATING_MB]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; rot=${2:-1024}
mkdir -p "$out"
old=configs/tunableop/gpt2-xl_mbs32_s2048_pp1_tp1.csv
SMP_TUNABLEOP_FILE=$out/new.csv SMP_TUNABLEOP_ROTATING_MB=$rot timeout -k 10 1000 python bench.py --tunableop tune \
  --steps 2 --warmup 2 > "$out/tune.log" 2>&1 || { tail -20 "$out/tune.log"; exit 1; }
echo "tuned: $(grep -c Tunable "$out/new.csv") GEMM entries"
for i in 1 2; do
  for f in "$old" "$out/new.csv"; do
    SMP_TUNABLEOP_FILE=$f timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$out/b_$(basename $f)_$i.log" 2>&1 || exit 1
    echo "[$f] $(grep -o '"ms_per_step": [0-9.]*' "$out/b_$(basename $f)_$i.log")"
  done
done
