#!/bin/bash
# Round 5: TunableOp entries for the padded LM head's GEMM shapes (the results file is seeded
# with the shipped one, so only missing shapes are tuned), then the bench with the new file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5y
cp configs/tunableop/gpt2-xl_mbs32_s2048_pp1_tp1.csv gpurun_out/r5y/tuned.csv
SMP_TUNABLEOP_FILE=gpurun_out/r5y/tuned.csv timeout -k 10 900 python bench.py --tunableop tune --steps 2 --warmup 3 \
  > gpurun_out/r5y/tune.log 2>&1 || { tail -20 gpurun_out/r5y/tune.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5y/tune.log
diff <(sort configs/tunableop/gpt2-xl_mbs32_s2048_pp1_tp1.csv) <(sort gpurun_out/r5y/tuned.csv) | head -20
for f in gpurun_out/r5y/tuned.csv configs/tunableop/gpt2-xl_mbs32_s2048_pp1_tp1.csv gpurun_out/r5y/tuned.csv configs/tunableop/gpt2-xl_mbs32_s2048_pp1_tp1.csv; do
  SMP_TUNABLEOP_FILE=$f timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r5y/b.log 2>&1 || { tail -20 gpurun_out/r5y/b.log; exit 1; }
  echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5y/b.log)"
done
