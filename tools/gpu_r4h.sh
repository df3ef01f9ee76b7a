#!/bin/bash
# Round 4: dropout keep bits from a separate kernel (in-tree) vs hashed inside the forward
# (abtest/_C_inbits.so) vs round 3 (abtest/_C_base.so): attention GPU tests, per-kernel traces of
# tools/attn_time.py, then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_dropout_gpu.py > gpurun_out/r4h/pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r4h/pytest.log | head; tail -5 gpurun_out/r4h/pytest.log; exit 1; }
tail -1 gpurun_out/r4h/pytest.log
for b in intree inbits base intree; do
  so=""; [ $b != intree ] && so=abtest/_C_$b.so
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r4h/p_$b -o r -- python3 tools/attn_time.py $so \
    > gpurun_out/r4h/$b.log 2>&1 || { tail -5 gpurun_out/r4h/$b.log; exit 1; }
  echo "== $b"; grep "fwd_" gpurun_out/r4h/$b.log | tail -2
  db=$(find gpurun_out/r4h/p_$b -name "*.db" | head -1)
  python3 tools/prof_db_summary.py "$db" 11 | grep -i "attn\|bits"
  rm -rf gpurun_out/r4h/p_$b
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r4h/bench.log 2>&1 || { tail -20 gpurun_out/r4h/bench.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/r4h/bench.log
