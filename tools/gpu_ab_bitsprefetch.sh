#!/bin/bash
# same-box A/B of the keep-bits prefetch
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 tests/test_attention_gpu.py tests/test_dropout_gpu.py > gpurun_out/r6g/pytest.log 2>&1; tail -2 gpurun_out/r6g/pytest.log
for v in 1 0 1 0; do
  SMP_ATTN_BITS_PREFETCH=$v timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r6g/bench_$v.log 2>&1 || exit 1
  echo "prefetch=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6g/bench_$v.log)"
done
