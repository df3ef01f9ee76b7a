#!/bin/bash
# Round 4: 16-B add3 -- numerics, GPT-J / NeoX width hybrid tests, GPT-J shard A/B and trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_hybrid_gpu.py -k "add3 or add_layernorm or gptj or neox" \
  > gpurun_out/r4l/tests.log 2>&1 || { tail -30 gpurun_out/r4l/tests.log; exit 1; }
tail -2 gpurun_out/r4l/tests.log
for f in 0 1 0 1; do
  SMP_FUSE_PARALLEL_RESIDUAL=$f timeout -k 10 300 python -u tools/shard_bench.py gptj_tp4 --mbs 8 --steps 5 --warmup 3 \
    > gpurun_out/r4l/gptj.$f.log 2>&1 || { tail -20 gpurun_out/r4l/gptj.$f.log; exit 1; }
  echo "gptj fuse=$f $(grep SHARD gpurun_out/r4l/gptj.$f.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"], r["peak_mem_gb"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4l/p -o r -- python3 tools/shard_bench.py gptj_tp4 --mbs 8 --steps 3 --warmup 2 \
  > gpurun_out/r4l/prof.log 2>&1 || { tail -20 gpurun_out/r4l/prof.log; exit 1; }
db=$(find gpurun_out/r4l/p -name "*.db" | head -1)
python3 tools/prof_db_summary.py "$db" 30 > gpurun_out/r4l/kern.txt
rm -rf gpurun_out/r4l/p
grep -i "add" gpurun_out/r4l/kern.txt
