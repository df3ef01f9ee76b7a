#!/bin/bash
# Round 4: parallel-attention residual fusion A/B on one box (SMP_FUSE_PARALLEL_RESIDUAL=0/1),
# alternating, plus one kernel trace of each setting for the GPT-J shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
for s in gptj_tp4 neox_pp2tp4; do
  for f in 0 1 0 1; do
    SMP_FUSE_PARALLEL_RESIDUAL=$f timeout -k 10 300 python -u tools/shard_bench.py $s --mbs 8 --steps 5 --warmup 3 \
      > gpurun_out/r4k/$s.$f.log 2>&1 || { tail -20 gpurun_out/r4k/$s.$f.log; exit 1; }
    echo "$s fuse=$f $(grep SHARD gpurun_out/r4k/$s.$f.log | python3 -c 'import sys,json; r=json.loads(sys.stdin.read()[6:]); print(r["ms_per_step"], r["peak_mem_gb"])')"
  done
done
for f in 0 1; do
  export SMP_FUSE_PARALLEL_RESIDUAL=$f
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4k/p$f -o r -- python3 tools/shard_bench.py gptj_tp4 --mbs 8 --steps 3 --warmup 2 \
    > gpurun_out/r4k/prof$f.log 2>&1 || { tail -20 gpurun_out/r4k/prof$f.log; exit 1; }
  db=$(find gpurun_out/r4k/p$f -name "*.db" | head -1)
  python3 tools/prof_db_summary.py "$db" 25 > gpurun_out/r4k/kern$f.txt
  rm -rf gpurun_out/r4k/p$f
done
timeout -k 10 600 python3 tools/kvariant_time.py intree abtest/_C_w4.so > gpurun_out/r4k/wgrad_w4.log 2>&1 \
  || { tail -20 gpurun_out/r4k/wgrad_w4.log; exit 1; }
cat gpurun_out/r4k/wgrad_w4.log
