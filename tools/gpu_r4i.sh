#!/bin/bash
# Round 4: attention variant A/B (abtest/_C_<tag>.so) vs in-tree, per-kernel traces, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
for b in intree ${VARIANTS:-prio} intree ${VARIANTS:-prio}; do
  so=""; [ $b != intree ] && so=abtest/_C_$b.so
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r4i/p_$b -o r -- python3 tools/attn_time.py $so \
    > gpurun_out/r4i/$b.log 2>&1 || { tail -5 gpurun_out/r4i/$b.log; exit 1; }
  echo "== $b"; grep "fwd_" gpurun_out/r4i/$b.log | tail -2
  db=$(find gpurun_out/r4i/p_$b -name "*.db" | head -1)
  python3 tools/prof_db_summary.py "$db" 9 | grep -i "bwd"
  rm -rf gpurun_out/r4i/p_$b
done
