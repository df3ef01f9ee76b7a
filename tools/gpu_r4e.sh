#!/bin/bash
# Round 4: attention compile-time variants (abtest/_C_<tag>.so from tools/build_kvariant.sh)
# against the in-tree build and the round-3 build: tools/attn_time.py under a kernel trace,
# one process per build, per-kernel means from the rocpd database.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py -k "bench_shape or gpt2xl_width" > gpurun_out/r4e/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4e/pytest.log | head -20; [ $rc -le 1 ] || exit $rc
for b in intree base scalar bwscalar novpre fw3 intree; do
  so=""; [ $b != intree ] && so=abtest/_C_$b.so
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r4e/p_$b -o r -- python3 tools/attn_time.py $so \
    > gpurun_out/r4e/$b.log 2>&1 || { tail -5 gpurun_out/r4e/$b.log; exit 1; }
  echo "== $b"; grep "fwd_" gpurun_out/r4e/$b.log | tail -2
  db=$(find gpurun_out/r4e/p_$b -name "*.db" | head -1)
  python3 tools/prof_db_summary.py "$db" 9
  rm -rf gpurun_out/r4e/p_$b
done
