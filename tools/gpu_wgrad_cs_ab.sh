set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6cs; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wgrad_gpu.py > $out/tests.log 2>&1; rc=$?
tail -1 $out/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $out/tests.log | head; exit $rc; }
for i in 1 2; do
  for v in default idle; do
    for m in gptj_tp4 neox_pp2tp4; do
      SMP_WGRAD_PP_CS=$v timeout -k 10 300 python tools/shard_bench.py $m --mbs 8 --steps 5 --warmup 3 > $out/${m}_${v}_$i.log 2>&1 || exit 1
      echo "$m $v $i $(grep -o '"ms_per_step": [0-9.]*' $out/${m}_${v}_$i.log)"
    done
  done
done
