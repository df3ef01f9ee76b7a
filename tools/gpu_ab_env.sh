#!/bin/bash
# Same-box bench A/B of one environment switch: AB_VAR=0 / 1 alternating, twice each.
# Usage: AB_VAR=SMP_WGRAD_AUTOTUNE [AB_A=0 AB_B=1] bash tools/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=${AB_A:-0}; B=${AB_B:-1}
for m in $A $B $A $B; do
  env "$AB_VAR=$m" timeout -k 10 400 python bench.py --steps 8 --warmup 3 $BENCH_ARGS > gpurun_out/ab_${AB_VAR}_$m.log 2>&1
  rc=$?; echo -n "$AB_VAR=$m rc=$rc "
  [ $rc -ne 0 ] && exit $rc
  grep '"metric"' gpurun_out/ab_${AB_VAR}_$m.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], 'ms/step', r['value'], 'samples/s')"
done
exit 0
