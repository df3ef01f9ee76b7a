#!/bin/bash
# Same-box bench A/B over several environment variants (AB_VARIANTS: ';'-separated lists of
# VAR=value assignments, "-" for the defaults), ROUNDS rounds, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
IFS=';' read -ra VS <<< "${AB_VARIANTS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 400 python bench.py --steps ${STEPS:-8} --warmup 3 $BENCH_ARGS > gpurun_out/abm/v${i}_r$r.log 2>&1
    rc=$?; echo -n "[$v] rc=$rc "
    [ $rc -ne 0 ] && { tail -5 gpurun_out/abm/v${i}_r$r.log; exit $rc; }
    grep '"metric"' gpurun_out/abm/v${i}_r$r.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], 'ms/step', r['value'], 'samples/s')"
    i=$((i+1))
  done
done
exit 0
