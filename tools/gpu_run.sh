#!/bin/bash
# One parametrised GPU-box runner (replaces the per-session tools/gpu_r*.sh one-offs).
#
#   tools/gpu_run.sh OUT STEP [STEP ...]
#
# OUT is a directory name under gpurun_out/.  Steps run in order; each runs under its own
# time limit, and the script stops at the first step that crashes, aborts or times out (no
# retries).  Steps:
#   smoke                       __graft_entry__.smoke()
#   tests[=PATHS]               pytest -m gpu (default: tests/), per-test 300 s limit
#   bench[=ARGS]                python bench.py ARGS (default: --steps 10 --warmup 3)
#   trace[=ARGS]                rocprofv3 --kernel-trace of bench.py ARGS (default --steps 3
#                               --warmup 2) -> OUT/kernels.txt (tools/step_kernels.py table)
#   pmc=SCRIPT:C1,C2,...        rocprofv3 --kernel-trace --pmc C1 C2 ... -- python3 SCRIPT
#                               (one counter pass; csv under OUT/pmc_<n>/)
#   py=SCRIPT[:ARGS]            python3 SCRIPT ARGS (kernel benchmarks under tools/)
# Environment variables are passed through (e.g. SMP_* switches for A/B runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
( while sleep 50; do echo "heartbeat $(date +%T)" >> "$OUT/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT

stop_if_fatal() {  # rc label
  case $1 in
    0) return 0 ;;
    1) [ "$2" = tests ] && return 0 ;;  # pytest: some tests failed -- report, keep going
  esac
  echo "step $2 failed rc=$1: stopping"
  exit "$1"
}

npmc=0
for step in "$@"; do
  name=${step%%=*}
  arg=
  [ "$step" != "$name" ] && arg=${step#*=}
  case $name in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -1 "$OUT/smoke.log"; stop_if_fatal $rc smoke ;;
    tests)
      timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread ${arg:-tests/} \
        > "$OUT/pytest.log" 2>&1
      rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/pytest.log" | tail -15; stop_if_fatal $rc tests ;;
    bench)
      timeout -k 10 600 python bench.py ${arg:---steps 10 --warmup 3} > "$OUT/bench.log" 2>&1
      rc=$?; grep '"metric"' "$OUT/bench.log" || tail -20 "$OUT/bench.log"; stop_if_fatal $rc bench ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT/trace" -o t -- python3 bench.py ${arg:---steps 3 --warmup 2} \
        > "$OUT/trace.log" 2>&1
      rc=$?; stop_if_fatal $rc trace
      f=$(find "$OUT/trace" -name "*.db" | head -1)
      python3 tools/step_kernels.py "$f" > "$OUT/kernels.txt" && head -40 "$OUT/kernels.txt"
      rm -f "$f" ;;
    pmc)
      npmc=$((npmc + 1))
      script=${arg%%:*}
      counters=${arg#*:}
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${counters//,/ } -d "$OUT/pmc_$npmc" -o run \
        --output-format csv -- python3 "$script" > "$OUT/pmc_$npmc.log" 2>&1
      rc=$?; echo "pmc pass $npmc ($counters) rc=$rc"; stop_if_fatal $rc pmc ;;
    py)
      script=${arg%%:*}
      pargs=
      [ "$arg" != "$script" ] && pargs=${arg#*:}
      base=$(basename "$script" .py)
      timeout -k 10 600 python3 "$script" $pargs > "$OUT/$base.log" 2>&1
      rc=$?; tail -25 "$OUT/$base.log"; stop_if_fatal $rc py ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
done
exit 0
