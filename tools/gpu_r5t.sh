#!/bin/bash
# Round 5: ping-pong weight-gradient latency / FIFO counters (fc1 dW 6400 x 1600, T 65536, s7):
# average VMEM and LDS instruction latency (INST_LEVEL accumulated by ACCUM_PREV_HIRES / INSTS)
# and the LDS / TA FIFO-full stall cycles.  kernel-trace + pmc only, one set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r5t
mkdir -p $out
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $out/$tag -o run --output-format csv -- python3 tools/wgrad_one.py > $out/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) tail -3 $out/$tag.log; exit $rc;; esac
}
export WG_N=6400 WG_K=1600 WG_SPLITS=7 WG_ITERS=3
run vmem SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES
run lds SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES
run fifo SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run coexec SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE
for t in vmem lds fifo coexec; do
  python3 - $out/$t/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); nd = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    k = "pp" if "wgrad_pp" in n else "lib" if "Cijk" in n else None
    if k:
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    print(sys.argv[1].split("/")[-2], k, {c: f"{x / len(nd[k]):.4g}" for c, x in v.items()})
PY
done
