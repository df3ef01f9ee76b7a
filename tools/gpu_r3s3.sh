#!/bin/bash
# Session-3 GPU call: weight-gradient tests + in-step fused-bias traces (tools/gpu_dbias_trace.sh),
# then hardware counters of the fc1 weight-gradient kernel vs the library GEMM.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_dbias_trace.sh || exit $?
export WG_N=${WG_N:-6400} WG_K=${WG_K:-1600} WG_SPLITS=${WG_SPLITS:-4}
bash tools/gpu_pmc_wgrad.sh || exit $?
python3 tools/pmc_summary.py gpurun_out/pmcw/*/ > gpurun_out/pmcw/summary.md 2>&1
cat gpurun_out/pmcw/summary.md | cut -c1-400
