#!/bin/bash
# Round 5: which PC-sampling configurations rocprofv3 offers on this box (read-only listing).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r5r/list.txt 2>&1
echo "rc=$?"
grep -i -n -A12 "pc.sampl\|PC_SAMPL\|stochastic\|host_trap" gpurun_out/r5r/list.txt | head -60
