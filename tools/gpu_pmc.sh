#!/bin/bash
# Hardware counters for the attention kernels (kernel-trace + pmc only; no sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/$tag -o run --output-format csv -- python3 tools/attn_only.py > gpurun_out/pmc/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
done
exit 0
