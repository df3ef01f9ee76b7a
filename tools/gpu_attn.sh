#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py -q -x -m gpu > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "attn pytest rc=$rc"; tail -25 gpurun_out/pytest_attn.log
exit $rc
