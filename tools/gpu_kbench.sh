#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py -q -x -m gpu > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "attn pytest rc=$rc"; tail -3 gpurun_out/pytest_attn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_kernels.py > gpurun_out/kbench.json 2> gpurun_out/kbench.err
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench.json; tail -3 gpurun_out/kbench.err
exit $rc
