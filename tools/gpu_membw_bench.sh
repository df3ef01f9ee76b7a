#!/bin/bash
# HBM streaming variants (tools/membw/stream_variants), the in-tree memory-bound kernels
# (tools/membw_probe.py), then the default bench (wgrad 16x16x32 default).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/membw
timeout -k 10 120 ./tools/membw/stream_variants > gpurun_out/membw/stream.jsonl 2>&1 || { cat gpurun_out/membw/stream.jsonl; exit 1; }
cat gpurun_out/membw/stream.jsonl
timeout -k 10 120 python tools/membw_probe.py > gpurun_out/membw/probe.json 2>&1 || { tail gpurun_out/membw/probe.json; exit 1; }
grep -v amdgpu.ids gpurun_out/membw/probe.json | tr -d '\n '; echo
timeout -k 10 600 python bench.py > gpurun_out/membw/bench.log 2>&1 || { tail -20 gpurun_out/membw/bench.log; exit 1; }
grep '"metric"' gpurun_out/membw/bench.log | cut -c1-400
