#!/bin/bash
# Long-sequence GPT-2 XL on one MI355X (dropout 0.1): seq 8192 mbs 4 (keep bits 839 MB per
# layer: stored, below the 1 GB budget) and seq 16384 mbs 2 (1.68 GB per layer: above the
# budget, so the backward regenerates the keep bits from the hash).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5ls
timeout -k 10 400 python bench.py --seq 8192 --mbs 4 --steps 4 --warmup 2 > gpurun_out/r5ls/s8192.log 2>&1 || { tail -20 gpurun_out/r5ls/s8192.log; exit 1; }
grep '"metric"' gpurun_out/r5ls/s8192.log
timeout -k 10 500 python bench.py --seq 16384 --mbs 2 --steps 4 --warmup 2 > gpurun_out/r5ls/s16384.log 2>&1 || { tail -20 gpurun_out/r5ls/s16384.log; exit 1; }
grep '"metric"' gpurun_out/r5ls/s16384.log
