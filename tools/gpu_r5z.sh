#!/bin/bash
# A/B of the attention dropout element hash (SMPK_HASH_AB 0 lowbias32 / 1 two 24-bit
# multiplies / 2 one 32-bit + one 24-bit multiply): forward + backward times at GPT-2 XL shape.
set -o pipefail
mkdir -p gpurun_out/r5z
for rep in 1 2; do
  for v in h0 h1 h2; do
    timeout -k 10 120 python -u tools/attn_time.py abtest/_C_$v.so >> gpurun_out/r5z/ab.log 2>&1 || exit 1
  done
done
