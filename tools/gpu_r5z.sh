#!/bin/bash
# A/B of attention builds in abtest/ (VARIANTS="tag1 tag2 ..."; default: the r5z dropout
# element-hash builds h0 h1 h2): forward + backward times at GPT-2 XL shape, two passes.
set -o pipefail
mkdir -p gpurun_out/${OUT:-r5z}
for rep in 1 2; do
  for v in ${VARIANTS:-h0 h1 h2}; do
    timeout -k 10 120 python -u tools/attn_time.py abtest/_C_$v.so >> gpurun_out/${OUT:-r5z}/ab.log 2>&1 || exit 1
  done
done
