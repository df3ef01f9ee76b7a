"""Attention fwd+bwd only (GPT-2 XL shape), for rocprofv3 counter runs."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops.attention import _FlashAttentionPacked  # noqa: E402

b, s, h, d = int(os.environ.get("B", 8)), int(os.environ.get("S", 2048)), int(os.environ.get("H", 25)), \
    int(os.environ.get("D", 64))
qkv = torch.randn(b, s, 3, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
p = float(os.environ.get("P", "0.0"))  # attention dropout (the bench runs 0.1)
for _ in range(int(os.environ.get("ITERS", 3))):
    o = _FlashAttentionPacked.apply(qkv, 1.0 / math.sqrt(d), True, 0, None, p)
    o.backward(torch.randn_like(o))
torch.cuda.synchronize()
print("done")
