"""Attention backward at the GPT-2 XL bench shape (b 32, h 25, s 2048, d 64, causal, bf16):
the split kernels (dQ + dK/dV) vs the fused single kernel (+ its delta pre-kernel), dropout
0 and 0.1, interleaved rounds in one process; also checks the fused error word stays 0."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops import attention as A  # noqa: E402

b, s, h, d = (int(os.environ.get(k, v)) for k, v in (("AB", 32), ("AS", 2048), ("AH", 25), ("AD", 64)))
torch.manual_seed(0)
qkv = torch.randn(b, s, 3, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
err = torch.zeros(1, dtype=torch.int32, device="cuda")
res = {}
for p in (0.0, 0.1):
    o = A._FlashAttentionPacked.apply(qkv, 1.0 / math.sqrt(d), True, 0, None, p)
    arms = {}
    for fused in (False, True):
        def run(fused=fused):
            A.FUSED_BWD[0], A.FUSED_BWD_ERR[0] = fused, err
            qkv.grad = None
            o.backward(g, retain_graph=True)
        arms["fused" if fused else "split"] = run
    for fn in arms.values():
        fn()
    torch.cuda.synchronize()
    best = {}
    for _ in range(3):
        for name, fn in arms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            e1.synchronize()
            best[name] = min(best.get(name, 1e9), e0.elapsed_time(e1) / 5 * 1e3)
    res[f"p{p}"] = {k: round(v, 1) for k, v in best.items()}
print(json.dumps({"shape": [b, s, h, d], "bwd_us": res, "fused_err": int(err.item())}), flush=True)
