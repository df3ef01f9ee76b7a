"""Time the wide-row LayerNorm backward of one `_C` build (path in argv[1], default: in-tree)
at the config 4 / 5 widths (T = 16384 rows; cols 6144 / 8192 / 12288, bf16), with and without
the residual-gradient input -- the A/B harness of the two-row register ring (tools/gpu_r5ln.sh)."""
import importlib.machinery
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = sys.argv[1] if len(sys.argv) > 1 else None
if path:
    loader = importlib.machinery.ExtensionFileLoader("_C", path)
    C = importlib.util.module_from_spec(importlib.util.spec_from_loader("_C", loader))
    loader.exec_module(C)
else:
    sys.path.insert(0, ROOT)
    from smdistributed_modelparallel_amd.ops._ext import ext
    C = ext()


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


res = {}
for cols in (6144, 8192, 12288):
    x = torch.randn(16384, cols, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(cols, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(cols, device="cuda", dtype=torch.bfloat16)
    y, mean, rstd = C.layernorm_fwd(x, None, w, b, 1e-5)
    dy = torch.randn_like(y)
    dr = torch.randn_like(y)
    res[f"{cols}"] = round(t(lambda: C.layernorm_bwd(dy, x, w, mean, rstd, True, True, None, None, None, None, 0.0)), 1)
    res[f"{cols}+dres"] = round(t(lambda: C.layernorm_bwd(dy, x, w, mean, rstd, True, True, dr, None, None, None, 0.0)), 1)
print(path or "in-tree", res, flush=True)
