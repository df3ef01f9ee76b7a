"""HBM streaming probe: copy vs the bias-GeLU / LayerNorm kernels at the GPT-2 XL shapes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

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
    return s.elapsed_time(e) / it


res = {}
x = torch.randn(65536, 6400, device="cuda", dtype=torch.bfloat16)
b = torch.randn(6400, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
nb = 2 * x.numel() * 2
for name, fn in (("copy_", lambda: y.copy_(x)), ("bias_gelu_fwd", lambda: C.bias_gelu_fwd(x, b) if hasattr(C, "bias_gelu_fwd") else None),
                 ("torch_gelu_tanh", lambda: torch.nn.functional.gelu(x, approximate="tanh")),
                 ("torch_add_scalar", lambda: torch.add(x, 1.0, out=y))):
    try:
        ms = t(fn)
        res[name] = {"us": round(ms * 1e3, 1), "TBps": round(nb / ms / 1e9, 2)}
    except Exception as ex:  # pragma: no cover
        res[name] = str(ex)[:100]
from smdistributed_modelparallel_amd.ops import gelu  # noqa: E402

ms = t(lambda: gelu.bias_gelu(x, b))
res["ops.bias_gelu"] = {"us": round(ms * 1e3, 1), "TBps": round(nb / ms / 1e9, 2)}
dg = torch.randn_like(x)
ms = t(lambda: C.bias_gelu_bwd_dbias(dg, x, b))
res["bias_gelu_bwd_dbias"] = {"us": round(ms * 1e3, 1), "TBps": round(3 * x.numel() * 2 / ms / 1e9, 2)}
xl = torch.randn(65536, 1600, device="cuda", dtype=torch.bfloat16)
w = torch.randn(1600, device="cuda", dtype=torch.bfloat16)
ms = t(lambda: C.layernorm_fwd(xl, None, w, w, 1e-5))
res["ln_fwd_1600"] = {"us": round(ms * 1e3, 1), "TBps": round(2 * xl.numel() * 2 / ms / 1e9, 2)}
yl = torch.empty_like(xl)
ms = t(lambda: yl.copy_(xl))
res["copy_1600"] = {"us": round(ms * 1e3, 1), "TBps": round(2 * xl.numel() * 2 / ms / 1e9, 2)}
ms = t(lambda: gelu.bias_gelu(x, b))
res["ops.bias_gelu_flat"] = {"us": round(ms * 1e3, 1), "TBps": round(nb / ms / 1e9, 2)}
ref = torch.nn.functional.gelu(x.float() + b.float(), approximate="tanh")
res["flat_max_err"] = float((gelu.bias_gelu(x, b).float() - ref).abs().max())
print(json.dumps(res, indent=1))
