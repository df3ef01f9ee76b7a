"""Time the flash-attention kernels of one `_C` build (path in argv[1], default: in-tree),
GPT-2 XL shape b32 h25 s2048 d64 causal: plain / zero key bias / dropout 0.1."""
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


b, s, h, d = 32, 2048, 25, 64
qkv = torch.randn(b, s, 3, h, d, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
o, lse = C.attention_fwd(q, k, v, 0.125, True, 0)[:2]
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
zb = torch.zeros(b, s, device="cuda")
def drop_times():
    """dropout 0.1: round-3 builds regenerate the keep hash in the backward; round-4 builds
    store the forward's keep bits (a third output) and the backward reads them."""
    out = {}
    args = (q, k, v, 0.125, True, 0, None, 0.1, 1234, 0)
    res = C.attention_fwd(*args)
    extra = {"drop_bits": res[2]} if len(res) > 2 else {}
    out["fwd_drop_us"] = round(t(lambda: C.attention_fwd(*args)), 1)
    if hasattr(C, "attention_keep_bits"):  # round 6: part of fwd_drop_us (generated before the forward)
        out["keep_bits_us"] = round(t(lambda: C.attention_keep_bits(q, k, v, True, 0, 0.1, 1234, 0)), 1)
    out["bwd_drop_us"] = round(t(lambda: C.attention_bwd_into(do, q, k, v, res[0], res[1], dqkv[:, :, 0], dqkv[:, :, 1],
                                                              dqkv[:, :, 2], 0.125, True, 0, None, 0.1, 1234, 0,
                                                              **extra)), 1)
    out["keep_bits"] = bool(extra)
    return out


for _ in range(2):
    print(path or "in-tree", drop_times(), flush=True)
    print(path or "in-tree", {
        "fwd_us": round(t(lambda: C.attention_fwd(q, k, v, 0.125, True, 0)), 1),
        "fwd_zero_bias_us": round(t(lambda: C.attention_fwd(q, k, v, 0.125, True, 0, zb)), 1),
        "bwd_us": round(t(lambda: C.attention_bwd_into(do, q, k, v, o, lse, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                                                       0.125, True, 0)), 1),
        "bwd_zero_bias_us": round(t(lambda: C.attention_bwd_into(do, q, k, v, o, lse, dqkv[:, :, 0], dqkv[:, :, 1],
                                                                 dqkv[:, :, 2], 0.125, True, 0, zb)), 1),
    }, flush=True)
