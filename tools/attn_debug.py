"""Forward-attention error map: max |O - O_ref| per 32-query wave for a few shapes, for the
in-tree build or (argv[1]) an A/B build (one build per process: both register the same
pybind types)."""
import importlib.machinery
import importlib.util
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:
    sys.path.insert(0, ROOT)
    from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402
    mods = {"intree": ext()}
else:
    loader = importlib.machinery.ExtensionFileLoader("_C", sys.argv[1])
    m = importlib.util.module_from_spec(importlib.util.spec_from_loader("_C", loader))
    loader.exec_module(m)
    mods = {"ab": m}


def ref(q, k, v, scale, causal):
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if causal:
        sq, sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(sq, sk, dtype=torch.bool, device=s.device).triu(sk - sq + 1), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v.float())


torch.manual_seed(0)
for d in (64, 128):
    for causal in (True, False):
        for s in (64, 128, 200, 256):
            q, k, v = (torch.randn(2, s, 3, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
            scale = 1.0 / math.sqrt(d)
            orf = ref(q, k, v, scale, causal)
            line = [f"d{d} causal={int(causal)} s{s}"]
            for name, C in mods.items():
                o = C.attention_fwd(q, k, v, scale, causal, 0)[0].float()
                err = (o - orf).abs().amax(dim=(0, 2, 3))  # per query row
                per32 = [round(x, 3) for x in err.view(-1)[: (s // 32) * 32].view(-1, 32).amax(1).tolist()]
                line.append(f"{name}: max {err.max().item():.3f} per32 {per32}")
            print(" | ".join(line), flush=True)
