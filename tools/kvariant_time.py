"""Time the weight-gradient kernel of several `_C` builds (paths in argv; "intree" = the
in-tree build) on the GPT-2 XL step shapes at T = 65536 with the table's split counts and the
in-step fused bias sums; builds interleaved, best of `rounds`.  One JSON line per build."""
import importlib.machinery
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    if path == "intree":
        sys.path.insert(0, ROOT)
        from smdistributed_modelparallel_amd.ops._ext import ext

        return ext()
    loader = importlib.machinery.ExtensionFileLoader("_C", path)
    mod = importlib.util.module_from_spec(importlib.util.spec_from_loader("_C", loader))
    loader.exec_module(mod)
    return mod


T = 65536
SHAPES = {"qkv": (4800, 1600, 7, True), "proj": (1600, 1600, 5, True), "fc1": (6400, 1600, 4, True),
          "fc2_kernel_s4": (1600, 6400, 4, False)}
builds = sys.argv[1:] or ["intree"]
mods = {b: load(b) for b in builds}
ops = {}
for name, (n, k, sp, db) in SHAPES.items():
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
    bias = torch.zeros(n, device="cuda", dtype=torch.bfloat16) if db else None
    ops[name] = (dy, x, g, bias, sp, 2.0 * T * n * k)
best = {b: {} for b in builds}
for rnd in range(3):
    for b, C in mods.items():
        for name, (dy, x, g, bias, sp, fl) in ops.items():
            fn = lambda: C.wgrad_(g, dy, x, True, sp, bias, True)  # noqa: E731
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            e.synchronize()
            us = s.elapsed_time(e) / 10 * 1e3
            best[b][name] = min(best[b].get(name, 1e30), us)
for b in builds:
    tot = best[b]["qkv"] + best[b]["proj"] + best[b]["fc1"]
    print(json.dumps({"build": b, **{k: round(v, 1) for k, v in best[b].items()},
                      "tflops": {k: round(ops[k][5] / v / 1e6, 1) for k, v in best[b].items()},
                      "qkv+proj+fc1_us": round(tot, 1)}), flush=True)
