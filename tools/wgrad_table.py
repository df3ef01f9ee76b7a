"""Weight-gradient pick table for the BASELINE config 3-5 rank shapes (scaled-batch TP: each TP
rank computes its slice for the TP group's tokens): hipBLASLt (addmm_, beta = 1) vs the MFMA
split-K kernel (wgrad.hip) at a ladder of split counts.  Prints one JSON line per shape and a
final {"table": {(N, K): best split or 0}} summary for ops/linear.py _WGRAD_STATIC."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()


def timeit(fn, iters=6):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(2):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


SHAPES = {  # name: (N, K) of dW = dY^T X
    "gptj_tp4_qkv": (3072, 4096), "gptj_tp4_proj": (4096, 1024), "gptj_tp4_fc1": (4096, 4096),
    "gptj_tp4_fc2": (4096, 4096),
    "neox_tp4_qkv": (4608, 6144), "neox_tp4_proj": (6144, 1536), "neox_tp4_fc1": (6144, 6144),
    "neox_tp4_fc2": (6144, 6144),
    "gpt175_tp2_qkv": (18432, 12288), "gpt175_tp2_proj": (12288, 6144), "gpt175_tp2_fc1": (24576, 12288),
    "gpt175_tp2_fc2": (12288, 24576),
}
T = int(os.environ.get("WG_T", "16384"))
only = os.environ.get("WG_ONLY")
cus = torch.cuda.get_device_properties(0).multi_processor_count
table = {}
for name, (n, k) in SHAPES.items():
    if only and only not in name:
        continue
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * n * k
    model = C.wgrad_splits(T, n, k, cus)
    r = {"T": T, "N": n, "K": k, "model_splits": model, "library_ms": timeit(lambda: g.addmm_(dy.t(), x))}
    for sp in sorted({model, max(1, model // 2), 8, 6, 4, 2, 1}):
        r[f"s{sp}_ms"] = timeit(lambda sp=sp: C.wgrad_(g, dy, x, True, sp))
    cand = {0: r["library_ms"]}
    cand.update({int(k_[1:-3]): v for k_, v in r.items() if k_.startswith("s") and k_.endswith("_ms")})
    best = min(cand, key=cand.get)
    if best != 0 and cand[best] > 0.97 * cand[0]:
        best = 0  # the kernel must beat the library by > 3 %
    r["best"] = best
    r["best_pflops"] = round(fl / cand[best] / 1e12, 3)
    table[f"{n},{k}"] = best
    print(json.dumps({name: {a: (round(b, 3) if isinstance(b, float) else b) for a, b in r.items()}}), flush=True)
    del dy, x, g
    torch.cuda.empty_cache()
print(json.dumps({"table": table}), flush=True)
