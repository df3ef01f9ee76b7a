"""(WG_IMPLS selects the arms, default "1,0": ping-pong, round-4 kernel; a temporary variant
built as impl 2 is named "ppv".)
Weight-gradient kernels A/B in one process (cdna_hip_programming.md §5.4 rule 24): the
ping-pong kernel (impl 1) and the round-4 one-barrier-per-tile kernel (impl 0) at a ladder of
split counts, and hipBLASLt (addmm_), on the GPT-2 XL b32 shapes (T = 65536), interleaved
rounds, best of each.  One JSON line per shape."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()
T = int(os.environ.get("WG_T", "65536"))
SHAPES = [tuple(int(v) for v in s.split("x")) for s in
          os.environ.get("WG_SHAPES", "6400x1600,1600x6400,4800x1600,1600x1600").split(",")]
SPLITS = [int(v) for v in os.environ.get("WG_SPLITS", "1,2,3,4,5,7").split(",")]
ROUNDS = int(os.environ.get("WG_ROUNDS", "3"))
IMPLS = [int(v) for v in os.environ.get("WG_IMPLS", "1,0").split(",")]
NAMES = {0: "glds", 1: "pp", 2: "ppv"}


def timed(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


for n, k in SHAPES:
    g0 = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16, generator=g0)
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
    cands = {"library": lambda: g.addmm_(dy.t(), x)}
    for sp in SPLITS:
        for im in IMPLS:
            cands[f"{NAMES[im]}_s{sp}"] = (lambda sp=sp, im=im: C.wgrad_(g, dy, x, True, sp, impl=im))
    for fn in cands.values():
        fn()
    torch.cuda.synchronize()
    best = {}
    for _ in range(ROUNDS):
        for name, fn in cands.items():
            best[name] = min(best.get(name, 1e9), timed(fn))
    fl = 2.0 * T * n * k
    r = {name: [round(ms * 1e3, 1), round(fl / ms / 1e9, 1)] for name, ms in best.items()}  # us, TFLOP/s
    bests = {f"best_{NAMES[im]}_us": round(min(v for k_, v in best.items() if k_.startswith(NAMES[im] + "_s")) * 1e3, 1)
             for im in IMPLS}
    print(json.dumps({"shape": f"{n}x{k}", "T": T, **bests,
                      "library_us": round(best["library"] * 1e3, 1), "all_us_tflops": r}), flush=True)
    del dy, x, g
    torch.cuda.empty_cache()
