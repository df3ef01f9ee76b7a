"""Weight-gradient kernel timings at the GPT-2 XL shapes (T = 65536) for the kernel variant
selected by SMP_WGRAD_PIPE (one variant per process: the choice is read once), at the
bench's static split counts and two neighbours; one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()
T = 65536


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


pipe = os.environ.get("SMP_WGRAD_PIPE", "default")
for (n, k), splits in (((4800, 1600), (7, 6, 8)), ((1600, 1600), (5, 4, 6)), ((6400, 1600), (4, 3, 5)),
                       ((1600, 6400), (4, 3, 5))):
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
    # numerics: kernel vs fp32 reference on a token slice
    ts = 4096
    ref = dy[:ts].float().t() @ x[:ts].float()
    gg = torch.zeros(n, k, device="cuda", dtype=torch.float32)
    C.wgrad_(gg, dy[:ts], x[:ts], True, 2)
    err = float((gg - ref).abs().max() / ref.abs().max())
    r = {"pipe": pipe, "shape": f"{n}x{k}", "rel_err": round(err, 6)}
    bias = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    for sp in splits:
        ms = timeit(lambda: C.wgrad_(g, dy, x, True, sp))
        r[f"s{sp}"] = [round(ms, 3), round(2.0 * T * n * k / ms / 1e9, 1)]
        if os.environ.get("WG_DBIAS") == "1":
            ms = timeit(lambda: C.wgrad_(g, dy, x, True, sp, bias, True))
            r[f"s{sp}_dbias"] = round(ms, 3)
    if os.environ.get("WG_DBIAS") == "1":
        r["col_sum_ms"] = round(timeit(lambda: C.col_sum(dy, bias)), 3)
        r["library_ms"] = round(timeit(lambda: g.addmm_(dy.t(), x)), 3)
    print(json.dumps(r), flush=True)
    del dy, x, g, gg, ref
