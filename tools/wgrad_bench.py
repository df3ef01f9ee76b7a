"""Weight-gradient GEMM: hand-written split-K MFMA kernel (wgrad.hip) vs hipBLASLt
(TunableOp-selected as in the bench) at the GPT-2 XL shapes, T = 65536 tokens."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(False)
tun.set_filename(os.path.join(ROOT, "configs", "tunableop", "gpt2-xl_mbs32_s2048_pp1_tp1.csv"),
                 insert_device_ordinal=False)
tun.read_file()
C = ext()


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


T = int(os.environ.get("WG_T", "65536"))
res = {}
cus = torch.cuda.get_device_properties(0).multi_processor_count
for n, k in ((4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400), (50304, 1600)):
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * n * k
    r = {"splits": C.wgrad_splits(T, n, k, cus)}
    r["hipblaslt_ms"] = timeit(lambda: g.addmm_(dy.t(), x))
    r["kernel_ms"] = timeit(lambda: C.wgrad_(g, dy, x, True))  # stream-K (default)
    for sp in (1, 2, 4):
        r[f"kernel_s{sp}_ms"] = timeit(lambda: C.wgrad_(g, dy, x, True, sp))
    r["hipblaslt_tflops"] = fl / r["hipblaslt_ms"] / 1e9
    r["kernel_tflops"] = fl / r["kernel_ms"] / 1e9
    res[f"{n}x{k}"] = {a: (round(b, 3) if isinstance(b, float) else b) for a, b in r.items()}
    print(json.dumps({f"{n}x{k}": res[f"{n}x{k}"]}), flush=True)
    del dy, x, g
