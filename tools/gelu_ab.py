"""Same-process A/B of the GeLU kernels at the GPT-2 XL MLP shape (T = mbs 32 x 2048 tokens,
4h = 6400): row streaming (SMP_GELU_ROWS=1) vs the column walker (0), forward and the fused
backward + dbias.  Prints us and effective HBM TB/s per variant, alternating the variants
over several rounds so clock drift hits both."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()
T, H = int(os.environ.get("T", 65536)), int(os.environ.get("H", 6400))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for cols in (H, H // 4, 3 * H // 4):
    x = torch.randn(T, cols, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(cols, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    nb = x.numel() * 2
    res = {}
    for rnd in range(3):
        for mode in ("0", "1"):
            os.environ["SMP_GELU_ROWS"] = mode
            f = timeit(lambda: C.bias_gelu_fwd(x, b, False))
            bw = timeit(lambda: C.bias_gelu_bwd_dbias(dy, x, b, None, False))
            res.setdefault(mode, []).append((f, bw))
    for mode, v in res.items():
        f = min(a for a, _ in v)
        bw = min(c for _, c in v)
        print(f"T={T} cols={cols} rows_stream={mode}: fwd {f:.1f} us ({2 * nb / f / 1e6:.2f} TB/s)  "
              f"bwd+dbias {bw:.1f} us ({3 * nb / bw / 1e6:.2f} TB/s)", flush=True)
    del x, dy
    torch.cuda.empty_cache()
