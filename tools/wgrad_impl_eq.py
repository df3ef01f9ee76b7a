"""impl 2 (temporary A/B variant of the ping-pong weight-gradient kernel) must give bitwise the
same dW (and bias sums) as impl 1 on the GPT-2 XL shapes and an edge shape."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()
for (n, k, t, sp) in [(6400, 1600, 16384, 4), (1600, 6400, 16384, 4), (4800, 1600, 8192, 3), (1000, 1320, 4160, 2)]:
    g0 = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(t, n, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(t, k, device="cuda", dtype=torch.bfloat16, generator=g0)
    outs = []
    for impl in (1, 2):
        g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)
        C.wgrad_(g, dy, x, True, sp, impl=impl)
        outs.append(g)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), (n, k)
    print(f"{n}x{k} T{t} s{sp}: impl 2 == impl 1", flush=True)
print("OK", flush=True)
