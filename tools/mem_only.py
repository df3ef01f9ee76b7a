"""The framework's memory-bound HIP kernels once each at GPT-2 XL training shapes
(mbs 16 x seq 2048 = 32768 tokens, h 1600, 4h 6400), for rocprofv3 counter passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops import multi_tensor as mt  # noqa: E402
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

C = ext()
T, H, I = 32768, 1600, 6400
bf = dict(device="cuda", dtype=torch.bfloat16)
x, dy = torch.randn(T, H, **bf), torch.randn(T, H, **bf)
w, b = torch.randn(H, **bf), torch.randn(H, **bf)
z, dz = torch.randn(T, I, **bf), torch.randn(T, I, **bf)
bi = torch.randn(I, **bf)
W, WT = torch.randn(I, H, **bf), torch.empty(H, I, **bf)
n = 100_000_000
p, g = torch.randn(n, **bf), torch.randn(n, **bf)
ms, m, v = torch.randn(n, device="cuda"), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
for _ in range(int(os.environ.get("ITERS", 2))):
    y, mean, rstd = C.layernorm_fwd(x, None, w, b, 1e-5)
    C.layernorm_bwd(dy, x, w, mean, rstd, True, True, dy)
    C.bias_gelu_fwd(z, bi, False)
    C.bias_gelu_bwd_dbias(dz, z, bi, None, False)
    C.col_sum(x)
    C.transpose_into(W, WT)
    mt.fused_adam_(p, g, ms, m, v, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1)
torch.cuda.synchronize()
print("done")
