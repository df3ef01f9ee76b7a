"""Weight-gradient kernel alone (for hardware-counter passes): WG_N x WG_K at T tokens,
WG_ITERS launches of the MFMA kernel, then the same count of the library GEMM."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

T = int(os.environ.get("WG_T", "65536"))
N = int(os.environ.get("WG_N", "1600"))
K = int(os.environ.get("WG_K", "6400"))
S = int(os.environ.get("WG_SPLITS", "0"))
it = int(os.environ.get("WG_ITERS", "5"))
dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    ext().wgrad_(g, dy, x, True, S)
for _ in range(it):
    g.addmm_(dy.t(), x)
torch.cuda.synchronize()
print("done", flush=True)
