"""Weight-gradient GEMM probe at GPT-2 XL training shapes (T = mbs 32 x 2048 tokens).

dW[N, K] += dY[T, N]^T X[T, K] has only N x K outputs (81-280 macro tiles of 192-256) for
256 CUs, so one GEMM leaves most of the chip idle for its ~65k-long reduction.  Compares the
committed ``grad.addmm_`` (TunableOp-selected) with split-K forms: S reduction chunks as a
batched GEMM into partial sums, then one reduction into the gradient.

Prints one line per (shape, method): ms and TFLOP/s.
"""
import os
import sys

import torch

T = int(os.environ.get("T", 32 * 2048))
tun = torch.cuda.tunable
csv = os.environ.get("TUNE_FILE")
if csv:
    tun.enable(True)
    tun.tuning_enable(os.environ.get("TUNE", "0") == "1")
    tun.set_max_tuning_duration(20)
    tun.set_max_tuning_iterations(30)
    tun.set_filename(csv, insert_device_ordinal=False)
    if os.path.exists(csv):
        tun.read_file(csv)


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def split_k(dy, x, g, S, fp32):
    Tc = dy.shape[0] // S
    a = dy.view(S, Tc, dy.shape[1]).transpose(1, 2)
    b = x.view(S, Tc, x.shape[1])
    if fp32:
        parts = torch.bmm(a, b, out_dtype=torch.float32)
    else:
        parts = torch.bmm(a, b)
    g.add_(parts.sum(0, dtype=torch.float32).to(g.dtype) if not fp32 else parts.sum(0).to(g.dtype))


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

METHODS = os.environ.get("METHODS", "addmm,splitk,tn").split(",")


def transposed(t):
    out = torch.empty(t.shape[1], t.shape[0], dtype=t.dtype, device=t.device)
    ext().transpose_into(t, out)
    return out


shapes = [("qkv", 4800, 1600), ("proj", 1600, 1600), ("fc1", 6400, 1600), ("fc2", 1600, 6400)]
for name, N, K in shapes:
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    flop = 2.0 * T * N * K
    ref = (dy.float().t() @ x.float())
    rows = [("addmm", lambda: g.addmm_(dy.t(), x))]
    if "splitk" in METHODS:
        for S in (4, 8, 16):
            rows.append((f"splitk{S}", lambda S=S: split_k(dy, x, g, S, False)))
    if "tn" in METHODS:
        dyT, xT = transposed(dy), transposed(x)
        # both operands contiguous along the T reduction (the forward GEMM's layout)
        rows.append(("tn_gemm_only", lambda: g.add_(torch.nn.functional.linear(dyT, xT))))
        rows.append(("tn_addmm_only", lambda: g.addmm_(dyT, xT.t())))
        rows.append(("transpose_dy", lambda: ext().transpose_into(dy, dyT)))
        rows.append(("transpose_x", lambda: ext().transpose_into(x, xT)))
    for meth, fn in rows:
        g.zero_()
        fn()
        err = (g.float() - ref).abs().max().item() / ref.abs().max().item() if "transpose" not in meth else 0.0
        ms = timeit(fn)
        print(f"{name} N={N} K={K} {meth}: {ms:.3f} ms {flop / ms / 1e9:.0f} TFLOP/s relerr {err:.2e}", flush=True)
    del dy, x, g, ref, rows
    dyT = xT = None
    torch.cuda.empty_cache()
sys.stdout.flush()
# TunableOp writes the results file itself at process exit (set_filename above)
