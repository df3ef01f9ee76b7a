"""Micro-benchmarks of the HIP kernels (one process, interleaved rounds, random data).

Reports attention fwd/bwd TFLOP/s (causal FLOPs counted as half) against torch SDPA as
an external reference point, and achieved HBM bandwidth of the memory-bound kernels.
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bench_attention(b, s, h, d, causal=True, dropout=0.0, sdpa=True, zero_bias=False):
    from smdistributed_modelparallel_amd.ops.attention import KeyBias, _FlashAttentionPacked

    qkv = torch.randn(b, s, 3, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    scale = 1.0 / math.sqrt(d)
    flops = 4 * b * h * s * s * d * (0.5 if causal else 1.0)
    out = {}
    kb = KeyBias(torch.zeros(b, s, device="cuda")) if zero_bias else None  # all-ones padding mask
    fwd = lambda: _FlashAttentionPacked.apply(qkv, scale, causal, 0, kb, dropout)  # noqa: E731
    out["ours_fwd_ms"] = timeit(fwd)
    o = fwd()
    g = torch.randn_like(o)
    bwd = lambda: torch.autograd.grad(o, qkv, g, retain_graph=True)  # noqa: E731
    out["ours_bwd_ms"] = timeit(bwd)
    out["ours_fwd_tflops"] = flops / out["ours_fwd_ms"] / 1e9
    out["ours_bwd_tflops"] = 2.5 * flops / out["ours_bwd_ms"] / 1e9
    if not sdpa:
        return out
    try:
        q, k, v = (qkv[:, :, i].transpose(1, 2).detach().contiguous().requires_grad_() for i in range(3))
        sd = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)  # noqa: E731
        out["sdpa_fwd_ms"] = timeit(sd)
        o2 = sd()
        g2 = torch.randn_like(o2)
        out["sdpa_bwd_ms"] = timeit(lambda: torch.autograd.grad(o2, (q, k, v), g2, retain_graph=True))
    except Exception as e:  # pragma: no cover
        out["sdpa_error"] = str(e)[:200]
    return out


def bench_memory_bound():
    from smdistributed_modelparallel_amd.ops import layernorm, gelu, multi_tensor
    from smdistributed_modelparallel_amd.ops._ext import ext

    res = {}
    x = torch.randn(16384, 1600, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(1600, device="cuda", dtype=torch.bfloat16)
    bb = torch.zeros(1600, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: layernorm.layer_norm(x, w, bb))
    res["layernorm_fwd_GBps"] = 2 * x.numel() * 2 / t / 1e6
    C = ext()
    xl = torch.randn(32768, 1600, device="cuda", dtype=torch.bfloat16)
    dyl = torch.randn_like(xl)
    wl = torch.randn(1600, device="cuda", dtype=torch.bfloat16)
    bl = torch.randn(1600, device="cuda", dtype=torch.bfloat16)
    _, mu, rs = C.layernorm_fwd(xl, None, wl, bl, 1e-5)
    t = timeit(lambda: C.layernorm_bwd(dyl, xl, wl, mu, rs, True, True, dyl))
    res["layernorm_bwd_dres_32768x1600_us"] = t * 1e3
    res["layernorm_bwd_dres_GBps"] = 4 * xl.numel() * 2 / t / 1e6
    del xl, dyl
    xg = torch.randn(32768, 6400, device="cuda", dtype=torch.bfloat16)
    bg = torch.randn(6400, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: gelu.bias_gelu(xg, bg))
    res["bias_gelu_fwd_GBps"] = 2 * xg.numel() * 2 / t / 1e6
    res["bias_gelu_fwd_us"] = t * 1e3
    t = timeit(lambda: torch.nn.functional.gelu(xg, approximate="tanh"))
    res["torch_gelu_tanh_fwd_GBps"] = 2 * xg.numel() * 2 / t / 1e6
    t = timeit(lambda: xg.clone())
    res["torch_clone_GBps"] = 2 * xg.numel() * 2 / t / 1e6
    dg = torch.randn_like(xg)
    t = timeit(lambda: C.bias_gelu_bwd_dbias(dg, xg, bg))
    res["bias_gelu_bwd_dbias_GBps"] = 3 * xg.numel() * 2 / t / 1e6
    res["bias_gelu_bwd_dbias_us"] = t * 1e3
    del dg
    for cols in (1600, 4800):
        xc = torch.randn(32768, cols, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: C.col_sum(xc))
        res[f"col_sum_32768x{cols}_GBps"] = xc.numel() * 2 / t / 1e6
        res[f"col_sum_32768x{cols}_us"] = t * 1e3
    del xg
    w = torch.randn(6400, 1600, device="cuda", dtype=torch.bfloat16)
    wt = torch.empty(1600, 6400, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: C.transpose_into(w, wt))
    res["transpose_6400x1600_GBps"] = 2 * w.numel() * 2 / t / 1e6
    n = 200_000_000
    p = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    gr = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    ms = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    t = timeit(lambda: multi_tensor.fused_adam_(p, gr, ms, m, v, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1), iters=10)
    res["adam_GBps"] = n * 28 / t / 1e6
    return res


if __name__ == "__main__":
    only_attn = "--attention" in sys.argv
    results = {"attention_gpt2xl_b32_s2048": bench_attention(32, 2048, 25, 64, sdpa=False),
               "attention_gpt2xl_b32_s2048_dropout0.1": bench_attention(32, 2048, 25, 64, dropout=0.1, sdpa=False),
               "attention_gpt2xl_b32_s2048_onesmask": bench_attention(32, 2048, 25, 64, sdpa=False, zero_bias=True),
               "attention_gpt2xl_b8_s2048": bench_attention(8, 2048, 25, 64),
               "attention_neox_b4_s2048_h16_d96": bench_attention(4, 2048, 16, 96, sdpa=False),
               "attention_b4_s4096_h32_d128": bench_attention(4, 4096, 32, 128),
               "attention_gptj_b8_s2048_h16_d256": bench_attention(8, 2048, 16, 256, sdpa=False)}
    if not only_attn:
        results.update(bench_memory_bound())
    print(json.dumps(results, indent=1))
