"""Does a side-stream kernel run beside the main stream's kernels on this GPU?  Times the
attention keep-bits kernel (GPT-2 XL b32 shape) alone, a LayerNorm / the QKV GEMM alone, and
both with the keep bits on a second stream (as ops/attention.prefetch_keep_bits issues them)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402
from smdistributed_modelparallel_amd.ops.layernorm import layer_norm  # noqa: E402

C = ext()
dev = "cuda"
x = torch.randn(65536, 1600, device=dev, dtype=torch.bfloat16)
w = torch.ones(1600, device=dev, dtype=torch.bfloat16)
b = torch.zeros(1600, device=dev, dtype=torch.bfloat16)
wq = torch.randn(4800, 1600, device=dev, dtype=torch.bfloat16) * 0.02
bq = torch.zeros(4800, device=dev, dtype=torch.bfloat16)
# the bench's GEMM selections (TunableOp file), so the QKV GEMM is the in-step kernel
tun = torch.cuda.tunable
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "tunableop",
                    "gpt2-xl_mbs32_s2048_pp1_tp1.csv")
tun.enable(True)
tun.tuning_enable(False)
tun.set_filename(path, insert_device_ordinal=False)
tun.read_file(path)
side = torch.cuda.Stream()
main = torch.cuda.current_stream()


def kb():
    return C.attention_keep_bits_for(32, 25, 2048, 2048, True, 0.1, 1234, 0, x)


ops = {"layernorm": lambda: layer_norm(x, w, b, 1e-5), "qkv_gemm": lambda: torch.nn.functional.linear(x, wq, bq)}


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def both(op):
    def f():
        side.wait_stream(main)
        with torch.cuda.stream(side):
            kb()
        op()
        main.wait_stream(side)
    return f


for rnd in range(4):
    res = {"keep_bits": timed(kb)}
    for name, op in ops.items():
        res[name] = timed(op)
        res[f"{name}+keep_bits (2 streams)"] = timed(both(op))
        res[f"{name}+keep_bits (1 stream)"] = timed(lambda: (kb(), op()))
    print({k: round(v, 1) for k, v in res.items()}, flush=True)
