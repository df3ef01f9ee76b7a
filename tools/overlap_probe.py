"""Does running the weight-gradient GEMM on a side stream, concurrently with the
input-gradient GEMM, fill the CUs the wgrad GEMM leaves idle?  (GPT-2 XL shapes,
T = 65536 tokens, bf16, TunableOp results of the bench.)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T = 65536
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(False)
tun.set_filename(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "tunableop",
                              "gpt2-xl_mbs32_s2048_pp1_tp1.csv"), insert_device_ordinal=False)
tun.read_file()


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


res = {}
side = torch.cuda.Stream()
main = torch.cuda.current_stream()
for n, k in ((4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400)):
    x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(n, k, device="cuda", dtype=torch.bfloat16).t().contiguous()  # [k, n]
    g = torch.zeros(n, k, device="cuda", dtype=torch.bfloat16)

    def dgrad():
        return torch.nn.functional.linear(dy, wt)

    def wgrad():
        g.addmm_(dy.t(), x)

    def seq():
        dgrad()
        wgrad()

    def conc():
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        ev2 = torch.cuda.Event()
        ev2.record(side)
        main.wait_event(ev2)

    r = {"dgrad_ms": timeit(dgrad), "wgrad_ms": timeit(wgrad), "seq_ms": timeit(seq), "concurrent_ms": timeit(conc)}
    res[f"{n}x{k}"] = {a: round(b, 3) for a, b in r.items()}
    print(json.dumps({f"{n}x{k}": res[f"{n}x{k}"]}), flush=True)
print(json.dumps(res, indent=1))
