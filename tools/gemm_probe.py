import torch, time
torch.cuda.tunable.enable(True); torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(30); torch.cuda.tunable.set_max_tuning_iterations(40)
torch.cuda.tunable.set_filename("/tmp/probe_tune.csv", insert_device_ordinal=False)
x = torch.randn(32768, 1600, device="cuda", dtype=torch.bfloat16)
res = {}
for n in (4800, 1600, 6400):
    W = torch.randn(n, 1600, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    for name, fn in (("bias", lambda: torch.nn.functional.linear(x, W, b)), ("nobias", lambda: torch.nn.functional.linear(x, W))):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): fn()
        e.record(); torch.cuda.synchronize()
        t = s.elapsed_time(e) / 20
        res[f"{n}_{name}"] = (round(t, 4), round(2 * 32768 * 1600 * n / t / 1e9, 1))
print(res)
