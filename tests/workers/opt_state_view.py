"""Worker (argv: adamw|sgd|adagrad): ``optimizer.state[param]`` of smp.DistributedOptimizer holds
the torch-named moments of the fused flat-buffer optimizer, equal to a plain torch optimizer's
after two steps, and an in-place edit through it reaches the next step."""
import copy
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp

kind = sys.argv[1]
smp.init({})
torch.manual_seed(0)
net = nn.Sequential(nn.Linear(8, 16), nn.Tanh(), nn.Linear(16, 4))
ref = copy.deepcopy(net)
make = {"adamw": lambda ps: torch.optim.AdamW(ps, lr=1e-2),
        "sgd": lambda ps: torch.optim.SGD(ps, lr=1e-2, momentum=0.9),
        "adagrad": lambda ps: torch.optim.Adagrad(ps, lr=1e-2)}[kind]
model = smp.DistributedModel(net)
opt = smp.DistributedOptimizer(make(model.parameters()))
ropt = make(ref.parameters())


@smp.step
def step(model, x):
    loss = model(x).square().mean()
    model.backward(loss)
    return loss


x = torch.randn(4, 8)
for _ in range(2):
    opt.zero_grad()
    step(model, x)
    opt.step()
    ropt.zero_grad()
    ref(x).square().mean().backward()
    ropt.step()
keys = {"adamw": ("exp_avg", "exp_avg_sq"), "sgd": ("momentum_buffer",), "adagrad": ("sum",)}[kind]
for p, rp in zip(net.parameters(), ref.parameters()):
    s, r = opt.state[p], ropt.state[rp]
    for k in keys:
        assert torch.allclose(s[k], r[k], atol=1e-6), (k, (s[k] - r[k]).abs().max())
    if "step" in r:
        assert float(s["step"]) == float(r["step"]) == 2.0
# an edit through the view is the optimizer's state
p0, rp0 = next(net.parameters()), next(ref.parameters())
k = keys[0]
opt.state[p0][k].zero_()
ropt.state[rp0][k].zero_()
opt.zero_grad()
step(model, x)
opt.step()
ropt.zero_grad()
ref(x).square().mean().backward()
ropt.step()
assert torch.allclose(p0.detach(), rp0.detach(), atol=1e-5), (p0 - rp0).abs().max()
print(f"rank {smp.rank()} OK {kind}", flush=True)
