"""Worker: DistributedOptimizer(FusedLAMB) -- whole-domain segmented LAMB (per-parameter
trust ratios, two launches per domain) -- against a plain per-parameter LAMB, and
FusedNovoGrad (device-resident per-tensor moments) against a float reference."""
import copy

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.ops import multi_tensor as mt
from smdistributed_modelparallel_amd.optimizers import FusedLAMB, FusedNovoGrad


def ref_lamb_step(params, state, lr, b1, b2, eps, wd, step):
    for p in params:
        g = p.grad
        st = state.setdefault(p, {"m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["m"].mul_(b1).add_(g, alpha=1 - b1)
        st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = (st["m"] / (1 - b1 ** step)) / ((st["v"] / (1 - b2 ** step)).sqrt() + eps) + wd * p
        a, b = p.norm(), upd.norm()
        trust = (a / b) if (a > 0 and b > 0) else 1.0
        p.sub_(lr * trust * upd)


def lamb():
    smp.init({"ddp": True})
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(20, 30), nn.Tanh(), nn.Linear(30, 7))
    ref = copy.deepcopy(net)
    mt.LAMB_CHUNK = 64  # several chunks per parameter
    model = smp.DistributedModel(net, bucket_cap_mb=0.001)  # several domains
    opt = smp.DistributedOptimizer(FusedLAMB(model.parameters(), lr=0.05, weight_decay=0.01))
    state = {}

    @smp.step
    def train(model, x):
        loss = model(x).pow(2).mean()
        model.backward(loss)
        return loss

    for step in range(1, 4):
        x = torch.randn(6, 20)
        opt.zero_grad()
        train(model, x)
        opt.step()
        for p in ref.parameters():
            p.grad = None
        ref(x).pow(2).mean().backward()
        with torch.no_grad():
            ref_lamb_step(list(ref.parameters()), state, 0.05, 0.9, 0.999, 1e-6, 0.01, step)
    assert len(opt.domains) > 1, len(opt.domains)
    for (n, p), (_, q) in zip(model.module.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.detach(), q.detach(), atol=1e-5), (n, (p - q).abs().max())
    print("OK lamb", flush=True)


def novograd():
    torch.manual_seed(1)
    ps = [torch.randn(5, 4, requires_grad=True), torch.randn(3, requires_grad=True)]
    rs = [p.detach().clone().double() for p in ps]
    opt = FusedNovoGrad(ps, lr=0.1, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01)
    v = [None, None]
    m = [torch.zeros_like(r) for r in rs]
    for step in range(1, 4):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        opt.step()
        for i, (r, g) in enumerate(zip(rs, gs)):
            g = g.double()
            n2 = float((g * g).sum())
            v[i] = n2 if v[i] is None else 0.98 * v[i] + 0.02 * n2
            upd = g / (v[i] ** 0.5 + 1e-8) + 0.01 * r
            m[i] = 0.9 * m[i] + 0.1 * upd
            r -= 0.1 * m[i] / (1 - 0.9 ** step)
    for p, r in zip(ps, rs):
        assert torch.allclose(p.detach().double(), r, atol=1e-5), (p - r).abs().max()
    print("OK novograd", flush=True)


if __name__ == "__main__":
    lamb()
    novograd()
    smp.barrier()
