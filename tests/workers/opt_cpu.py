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


def ref_novograd(rs, gs_steps, lr, b1, b2, eps, wd, reg_inside=False, norm_type=2, init_zero=False):
    """apex multi_tensor_novograd semantics, float64: per-tensor gradient NORM blended as
    sqrt(b2 n_old^2 + (1 - b2) n^2) (L2) / b2 n_old + (1 - b2) n (L-inf), first step from n."""
    v = [None] * len(rs)
    m = [torch.zeros_like(r) for r in rs]
    for step, gs in enumerate(gs_steps, 1):
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        for i, (r, g) in enumerate(zip(rs, gs)):
            g = g.double()
            n = float(g.norm()) if norm_type == 2 else float(g.abs().max())
            old = (0.0 if init_zero else n) if v[i] is None else v[i]
            v[i] = (b2 * old * old + (1 - b2) * n * n) ** 0.5 if norm_type == 2 else b2 * old + (1 - b2) * n
            denom = v[i] / bc2 + eps
            if reg_inside:
                m[i] = b1 * m[i] + (1 - b1) * (g / denom + wd * r)
                r -= lr * m[i] / bc1
            else:
                m[i] = b1 * m[i] + (1 - b1) * g
                r -= lr * ((m[i] / bc1) / denom + wd * r)


def ref_lamb_standalone(rs, gs_steps, lr, b1, b2, eps, wd, max_norm, adam_w=True):
    """apex FusedLAMB: global-norm clipped gradient, Adam direction (+ decoupled or L2 decay),
    per-tensor trust ratio."""
    m = [torch.zeros_like(r) for r in rs]
    v = [torch.zeros_like(r) for r in rs]
    for step, gs in enumerate(gs_steps, 1):
        gn = sum(float(g.double().pow(2).sum()) for g in gs) ** 0.5
        clip = gn / max_norm if gn > max_norm else 1.0
        for i, (r, g) in enumerate(zip(rs, gs)):
            sg = g.double() / clip
            if not adam_w:
                sg = sg + wd * r
            m[i] = b1 * m[i] + (1 - b1) * sg
            v[i] = b2 * v[i] + (1 - b2) * sg * sg
            u = (m[i] / (1 - b1 ** step)) / ((v[i] / (1 - b2 ** step)).sqrt() + eps)
            if adam_w:
                u = u + wd * r
            a, b = float(r.norm()), float(u.norm())
            r -= (lr * a / b if (a > 0 and b > 0) else lr) * u


def _grads(ps, steps, seed):
    g = torch.Generator().manual_seed(seed)
    return [[torch.randn(p.shape, generator=g) for p in ps] for _ in range(steps)]


def novograd():
    torch.manual_seed(1)
    for kw in (dict(), dict(reg_inside_moment=True), dict(norm_type=0), dict(init_zero=True)):
        ps = [torch.randn(5, 4, requires_grad=True), torch.randn(3, requires_grad=True)]
        rs = [p.detach().clone().double() for p in ps]
        opt = FusedNovoGrad(ps, lr=0.1, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, **kw)
        steps = _grads(ps, 3, 7)
        for gs in steps:
            for p, g in zip(ps, gs):
                p.grad = g.clone()
            opt.step()
        ref_novograd(rs, steps, 0.1, 0.9, 0.98, 1e-8, 0.01, reg_inside=kw.get("reg_inside_moment", False),
                     norm_type=kw.get("norm_type", 2), init_zero=kw.get("init_zero", False))
        for p, r in zip(ps, rs):
            assert torch.allclose(p.detach().double(), r, atol=1e-5), (kw, (p - r).abs().max())
    print("OK novograd", flush=True)


def lamb_standalone():
    torch.manual_seed(2)
    for adam_w in (True, False):
        ps = [torch.randn(6, 5, requires_grad=True), torch.randn(5, requires_grad=True)]
        rs = [p.detach().clone().double() for p in ps]
        opt = FusedLAMB(ps, lr=0.05, weight_decay=0.01, max_grad_norm=1.0, adam_w_mode=adam_w)
        steps = _grads(ps, 3, 9)
        for gs in steps:
            for p, g in zip(ps, gs):
                p.grad = g.clone()
            opt.step()
        ref_lamb_standalone(rs, steps, 0.05, 0.9, 0.999, 1e-6, 0.01, 1.0, adam_w)
        for p, r in zip(ps, rs):
            assert torch.allclose(p.detach().double(), r, atol=1e-5), (adam_w, (p - r).abs().max())
    print("OK lamb-standalone", flush=True)


if __name__ == "__main__":
    lamb()
    novograd()
    lamb_standalone()
    smp.barrier()
