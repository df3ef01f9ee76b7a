"""Fused optimizers (reference `smp/torch/optimizers/{fused_adam,fused_lamb,fused_novograd}.py`).

Standalone they update each parameter with the fused HIP kernel; wrapped in
``smp.DistributedOptimizer`` the whole model is updated per flat-buffer domain (one kernel
launch per gradient bucket).
"""
import torch

from ..ops import multi_tensor as mt
from .optimizer import DistributedOptimizer  # noqa: F401


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support amsgrad")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = adam_w_mode
        self.set_grad_none = set_grad_none

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    if p.dtype != torch.float32:
                        st["master"] = p.detach().float().clone()
                st["step"] += 1
                master = st.get("master", p)
                lowp = p if p.dtype != torch.float32 else None
                mt.fused_adam_(lowp.view(-1) if lowp is not None else None, p.grad.contiguous().view(-1),
                               master.view(-1), st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1), g["lr"], b1, b2,
                               g["eps"], g["weight_decay"], st["step"], 1.0, adamw=self.adam_w_mode,
                               bias_correction=g["bias_correction"])
        return loss


class FusedLAMB(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 amsgrad=False, adam_w_mode=True, grad_averaging=True, set_grad_none=True, max_grad_norm=1.0,
                 use_nvlamb=False):
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, use_nvlamb=use_nvlamb)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    st["master"] = p.detach().float().clone() if p.dtype != torch.float32 else p
                st["step"] += 1
                master = st["master"].view(-1)
                upd = torch.empty_like(master)
                mt.lamb_stage1_(p.grad.contiguous().view(-1), master, st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1),
                                upd, b1, b2, g["eps"], g["weight_decay"], st["step"], 1.0, g["bias_correction"])
                pn, un = mt.sumsq(master), mt.sumsq(upd)
                lowp = p.view(-1) if p.dtype != torch.float32 else None
                mt.lamb_stage2_(lowp, master, upd, g["lr"], pn, un, use_trust=g["use_nvlamb"] or g["weight_decay"] != 0)
        return loss


class FusedNovoGrad(torch.optim.Optimizer):
    """NovoGrad: per-tensor second moment (layer-wise), first moment on the normalised grad."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, reg_inside_moment=False, grad_averaging=True, norm_type=2, init_zero=False,
                 set_grad_none=True):
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, init_zero=init_zero)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                grad = p.grad.float()
                # the per-tensor second moment stays on the device (no host sync per tensor)
                gn2 = mt.sumsq(grad.view(-1))
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(gn2) if g["init_zero"] else gn2.clone()
                st["step"] += 1
                v = st["exp_avg_sq"]
                v.mul_(b2).add_(gn2, alpha=1 - b2)
                upd = grad / (v.sqrt() + g["eps"])
                if g["weight_decay"] != 0:
                    upd.add_(p.float(), alpha=g["weight_decay"])
                m = st["exp_avg"]
                m.mul_(b1).add_(upd, alpha=(1 - b1) if g["grad_averaging"] else 1.0)
                bc1 = 1 - b1 ** st["step"] if g["bias_correction"] else 1.0
                p.add_((m / bc1).to(p.dtype), alpha=-g["lr"])
        return loss


__all__ = ["DistributedOptimizer", "FusedAdam", "FusedLAMB", "FusedNovoGrad"]
