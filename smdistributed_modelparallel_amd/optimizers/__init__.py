"""Fused optimizers (reference `smp/torch/optimizers/fused_lamb.py`, apex
`optimizers/{fused_adam,fused_lamb,fused_novograd}.py` over `amp_C.multi_tensor_*`).

Standalone, each step is a handful of multi-tensor launches over the whole parameter list
(`optim.hip` mt_* kernels: one block per <= 64K-element chunk of any tensor, the tensor
pointers and chunk table in one device array) -- not one launch per parameter.  Low-precision
parameters keep an fp32 master copy in the optimizer state (updated in the same pass).
Wrapped in ``smp.DistributedOptimizer`` the model is instead updated per flat-buffer domain.
"""
import torch
import torch.distributed as dist

from .. import torch as _smp_torch  # noqa: F401  (the smp package first: it imports .optimizer itself)
from ..ops import multi_tensor as mt
from .optimizer import DistributedOptimizer  # noqa: F401


def _lists(opt, group, moments):
    """Active parameters of `group` bucketed by (param dtype, grad dtype): for each bucket the
    per-role tensor lists of one multi-tensor launch (state created on first use)."""
    buckets = {}
    for p in group["params"]:
        if p.grad is None:
            continue
        if p.grad.is_sparse:
            raise RuntimeError(f"{type(opt).__name__} does not support sparse gradients")
        st = opt.state[p]
        if not st:
            for name in moments:
                st[name] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
            if p.dtype != torch.float32:
                st["master"] = p.detach().float().clone()
        g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
        b = buckets.setdefault((p.dtype, g.dtype), {"grad": [], "param": [], "master": [], "params": []})
        b["grad"].append(g)
        b["param"].append(p.detach())
        b["master"].append(st.get("master"))
        b["params"].append(p)
        for name in moments:
            b.setdefault(name, []).append(st[name])
    return buckets


def _mtlist(opt, group_idx, key, roles):
    cache = opt.__dict__.setdefault("_mt_cache", {})
    lst = cache.get((group_idx, key))
    if lst is None:
        lst = cache[(group_idx, key)] = mt.MTList()
    return lst.set(**roles)


class FusedAdam(torch.optim.Optimizer):
    """Adam / AdamW (apex FusedAdam semantics), one multi-tensor launch per (group, dtype)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support amsgrad")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = adam_w_mode
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        super().zero_grad(set_to_none=self.set_grad_none if set_to_none is None else set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for gi, g in enumerate(self.param_groups):
            b1, b2 = g["betas"]
            g["step"] = g.get("step", 0) + 1
            bc1 = 1.0 - b1 ** g["step"] if g["bias_correction"] else 1.0
            bc2 = 1.0 - b2 ** g["step"] if g["bias_correction"] else 1.0
            for key, b in _lists(self, g, ("exp_avg", "exp_avg_sq")).items():
                master = b["master"][0] is not None
                if b["grad"][0].is_cuda:
                    lst = _mtlist(self, gi, key, dict(grad=b["grad"], param=b["param"],
                                                      master=b["master"] if master else None, m=b["exp_avg"],
                                                      v=b["exp_avg_sq"]))
                    meta, nt, nc = lst.meta(b["grad"][0].device)
                    mt.ext().mt_adam(meta, nt, nc, b["grad"][0], b["param"][0], master, g["lr"], b1, b2, g["eps"],
                                     g["weight_decay"], bc1, bc2, 1.0, self.adam_w_mode)
                    continue
                for i, gr in enumerate(b["grad"]):
                    ms = b["master"][i] if master else b["param"][i]
                    mt.fused_adam_(b["param"][i].view(-1) if master else None, gr.view(-1), ms.view(-1),
                                   b["exp_avg"][i].view(-1), b["exp_avg_sq"][i].view(-1), g["lr"], b1, b2, g["eps"],
                                   g["weight_decay"], g["step"], 1.0, adamw=self.adam_w_mode,
                                   bias_correction=g["bias_correction"])
        return loss


def _pp_sum_(x):
    """Sum a device scalar over the pipeline group when running under smp (the reference
    all-gathers the local gradient norms over PP_GROUP, `optimizers/fused_lamb.py`)."""
    try:
        from ..torch.state_mod import state
    except ImportError:  # pragma: no cover
        return x
    if state.initialized and state.core.pp_size() > 1 and state.pgs.pp is not None:
        dist.all_reduce(x, group=state.pgs.pp)
    return x


def _any_device(opt):
    """A device for this optimizer's collectives when it holds no gradient: a parameter's, else
    the current GPU, else the CPU."""
    for g in opt.param_groups:
        for p in g["params"]:
            return p.device
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class FusedLAMB(torch.optim.Optimizer):
    """LAMB (apex FusedLAMB + the reference's PP-global gradient norm): the gradient is divided
    by max(1, ||g||_global / max_grad_norm), stage 1 forms the Adam direction (+ decoupled or
    L2 weight decay), stage 2 applies it with the per-tensor trust ratio ||p|| / ||update||.
    Per step: 2 norm launches + 2 update launches per (group, dtype) and one PP all-reduce."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 amsgrad=False, adam_w_mode=True, grad_averaging=True, set_grad_none=True, max_grad_norm=1.0,
                 use_nvlamb=False):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support amsgrad")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.adam_w_mode = adam_w_mode
        self.use_nvlamb = use_nvlamb
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        super().zero_grad(set_to_none=self.set_grad_none if set_to_none is None else set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        groups = [(gi, g, _lists(self, g, ("exp_avg", "exp_avg_sq"))) for gi, g in enumerate(self.param_groups)]
        dev = next((b["grad"][0].device for _, _, bs in groups for b in bs.values()), None)
        if dev is None:
            # no local gradient (e.g. a pipeline stage whose parameters all went unused): still
            # join the pipeline-group norm all-reduce with a zero, as the reference's all-gather
            # does (`optimizers/fused_lamb.py:34-53`) -- the other stages are waiting in it
            _pp_sum_(torch.zeros(1, dtype=torch.float32, device=_any_device(self)))
            return loss
        # global gradient norm: every group, every dtype, then over the pipeline stages
        gsq = torch.zeros(1, dtype=torch.float32, device=dev)
        for gi, g, bs in groups:
            for key, b in bs.items():
                if dev.type == "cuda":
                    lst = _mtlist(self, gi, ("g",) + key, dict(grad=b["grad"]))
                    part = torch.zeros(lst.n, dtype=torch.float32, device=dev)
                    gsq += mt.mt_norms(lst, "grad", part).sum()
                else:
                    for gr in b["grad"]:
                        gsq += gr.float().pow(2).sum()
        gnorm = _pp_sum_(gsq).sqrt_()
        max_norm = self.defaults["max_grad_norm"]
        for gi, g, bs in groups:
            b1, b2 = g["betas"]
            b3 = 1.0 - b1 if g["grad_averaging"] else 1.0
            g["step"] = g.get("step", 0) + 1
            bc1 = 1.0 - b1 ** g["step"] if g["bias_correction"] else 1.0
            bc2 = 1.0 - b2 ** g["step"] if g["bias_correction"] else 1.0
            use_trust = self.use_nvlamb or g["weight_decay"] != 0
            for key, b in bs.items():
                master = b["master"][0] is not None
                mst = b["master"] if master else b["param"]
                upd = [torch.empty_like(x, dtype=torch.float32) for x in mst]
                if dev.type == "cuda":
                    lst = _mtlist(self, gi, key, dict(grad=b["grad"], param=b["param"],
                                                      master=b["master"] if master else None, m=b["exp_avg"],
                                                      v=b["exp_avg_sq"], update=upd))
                    meta, nt, nc = lst.meta(dev)
                    pn2 = mt.mt_norms(lst, "master" if master else "param", torch.zeros(nt, device=dev))
                    mt.ext().mt_lamb1(meta, nt, nc, b["grad"][0], b["param"][0], master, b1, b2, b3, bc1, bc2,
                                      g["eps"], g["weight_decay"], self.adam_w_mode, gnorm, max_norm, 1.0)
                    un2 = mt.mt_norms(lst, "update", torch.zeros(nt, device=dev))
                    mt.ext().mt_lamb2(meta, nt, nc, b["param"][0], master, pn2, un2, g["lr"], use_trust)
                    continue
                gn = float(gnorm)
                clip = gn / max_norm if (max_norm > 0 and gn > max_norm) else 1.0
                for i, gr in enumerate(b["grad"]):
                    p32, m, v = mst[i].float(), b["exp_avg"][i], b["exp_avg_sq"][i]
                    sg = gr.float() / clip
                    if not self.adam_w_mode:
                        sg = sg + g["weight_decay"] * p32
                    m.mul_(b1).add_(sg, alpha=b3)
                    v.mul_(b2).addcmul_(sg, sg, value=1 - b2)
                    u = (m / bc1) / ((v / bc2).sqrt() + g["eps"])
                    if self.adam_w_mode:
                        u = u + g["weight_decay"] * p32
                    pn, un = float(p32.norm()), float(u.norm())
                    ratio = g["lr"] * (pn / un) if (use_trust and pn != 0 and un != 0) else g["lr"]
                    mst[i].sub_(u.to(mst[i].dtype), alpha=ratio)
                    if master:
                        b["param"][i].copy_(mst[i])
        return loss


class FusedNovoGrad(torch.optim.Optimizer):
    """NovoGrad (apex FusedNovoGrad over `multi_tensor_novograd`): the second moment is a
    per-tensor gradient NORM (L2 or L-inf), blended as sqrt(b2 n_old^2 + (1 - b2) n^2) (L2) /
    b2 n_old + (1 - b2) n (L-inf) and initialised from the first step's norms (or zero);
    moment mode: ``reg_inside_moment`` puts weight decay inside the first moment, otherwise it
    is decoupled.  Per step: one norm launch, one blend launch and one update launch per
    (group, dtype) -- no host synchronisation."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, reg_inside_moment=False, grad_averaging=True, norm_type=2, init_zero=False,
                 set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedNovoGrad does not support the AMSGrad variant.")
        if norm_type not in (0, 2):
            raise RuntimeError("FusedNovoGrad only supports l2/inf norm now.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, norm_type=norm_type, init_zero=init_zero)
        super().__init__(params, defaults)
        self.moment_mode = 0 if reg_inside_moment else 1
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        super().zero_grad(set_to_none=self.set_grad_none if set_to_none is None else set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for gi, g in enumerate(self.param_groups):
            b1, b2 = g["betas"]
            b3 = 1.0 - b1 if g["grad_averaging"] else 1.0
            g["step"] = g.get("step", 0) + 1
            bc1 = 1.0 - b1 ** g["step"] if g["bias_correction"] else 1.0
            bc2 = 1.0 - b2 ** g["step"] if g["bias_correction"] else 1.0
            l2 = g["norm_type"] == 2
            norms_by_key = g.setdefault("exp_avg_sq", {})
            for key, b in _lists(self, g, ("exp_avg",)).items():
                master = b["master"][0] is not None
                dev = b["grad"][0].device
                nk = str(key)
                first = nk not in norms_by_key
                if first:
                    norms_by_key[nk] = torch.zeros(len(b["grad"]), dtype=torch.float32, device=dev)
                norms = norms_by_key[nk]
                lst = _mtlist(self, gi, key, dict(grad=b["grad"], param=b["param"],
                                                  master=b["master"] if master else None, m=b["exp_avg"]))
                fresh = mt.mt_norms(lst, "grad", torch.zeros(len(b["grad"]), dtype=torch.float32, device=dev),
                                    maxabs=not l2)
                if dev.type == "cuda":
                    mt.ext().novograd_blend(norms, fresh, b2, l2, first, g["init_zero"])
                    meta, nt, nc = lst.meta(dev)
                    mt.ext().mt_novograd(meta, nt, nc, b["grad"][0], b["param"][0], master, norms, b1, b3, bc1, bc2,
                                         g["eps"], g["lr"], g["weight_decay"], self.moment_mode == 1, 1.0)
                    continue
                n = fresh.sqrt() if l2 else fresh
                old = (torch.zeros_like(n) if g["init_zero"] else n) if first else norms
                norms.copy_((b2 * old * old + (1 - b2) * n * n).sqrt() if l2 else b2 * old + (1 - b2) * n)
                mst = b["master"] if master else b["param"]
                for i, gr in enumerate(b["grad"]):
                    p32, m = mst[i], b["exp_avg"][i]
                    denom = norms[i] / bc2 + g["eps"]
                    gf = gr.float()
                    if self.moment_mode == 0:
                        m.mul_(b1).add_(gf / denom + g["weight_decay"] * p32, alpha=b3)
                        p32.sub_(m / bc1, alpha=g["lr"])
                    else:
                        m.mul_(b1).add_(gf, alpha=b3)
                        p32.sub_((m / bc1) / denom + g["weight_decay"] * p32, alpha=g["lr"])
                    if master:
                        b["param"][i].copy_(p32)
        return loss


__all__ = ["DistributedOptimizer", "FusedAdam", "FusedLAMB", "FusedNovoGrad"]
