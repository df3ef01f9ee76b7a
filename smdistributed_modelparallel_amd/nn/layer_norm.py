"""LayerNorm modules.

* ``FusedLayerNorm`` / ``MixedFusedLayerNorm``: the HIP fused LayerNorm (apex replacement,
  reference `smp/torch/nn/layer_norm.py:140-152`).
* ``DistributedLayerNorm``: LayerNorm over a hidden dimension sharded across the TP group
  (``optimize="memory"`` layout; reference `layer_norm.py:24-135`): forward all-reduces the
  per-row mean and variance (fp32), backward all-reduces the two per-row partial sums.
"""
import numbers

import torch
import torch.nn as nn

from ..ops.layernorm import add_layer_norm, layer_norm, layer_norm_passthrough
from ..parallel.throttle import throttler
from .utils import get_local_channels, get_start_pos_for_slicing, tp_group, tp_size
from ..parallel import oneshot
from ..ops._ext import fused_ok


class FusedLayerNorm(nn.Module):
    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = tuple(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        n = 1
        for s in self.normalized_shape:
            n *= s
        if elementwise_affine:
            self.weight = nn.Parameter(torch.ones(n, device=device, dtype=dtype))
            self.bias = nn.Parameter(torch.zeros(n, device=device, dtype=dtype))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x):
        shape = x.shape
        y = layer_norm(x.reshape(-1, self.weight.numel() if self.weight is not None else shape[-1]), self.weight,
                       self.bias, self.eps)
        return y.view(shape)

    def reset_parameters(self):
        if self.weight is not None:
            with torch.no_grad():
                self.weight.fill_(1.0)
                self.bias.zero_()

    def forward_add(self, x, residual, dropout_p=0.0, drawn=None):
        """(LN(dropout(x) + residual), dropout(x) + residual) in one kernel."""
        return add_layer_norm(x, residual, self.weight, self.bias, self.eps, dropout_p, drawn)

    def forward_passthrough(self, x):
        """(LN(x), x) where x's two gradient paths (LN input, residual branch) are summed
        inside the LN backward kernel."""
        if type(self).forward is not FusedLayerNorm.forward or len(self.normalized_shape) != 1:
            return self(x), x
        return layer_norm_passthrough(x, self.weight, self.bias, self.eps)

    def extra_repr(self):
        return f"{self.normalized_shape}, eps={self.eps}, elementwise_affine={self.elementwise_affine}"


class MixedFusedLayerNorm(FusedLayerNorm):
    """apex ``MixedFusedLayerNorm`` (reference `smp/torch/apex/normalization/
    fused_layer_norm.py:198-218`, K10): input of any dtype, output in the parameters' dtype,
    written directly by the LayerNorm kernel."""

    def forward(self, x):
        if self.weight is None or len(self.normalized_shape) != 1:
            y = super().forward(x)
            return y.to(self.weight.dtype) if self.weight is not None else y
        from ..ops.layernorm import mixed_layer_norm

        return mixed_layer_norm(x, self.weight, self.bias, self.eps)


class _DistLNStats(torch.autograd.Function):
    """Global mean/var over a TP-sharded last dim (fp32), with the matching backward."""

    @staticmethod
    def forward(ctx, x, full_dim, group):
        xf = x.float()
        s1 = xf.sum(-1, keepdim=True)
        if group is not None:
            with throttler().throttle(s1):
                oneshot.all_reduce(s1, group=group)
        mean = s1 / full_dim
        s2 = (xf - mean).pow(2).sum(-1, keepdim=True)
        if group is not None:
            with throttler().throttle(s2):
                oneshot.all_reduce(s2, group=group)
        var = s2 / full_dim
        ctx.save_for_backward(xf, mean)
        ctx.full_dim, ctx.group = full_dim, group
        return mean, var

    @staticmethod
    def backward(ctx, gmean, gvar):
        xf, mean = ctx.saved_tensors
        n = ctx.full_dim
        if ctx.group is not None:
            # every rank's local y depends on the shared statistics: sum their grads
            g = torch.cat([gmean, gvar], dim=-1).contiguous()
            with throttler().throttle(g):
                oneshot.all_reduce(g, group=ctx.group)
            gmean, gvar = g[..., :1], g[..., 1:]
        # d mean / dx = 1/n ; d var / dx = 2 (x - mean) / n  (the mean term sums to zero)
        gx = gmean / n + gvar * 2.0 * (xf - mean) / n
        return gx, None, None


class _DistLayerNormHIP(torch.autograd.Function):
    """GPU form of the TP-sharded LayerNorm: native kernels K6-K8 (`csrc/kernels/layernorm.hip`)
    around two [rows, k] fp32 all-reduces; inputs stay in their dtype (no fp32 upcast of the
    activation), one all-reduce in each direction (reference `layer_norm.py:24-102` uses two
    in the forward)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, full_dim, group):
        from ..ops._ext import ext

        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        st = ext().layernorm_local_stats(x2)  # (n*m, M2, n*m*m) per row of the local shard
        if group is not None:
            with throttler().throttle(st):
                oneshot.all_reduce(st, group=group)
        n = float(full_dim)
        mean = st[:, 0] / n
        var = ((st[:, 1] + st[:, 2]) / n - mean * mean).clamp_min_(0.0)  # Chan's combination
        rstd = torch.empty_like(mean)
        y = ext().layernorm_apply_stats(x2, weight, bias, mean.contiguous(), var.contiguous(), rstd, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.shape, ctx.full_dim, ctx.group = shape, full_dim, group
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        from ..ops._ext import ext

        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape).contiguous()
        sums = ext().layernorm_bwd_local_sums(dy2, x2, w, mean, rstd)  # (sum g, sum g*xhat) local
        if ctx.group is not None:
            with throttler().throttle(sums):
                oneshot.all_reduce(sums, group=ctx.group)
        need_w = ctx.has_w and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        dx, dw, db = ext().layernorm_bwd(dy2, x2, w, mean, rstd, need_w, need_b, None, ext_sums=sums,
                                         ext_n=float(ctx.full_dim))
        return dx.view(ctx.shape), (dw if need_w else None), (db if need_b else None), None, None, None


class DistributedLayerNorm(nn.Module):
    """LayerNorm whose normalised dim is split across the TP group (uneven splits ok)."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (normalized_shape,)
        self.full_dim = normalized_shape[-1]
        self.local_dim = get_local_channels(self.full_dim)
        self.start = get_start_pos_for_slicing(self.full_dim)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if elementwise_affine:
            self.weight = nn.Parameter(torch.ones(self.local_dim, device=device, dtype=dtype))
            self.bias = nn.Parameter(torch.zeros(self.local_dim, device=device, dtype=dtype))
            self.weight._smp_scaled_batch = True
            self.bias._smp_scaled_batch = True
            from .utils import mark_tp

            mark_tp(self.weight, 0)
            mark_tp(self.bias, 0)
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def reset_parameters(self):
        if self.weight is not None:
            with torch.no_grad():
                self.weight.fill_(1.0)
                self.bias.zero_()

    def forward(self, x):
        group = tp_group() if tp_size() > 1 else None
        if fused_ok(x) and x.dtype in (torch.bfloat16, torch.float16, torch.float32):
            return _DistLayerNormHIP.apply(x, self.weight, self.bias, self.eps, self.full_dim, group)
        mean, var = _DistLNStats.apply(x, self.full_dim, group)
        y = (x.float() - mean) * torch.rsqrt(var + self.eps)
        if self.weight is not None:
            y = y * self.weight.float() + self.bias.float()
        return y.to(x.dtype)
