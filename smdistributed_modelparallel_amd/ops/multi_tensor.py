"""Fused optimizer / reduction kernels over flat contiguous ranges (K12-K16, K20).

GPU: one HIP kernel per call.  CPU: reference PyTorch math (test target).
"""
import math

import torch

from ._ext import ext


def fused_adam_(param_lowp, grad, master, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0,
                adamw=True, bias_correction=True):
    """Updates master/m/v in place (fp32) and writes param_lowp (if given) in the same pass."""
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    if master.is_cuda:
        ext().fused_adam(param_lowp, grad, master, m, v, lr, beta1, beta2, eps, weight_decay, bc1, bc2,
                         grad_scale, adamw)
        return
    g = grad.float() * grad_scale
    if adamw:
        master.mul_(1.0 - lr * weight_decay)
    else:
        g = g + weight_decay * master
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)
    if param_lowp is not None:
        param_lowp.copy_(master)


def fused_sgd_(param_lowp, grad, master, mom, lr, momentum, dampening, weight_decay, nesterov, first, grad_scale=1.0):
    if master.is_cuda:
        ext().fused_sgd(param_lowp, grad, master, mom, lr, momentum, dampening, weight_decay, nesterov, first,
                        grad_scale)
        return
    g = grad.float() * grad_scale + weight_decay * master
    if momentum != 0.0:
        if first:
            mom.copy_(g)
        else:
            mom.mul_(momentum).add_(g, alpha=1.0 - dampening)
        g = g + momentum * mom if nesterov else mom
    master.add_(g, alpha=-lr)
    if param_lowp is not None:
        param_lowp.copy_(master)


def fused_adagrad_(param_lowp, grad, master, state_sum, lr, eps, weight_decay, grad_scale=1.0):
    if master.is_cuda:
        ext().fused_adagrad(param_lowp, grad, master, state_sum, lr, eps, weight_decay, grad_scale)
        return
    g = grad.float() * grad_scale + weight_decay * master
    state_sum.addcmul_(g, g)
    master.addcdiv_(g, state_sum.sqrt().add_(eps), value=-lr)
    if param_lowp is not None:
        param_lowp.copy_(master)


def lamb_stage1_(grad, master, m, v, update, beta1, beta2, eps, weight_decay, step, grad_scale=1.0,
                 bias_correction=True):
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    if master.is_cuda:
        ext().lamb_stage1(grad, master, m, v, update, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale)
        return
    g = grad.float() * grad_scale
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    update.copy_((m / bc1) / ((v / bc2).sqrt() + eps) + weight_decay * master)


def lamb_stage2_(param_lowp, master, update, lr, p_norm_sq, u_norm_sq, use_trust=True):
    if master.is_cuda:
        ext().lamb_stage2(param_lowp, master, update, lr, p_norm_sq, u_norm_sq, use_trust)
        return
    trust = 1.0
    if use_trust:
        a, b = float(p_norm_sq.sqrt()), float(u_norm_sq.sqrt())
        trust = a / b if (a > 0 and b > 0) else 1.0
    master.add_(update, alpha=-lr * trust)
    if param_lowp is not None:
        param_lowp.copy_(master)


LAMB_CHUNK = 1 << 16


def lamb_chunk_table(pieces, device):
    """pieces: [(start, end)] element ranges (one per parameter piece, relative to the
    domain) -> int64 [n, 3] (segment, start, end) table of <= LAMB_CHUNK-element chunks."""
    rows = []
    for seg, (s, e) in enumerate(pieces):
        for c in range(s, e, LAMB_CHUNK):
            rows.append((seg, c, min(c + LAMB_CHUNK, e)))
    return torch.tensor(rows, dtype=torch.int64, device=device).view(-1, 3)


def lamb_segmented_(param_lowp, master, update, chunks, nseg, lr, use_trust=True):
    """LAMB stage 2 over a whole domain: each segment (parameter piece) gets its own trust
    ratio |p| / |update|, all in two kernel launches (no per-parameter host loop)."""
    if master.is_cuda:
        ext().lamb_chunked_(param_lowp, master, update, chunks, nseg, lr, use_trust)
        return
    norms = torch.zeros(nseg, 2)
    for seg, s, e in chunks.tolist():
        norms[seg, 0] += master[s:e].pow(2).sum()
        norms[seg, 1] += update[s:e].pow(2).sum()
    a, b = norms[:, 0].sqrt(), norms[:, 1].sqrt()
    trust = torch.where((a > 0) & (b > 0), a / b, torch.ones_like(a)) if use_trust else torch.ones_like(a)
    for seg, s, e in chunks.tolist():
        master[s:e].add_(update[s:e], alpha=-lr * float(trust[seg]))
        if param_lowp is not None:
            param_lowp[s:e].copy_(master[s:e])


def sumsq(x, out=None, scale=1.0):
    """Accumulates sum(x^2) * scale^2 into `out` (fp32 1-element tensor) and returns it."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.numel() == 0:
        return out
    if x.is_cuda:
        ext().sumsq_(x.contiguous(), out, scale)
    else:
        out += (x.float() * scale).pow(2).sum()
    return out


def nonfinite_flag(x, out=None):
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.numel() == 0:
        return out
    if x.is_cuda:
        ext().nonfinite_(x.contiguous(), out)
    else:
        if not torch.isfinite(x).all():
            out.fill_(1.0)
    return out


def axpby_(x, y, a, b):
    if y.is_cuda:
        ext().axpby_(x, y, a, b)
    else:
        y.mul_(b).add_(x, alpha=a)
    return y


def cast_copy_(src, dst, scale=1.0):
    if dst.is_cuda:
        ext().cast_copy_(src, dst, scale)
    else:
        dst.copy_(src.float() * scale if scale != 1.0 else src)
    return dst


# ------------------------------------------------------------------ multi-tensor apply
MT_CHUNK = 1 << 16  # elements per block (apex: 2048 x 32)
MT_ROLES = ("grad", "param", "master", "m", "v", "update")


class MTList:
    """A list of tensors for one multi-tensor launch (amp_C ``multi_tensor_applier``): role
    name -> list of tensors (same length; None = role absent).  On the GPU the role pointers
    and the <= 64K-element chunk table travel in one int64 tensor (`optim.hip` meta layout);
    it is rebuilt only when a pointer changed (gradients set to None re-allocate)."""

    __slots__ = ("roles", "n", "numel", "_key", "_meta", "_nchunks", "_host")

    def __init__(self):
        self._key = None
        self._meta = None
        self._host = None

    def set(self, **roles):
        self.roles = roles
        first = next(iter(roles.values()))
        self.n = len(first)
        self.numel = [t.numel() for t in first]
        return self

    def meta(self, device):
        ptrs = []
        for r in MT_ROLES:
            lst = self.roles.get(r)
            ptrs.extend([0] * self.n if lst is None else [0 if t is None else t.data_ptr() for t in lst])
        key = tuple(ptrs)
        if key != self._key:
            import numpy as np

            chunks = []
            for ti, n in enumerate(self.numel):
                st = np.arange(0, n, MT_CHUNK, dtype=np.int64)
                chunks.append(np.stack([np.full_like(st, ti), st, np.minimum(st + MT_CHUNK, n)], axis=1))
            table = np.concatenate(chunks) if chunks else np.zeros((0, 3), dtype=np.int64)
            host = np.concatenate([np.array(ptrs, dtype=np.uint64).view(np.int64), table.reshape(-1)])
            # pinned staging kept alive on the object until the next rebuild (async upload)
            self._host = torch.from_numpy(host).pin_memory()
            self._meta = self._host.to(device, non_blocking=True)
            self._nchunks = int(table.shape[0])
            self._key = key
        return self._meta, self.n, self._nchunks


def mt_norms(lst, role, out, maxabs=False, scale=1.0):
    """Per-tensor sum of squares (or max |x|) of `role` accumulated into out[t] (fp32)."""
    tensors = lst.roles[role]
    if out.is_cuda:
        meta, nt, nc = lst.meta(out.device)
        ext().mt_norm(meta, nt, nc, MT_ROLES.index(role), tensors[0], out, scale, maxabs)
        return out
    for i, t in enumerate(tensors):
        x = t.float() * scale
        out[i] = torch.maximum(out[i], x.abs().max()) if maxabs else out[i] + x.pow(2).sum()
    return out
