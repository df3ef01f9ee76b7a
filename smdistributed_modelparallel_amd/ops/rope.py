"""Rotary position embeddings (K18): GPT-J interleaved pairs and GPT-NeoX half rotation
(reference `smp/torch/nn/transformer.py:114-182,1565-1615`).

x layout ``[b, s, h, d]``; only the first ``rotary_dim`` channels rotate.  cos/sin
tables are built once per (seq, dim, base, device) in fp32 (precomputed tables rather
than on-device trig, per the elementwise guidance for CDNA).
"""
import torch

_cache = {}


def rope_tables(seq_len, rotary_dim, base, device, offset=0):
    key = (seq_len + offset, rotary_dim, base, device)
    t = _cache.get(key)
    if t is None:
        inv = 1.0 / (base ** (torch.arange(0, rotary_dim, 2, dtype=torch.float32, device=device) / rotary_dim))
        pos = torch.arange(seq_len + offset, dtype=torch.float32, device=device)
        f = torch.outer(pos, inv)
        t = (f.cos(), f.sin())
        _cache[key] = t
    cos, sin = t
    return cos[offset: offset + seq_len], sin[offset: offset + seq_len]


def _rotate_every_two(x):
    x1 = x[..., ::2]
    x2 = x[..., 1::2]
    return torch.stack((-x2, x1), dim=-1).flatten(-2)


def _rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


class _RopeHIP(torch.autograd.Function):
    """HIP kernel (csrc/kernels/rope.hip): reads q/k straight from their strided views into
    the packed QKV projection; backward is the inverse rotation of the gradient."""

    @staticmethod
    def forward(ctx, x, cos, sin, rotary_dim, neox, offset):
        from ._ext import ext

        ctx.save_for_backward(cos, sin)
        ctx.args = (rotary_dim, neox, offset)
        return ext().rope_apply(x, cos, sin, rotary_dim, neox, False, offset)

    @staticmethod
    def backward(ctx, g):
        from ._ext import ext

        cos, sin = ctx.saved_tensors
        rd, neox, offset = ctx.args
        g = g if g.stride(-1) == 1 else g.contiguous()
        return ext().rope_apply(g, cos, sin, rd, neox, True, offset), None, None, None, None, None


def apply_rotary(x, rotary_dim, base=10000, neox_style=False, offset=0):
    """Returns a new tensor with rotary applied (autograd-friendly)."""
    if rotary_dim is None or rotary_dim == 0:
        return x
    if x.is_cuda and x.dtype in (torch.float16, torch.bfloat16, torch.float32) and x.stride(-1) == 1 \
            and rotary_dim % 2 == 0:
        s = x.shape[1]
        cos, sin = rope_tables(s + offset, rotary_dim, base, x.device, 0)
        return _RopeHIP.apply(x, cos.contiguous(), sin.contiguous(), rotary_dim, neox_style, offset)
    return apply_rotary_torch(x, rotary_dim, base, neox_style, offset)


class _RopeQKVHIP(torch.autograd.Function):
    """Rotary on the q / k parts of a packed [b, s, 3, h, d] QKV projection, returning a packed
    tensor (v copied), so the attention runs on its packed path and the backward hands back ONE
    dqkv buffer.  Rotating q and k as separate views made autograd materialise a zero-filled
    [b, s, 3, h, d] gradient per view and add the three (GPT-J TP4 / NeoX PP2xTP4 shard traces:
    ~250 us per layer of fills, copies and adds, profiles/r5/shards_r5.md)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, rotary_dim, neox, offset):
        from ._ext import ext

        ctx.save_for_backward(cos, sin)
        ctx.args = (rotary_dim, neox, offset)
        out = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        C = ext()
        C.rope_apply_into(qkv[:, :, 0], out[:, :, 0], cos, sin, rotary_dim, neox, False, offset)
        C.rope_apply_into(qkv[:, :, 1], out[:, :, 1], cos, sin, rotary_dim, neox, False, offset)
        out[:, :, 2].copy_(qkv[:, :, 2])
        return out

    @staticmethod
    def backward(ctx, g):
        from ._ext import ext

        cos, sin = ctx.saved_tensors
        rd, neox, offset = ctx.args
        if g.stride(-1) != 1:
            g = g.contiguous()
        dqkv = torch.empty(g.shape, dtype=g.dtype, device=g.device)
        C = ext()
        C.rope_apply_into(g[:, :, 0], dqkv[:, :, 0], cos, sin, rd, neox, True, offset)
        C.rope_apply_into(g[:, :, 1], dqkv[:, :, 1], cos, sin, rd, neox, True, offset)
        dqkv[:, :, 2].copy_(g[:, :, 2])
        return dqkv, None, None, None, None, None


def apply_rotary_qkv(qkv, rotary_dim, base=10000, neox_style=False, offset=0):
    """Packed [b, s, 3, h, d] QKV -> packed tensor with rotary applied to q and k."""
    if rotary_dim is None or rotary_dim == 0:
        return qkv
    if qkv.is_cuda and qkv.dtype in (torch.float16, torch.bfloat16, torch.float32) and qkv.stride(-1) == 1 \
            and rotary_dim % 2 == 0:
        s = qkv.shape[1]
        cos, sin = rope_tables(s + offset, rotary_dim, base, qkv.device, 0)
        return _RopeQKVHIP.apply(qkv, cos.contiguous(), sin.contiguous(), rotary_dim, neox_style, offset)
    q = apply_rotary_torch(qkv[:, :, 0], rotary_dim, base, neox_style, offset)
    k = apply_rotary_torch(qkv[:, :, 1], rotary_dim, base, neox_style, offset)
    return torch.stack((q, k, qkv[:, :, 2]), dim=2)


def apply_rotary_torch(x, rotary_dim, base=10000, neox_style=False, offset=0):
    """Plain torch implementation (CPU path and the numerics reference)."""
    if rotary_dim is None or rotary_dim == 0:
        return x
    b, s, h, d = x.shape
    cos, sin = rope_tables(s, rotary_dim, base, x.device, offset)
    rot, rest = x[..., :rotary_dim], x[..., rotary_dim:]
    if neox_style:
        c = torch.cat((cos, cos), dim=-1).view(1, s, 1, rotary_dim)
        sn = torch.cat((sin, sin), dim=-1).view(1, s, 1, rotary_dim)
        out = rot.float() * c + _rotate_half(rot.float()) * sn
    else:
        c = cos.repeat_interleave(2, dim=-1).view(1, s, 1, rotary_dim)
        sn = sin.repeat_interleave(2, dim=-1).view(1, s, 1, rotary_dim)
        out = rot.float() * c + _rotate_every_two(rot.float()) * sn
    out = out.to(x.dtype)
    if rest.shape[-1] == 0:
        return out
    return torch.cat((out, rest), dim=-1)
