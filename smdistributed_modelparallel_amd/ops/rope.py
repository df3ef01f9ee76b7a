"""Rotary position embeddings (K18): GPT-J interleaved pairs and GPT-NeoX half rotation
(reference `smp/torch/nn/transformer.py:114-182,1565-1615`).

x layout ``[b, s, h, d]``; only the first ``rotary_dim`` channels rotate.  cos/sin
tables are built once per (seq, dim, base, device) in fp32 (precomputed tables rather
than on-device trig, per the elementwise guidance for CDNA).
"""
import torch
from ._ext import fused_ok

_cache = {}
PACKED_CALLS = [0]  # GPU in-place packed-QKV rotations (tests check the fast path engaged)


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
    if fused_ok(x) and x.dtype in (torch.float16, torch.bfloat16, torch.float32) and x.stride(-1) == 1 \
            and rotary_dim % 2 == 0:
        s = x.shape[1]
        cos, sin = rope_tables(s + offset, rotary_dim, base, x.device, 0)
        return _RopeHIP.apply(x, cos.contiguous(), sin.contiguous(), rotary_dim, neox_style, offset)
    return apply_rotary_torch(x, rotary_dim, base, neox_style, offset)


class _RopeQKVHIP(torch.autograd.Function):
    """Rotary on the q / k parts of the packed QKV projection output ``y`` [b, s, 3 h d], IN
    PLACE and on the rotary channels only (v and the pass-through channels are not touched), so
    the attention takes its packed path and its backward hands back one dqkv buffer, which is
    rotated back in place.  Rotating q and k as separate views made autograd build a zero-filled
    [b, s, 3, h, d] gradient per view and add the three (GPT-J TP4 / NeoX PP2xTP4 shard traces:
    ~250 us per layer of fills, copies and adds, profiles/r5/shards_r5.md).  ``y`` must be a
    non-view tensor that no other autograd node saved (a linear layer's output: its backward
    keeps the input and the weight); its gradient is rotated back in place only when its
    producer marked it a fresh buffer (``_smp_fresh_grad``, set by the packed attention)."""

    @staticmethod
    def forward(ctx, y, cos, sin, rotary_dim, neox, offset, batch, seq, heads, d):
        from ._ext import ext

        ctx.save_for_backward(cos, sin)
        ctx.args = (rotary_dim, neox, offset, batch, seq, heads, d)
        y5 = y.view(batch, seq, 3, heads, d)
        C = ext()
        for part in (0, 1):
            C.rope_apply_into(y5[:, :, part], y5[:, :, part], cos, sin, rotary_dim, neox, False, offset, False)
        ctx.mark_dirty(y)
        return y

    @staticmethod
    def backward(ctx, g):
        from ._ext import ext

        cos, sin = ctx.saved_tensors
        rd, neox, offset, batch, seq, heads, d = ctx.args
        # rotated back in place when the producer declared the buffer its own fresh allocation
        # (the packed attention's dqkv, seen here through the view); any other gradient -- e.g.
        # one a caller passed to backward() -- is copied first
        owner = g._base if g._base is not None else g
        if not (g.is_contiguous() and getattr(owner, "_smp_fresh_grad", False)):
            g = g.clone(memory_format=torch.contiguous_format)
        g5 = g.view(batch, seq, 3, heads, d)
        C = ext()
        for part in (0, 1):
            C.rope_apply_into(g5[:, :, part], g5[:, :, part], cos, sin, rd, neox, True, offset, False)
        return g, None, None, None, None, None, None, None, None, None


def apply_rotary_qkv(y, batch, seq, heads, head_dim, rotary_dim, base=10000, neox_style=False, offset=0):
    """Packed QKV projection output ``y`` (batch * seq * 3 * heads * head_dim elements, e.g. the
    2-D [batch * seq, 3 * heads * head_dim] output of a linear layer) -> [batch, seq, 3, heads,
    head_dim] with rotary applied to q and k.  GPU: in place on ``y``, which must then be a
    contiguous non-view tensor (a 2-D linear output is; a 3-D one is a view of the GEMM's 2-D
    result) -- otherwise the out-of-place torch path runs."""
    if rotary_dim is None or rotary_dim == 0:
        return y.view(batch, seq, 3, heads, head_dim)
    if fused_ok(y) and y.dtype in (torch.float16, torch.bfloat16, torch.float32) and y.is_contiguous() \
            and rotary_dim % 2 == 0 and y._base is None:
        cos, sin = rope_tables(seq + offset, rotary_dim, base, y.device, 0)
        PACKED_CALLS[0] += 1
        out = _RopeQKVHIP.apply(y, cos.contiguous(), sin.contiguous(), rotary_dim, neox_style, offset, batch, seq,
                                heads, head_dim)
        return out.view(batch, seq, 3, heads, head_dim)
    y5 = y.view(batch, seq, 3, heads, head_dim)
    q = apply_rotary_torch(y5[:, :, 0], rotary_dim, base, neox_style, offset)
    k = apply_rotary_torch(y5[:, :, 1], rotary_dim, base, neox_style, offset)
    return torch.stack((q, k, y5[:, :, 2]), dim=2)


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
