"""Dropout on the GPU without mask tensors.

Every dropout decision comes from a counter hash of (seed, offset, element index) --
`csrc/kernels/common.h` (element-wise) and `attention_impl.h` (attention probabilities) --
so the forward writes no mask and the backward regenerates the decisions from the two
integers saved on the autograd context.  (seed, offset) are drawn from the device
generator like a philox consumer: ``torch.manual_seed``, the TP-consistent RNG fork
(`parallel/random.py`) and activation-checkpoint RNG replay all apply.

Fused forms used by the transformer (reference `smp/torch/nn/transformer.py:449,1143,1524`):
* ``dropout_add(x, residual, p)``: residual + dropout(x) in one pass;
* ``add3(a, b, c)``: the dropout-free parallel-attention residual sum in one pass;
* ``add_layer_norm(..., dropout_p)`` (ops/layernorm.py): the attention-branch dropout and
  residual add run inside the LayerNorm kernel that follows them.
CPU tensors use ``torch.nn.functional.dropout``.
"""
import torch

from ._ext import ext, fused_ok
def dropout_seed_offset(device, increment=4):
    """(seed, offset) for the in-kernel dropout hash, advanced like a philox consumer; no
    device synchronisation."""
    if device.type == "cuda":
        idx = device.index if device.index is not None else torch.cuda.current_device()
        gen = torch.cuda.default_generators[idx]
        seed, off = gen.initial_seed(), gen.get_offset()
        gen.set_offset(off + increment)
        return int(seed) & ((1 << 63) - 1), int(off)
    return int(torch.randint(0, 1 << 62, (1,)).item()), 0


def _aligned(t):
    return t.data_ptr() % 16 == 0


class _DropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, p):
        seed, off = dropout_seed_offset(x.device)
        x2 = x.contiguous()
        r2 = residual.contiguous() if residual is not None else None
        if not _aligned(x2):
            x2 = x2.clone()
        if r2 is not None and not _aligned(r2):
            r2 = r2.clone()
        ctx.drop = (p, seed, off)
        ctx.has_res = residual is not None
        return ext().dropout_add(x2, r2, p, seed, off).view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        p, seed, off = ctx.drop
        dy2 = dy.contiguous()
        if not _aligned(dy2):
            dy2 = dy2.clone()
        dx = ext().dropout_bwd(dy2, p, seed, off).view(dy.shape)
        return dx, (dy if ctx.has_res else None), None


def dropout_add(x, residual, p, training=True):
    """residual + dropout(x, p) (residual may be None)."""
    if not training or p == 0.0:
        return x if residual is None else x + residual
    if not fused_ok(x) or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        y = torch.nn.functional.dropout(x, p, True)
        return y if residual is None else y + residual
    return _DropoutAdd.apply(x, residual, float(p))


class _Add3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c):
        return ext().add3(a, b, c)

    @staticmethod
    def backward(ctx, dy):
        return dy, dy, dy


def add3(a, b, c):
    """a + b + c in one pass over HBM (3 reads + 1 write instead of two adds' 4 reads + 2
    writes): the parallel-attention residual sum hidden + attn + mlp (GPT-J / NeoX layers,
    reference `smp/torch/nn/transformer.py` parallel_attention path).  Falls back to two adds
    for CPU tensors, mixed dtypes/shapes or non-contiguous / unaligned inputs."""
    ts = (a, b, c)
    if (fused_ok(a) and a.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and all(t.dtype == a.dtype and t.shape == a.shape and t.is_contiguous() and _aligned(t) for t in ts)):
        return _Add3.apply(a, b, c)
    return a + b + c


def dropout(x, p, training=True):
    return dropout_add(x, None, p, training)


def dropout_keep_reference(n, p, seed, offset, device="cpu"):
    """Host reconstruction of the element-wise keep factors (0 or 1/(1-p)) for elements
    0..n-1: test oracle for common.h dropout_key / dropout_factors8."""
    M = 0xFFFFFFFF

    def mix(x):
        x = x ^ (x >> 16)
        x = (x * 0x7FEB352D) & M
        x = x ^ (x >> 15)
        x = (x * 0x846CA68B) & M
        return x ^ (x >> 16)

    thr = max(1, min(65535, int(p * 65536.0 + 0.5)))
    s0, s1, o0, o1 = seed & M, (seed >> 32) & M, offset & M, (offset >> 32) & M
    t = lambda v: torch.tensor(v, dtype=torch.int64)  # noqa: E731
    key = mix(t(s0) ^ mix(t((s1 + 0x27D4EB2F) & M)) ^ mix(t(o0) ^ mix(t((o1 + 0x165667B1) & M))))
    e = torch.arange(n, dtype=torch.int64, device=device)
    hi = ((e >> 33) * 0x9E3779B1) & M
    h = mix((key.to(device) ^ hi ^ ((e >> 1) & M)) & M)
    u = torch.where((e & 1) == 1, h >> 16, h & 0xFFFF)
    return (u >= thr).float() / (1.0 - p)
