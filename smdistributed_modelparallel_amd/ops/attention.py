"""Attention core.

Inputs/outputs use the ``[batch, seq, heads, head_dim]`` layout that falls out of the
fused QKV GEMM without a permute copy.

GPU paths:
* flash (default, ``amd_fused_attention``): the HIP MFMA kernel in
  ``csrc/kernels/attention.hip`` -- online softmax, no ``[s, s]`` score tensor, causal
  block skipping, no sequence-length cap;
* materialised: QK^T GEMM + the fused scaled (masked / causal) softmax kernel + PV GEMM
  (the reference's fused-softmax path, `transformer.py:1617-1835`).
CPU: PyTorch reference math.
"""
import math
import os

import torch

from . import softmax as _sm
from ._ext import ext, fused_ok
from .dropout import dropout_seed_offset  # noqa: F401  (re-exported)

_FLASH_OK = None
FLASH_HEAD_DIMS = (64, 96, 128, 256)


class KeyBias:
    """Additive per-key bias [b|1, sk] (float32).  The kernels test each 64-key tile for a
    nonzero entry as they stage it (one ballot) and skip the bias work on all-zero tiles, so
    an all-ones padding mask costs nothing but the 256-byte staging per tile."""

    __slots__ = ("bias",)

    def __init__(self, bias):
        self.bias = bias.float().contiguous()


def key_padding_bias(mask, sq, sk, mask_value=-1e4):
    """A [b|1, 1, sq, sk] bool/uint8 mask (True = masked) that only depends on the key
    (the usual padding mask, expanded over queries) -> KeyBias (additive mask_value on
    masked keys); None when the mask varies over queries (the kernel then cannot take it).
    Cached on the mask tensor: every layer of a forward pass shares one conversion."""
    if mask is None:
        return None
    cached = getattr(mask, "_smp_kbias", None)
    if cached is not None and cached[0] == (sk, mask_value):
        return cached[1]
    if mask.dim() != 4 or mask.shape[1] != 1 or mask.shape[-1] != sk:
        return None
    if mask.shape[2] != 1 and mask.stride(2) != 0:
        if not bool((mask == mask[:, :, :1]).all()):  # one host sync for non-expanded masks
            return None
    row = mask[:, 0, 0, :]
    if row.dtype not in (torch.bool, torch.uint8):
        kb = KeyBias(row)  # already additive
    else:
        kb = KeyBias(torch.zeros(row.shape, dtype=torch.float32, device=row.device).masked_fill_(row.bool(),
                                                                                              mask_value))
    try:
        mask._smp_kbias = ((sk, mask_value), kb)
    except (AttributeError, RuntimeError):  # pragma: no cover
        pass
    return kb


def flash_supported(q, dropout_p=0.0, mask=None, kbias=None):
    """Flash kernel covers bf16/fp16, head dims 64/96/128/256, in-kernel dropout, causal /
    sliding-window masks and per-key additive masks (padding)."""
    global _FLASH_OK
    if not fused_ok(q) or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    if q.shape[-1] not in FLASH_HEAD_DIMS:
        return False
    if mask is not None and kbias is None:
        return False
    if _FLASH_OK is None:
        _FLASH_OK = hasattr(ext(), "attention_fwd")
    return _FLASH_OK


def _mix32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    return x ^ (x >> 16)


def flash_dropout_threshold(dropout_p):
    """(lo, frac) of the flash kernels' dropout: an element is dropped iff its 8-bit uniform is
    below a threshold that each 32-query x 32-key block draws from {lo, lo + 1}, lo + 1 with
    probability frac / 65536 -- so every element is dropped with probability
    (lo + frac / 65536) / 256 = dropout_p to 2^-24 (``bindings.cpp`` attn_params)."""
    x = dropout_p * 256.0
    lo = int(x)
    frac = int((x - lo) * 65536.0 + 0.5)
    if frac >= 65536:
        lo, frac = lo + 1, 0
    return lo, frac


def flash_dropout_keep_prob(dropout_p):
    lo, frac = flash_dropout_threshold(dropout_p)
    return 1.0 - (lo + frac / 65536.0) / 256.0


def flash_dropout_keep_mask(b, h, sq, sk, dropout_p, seed, offset, device="cpu"):
    """Host reconstruction of the kernel's dropout decisions ([b, h, sq, sk] bool, True =
    kept): test oracle for the in-kernel hash (csrc/kernels/attention_impl.h drop_key / mix32 /
    drop_block_thr): byte ``k % 4`` of ``mix32(key ^ (q * ceil(sk / 4) + k // 4))`` is key k's
    8-bit uniform; the threshold of block (q // 32, k // 32) is lo + 1 iff the low 16 bits of
    ``mix32(mix32(key + 0x632be5ab) ^ (q // 32 * ceil(sk / 32) + k // 32))`` are below frac."""
    M = 0xFFFFFFFF
    lo, frac = flash_dropout_threshold(dropout_p)
    s0, s1, o0, o1 = seed & M, (seed >> 32) & M, offset & M, (offset >> 32) & M
    bh = torch.arange(b * h, dtype=torch.int64, device=device)
    key = _mix32(torch.full_like(bh, s0) ^ _mix32((s1 + 0x9E3779B9 * (bh + 1)) & M) ^
                 _mix32(torch.full_like(bh, o0) ^ _mix32(torch.full_like(bh, (o1 + 0x85EBCA6B) & M))))
    bkey = _mix32((key + 0x632BE5AB) & M)
    nquads = (sk + 3) // 4
    nkb = (sk + 31) // 32
    q = torch.arange(sq, dtype=torch.int64, device=device).view(1, -1, 1)
    k = torch.arange(sk, dtype=torch.int64, device=device).view(1, 1, -1)
    x = (key.view(-1, 1, 1) ^ ((q * nquads + (k >> 2)) & M)) & M
    hsh = _mix32(x)
    u = (hsh >> (8 * (k & 3))) & 0xFF
    g = _mix32((bkey.view(-1, 1, 1) ^ (((q >> 5) * nkb + (k >> 5)) & M)) & M)
    thr = lo + ((g & 0xFFFF) < frac).to(torch.int64)
    return (u >= thr).view(b, h, sq, sk)


# forward launches of the flash kernels by variant, for run reports (bench.py "attention_calls":
# a pipeline stage whose padding masks were decided all-ones launches no key-bias variant)
FLASH_CALLS = {"plain": 0, "key_bias": 0}


# Per-layer budget of stored dropout keep bits (b h ceil(sk / 64) sq 8 bytes).  Above it the
# forward stores none and the backward regenerates them from the hash right before it runs
# (ext().attention_keep_bits): transient memory for one layer instead of saved activations that
# grow with sq * sk (GPT-2 XL b 32 s 2048 stores 419 MB per layer).
KEEPBITS_MAX_BYTES = [int(float(os.environ.get("SMP_ATTN_KEEPBITS_MAX_MB", "1024")) * (1 << 20))]


def _store_bits(q, k, dropout_p):
    if dropout_p <= 0.0:
        return True
    b, sq, h = q.shape[0], q.shape[1], q.shape[2]
    sk = k.shape[1]
    return b * h * ((sk + 63) // 64) * sq * 8 <= KEEPBITS_MAX_BYTES[0]


# Keep-bits prefetch (SMP_ATTN_BITS_PREFETCH, default on): the layer launches the dropout
# keep-bits kernel on a side stream right before its QKV projection GEMM, so the hash (pure
# VALU + stores) runs beside the MFMA-bound GEMM instead of in front of the attention forward.
BITS_PREFETCH = [os.environ.get("SMP_ATTN_BITS_PREFETCH", "1") != "0"]
_SIDE = {}


class KeepBits:
    """Dropout keep bits generated ahead of the flash forward: (seed, offset) drawn now, the
    words produced on a side stream; ``consume`` makes the current stream wait for them."""

    __slots__ = ("bits", "seed", "off", "event", "shape")

    def consume(self):
        torch.cuda.current_stream(self.bits.device).wait_event(self.event)
        return self.bits


def prefetch_keep_bits(b, h, sq, sk, causal, dropout_p, device, like):
    """Launch the keep-bits kernel for a (b, h, sq, sk) dropout attention on a side stream
    (ordered after the work already queued on the current stream).  Returns a KeepBits for
    ``attention_packed(..., keep_bits=...)``, or None when prefetching does not apply."""
    if not (BITS_PREFETCH[0] and dropout_p > 0.0 and device.type == "cuda"):
        return None
    seed, off = dropout_seed_offset(device)
    cur = torch.cuda.current_stream(device)
    side = _SIDE.get(device)
    if side is None:
        side = _SIDE[device] = torch.cuda.Stream(device=device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        bits = ext().attention_keep_bits_for(b, h, sq, sk, causal, dropout_p, seed, off, like)
        ev = torch.cuda.Event()
        ev.record(side)
    bits.record_stream(cur)  # read (and saved for the backward) on the compute stream
    kb = KeepBits()
    kb.bits, kb.seed, kb.off, kb.event, kb.shape = bits, seed, off, ev, (b, h, sq, sk, bool(causal), float(dropout_p))
    return kb


def _keep_bits(bits, q, k, v, causal, window, p, seed, off):
    """The forward's keep bits, or (forward stored none) the same words regenerated now."""
    if p <= 0.0:
        return None
    if bits.numel() == 0:
        return ext().attention_keep_bits(q, k, v, causal, window, p, seed, off)
    return bits


def _count_flash(kb):
    FLASH_CALLS["key_bias" if kb is not None else "plain"] += 1


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, window, kb, dropout_p):
        seed, off = dropout_seed_offset(q.device) if dropout_p > 0.0 else (0, 0)
        bias = kb.bias if kb is not None else None
        o, lse, bits = ext().attention_fwd(q, k, v, scale, causal, window, bias, dropout_p, seed, off,
                                           _store_bits(q, k, dropout_p))
        ctx.save_for_backward(q, k, v, o, lse, bits)
        ctx.kb = kb
        ctx.scale, ctx.causal, ctx.window = scale, causal, window
        ctx.drop = (dropout_p, seed, off)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, bits = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        p, seed, off = ctx.drop
        kb = ctx.kb
        bias = kb.bias if kb is not None else None
        bits = _keep_bits(bits, q, k, v, ctx.causal, ctx.window, p, seed, off)
        ext().attention_bwd_into(do.contiguous(), q, k, v, o, lse, dq, dk, dv, ctx.scale, ctx.causal, ctx.window,
                                 bias, p, seed, off, bits)
        return dq, dk, dv, None, None, None, None, None


class _FlashAttentionPacked(torch.autograd.Function):
    """Self-attention straight from the fused QKV projection output [b, s, 3, h, d]:
    the backward writes dQ/dK/dV into one packed gradient (no scatter/zero-fill copies)."""

    @staticmethod
    def forward(ctx, qkv, scale, causal, window, kb, dropout_p, pre=None):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        bits_in = None
        if pre is not None and dropout_p > 0.0 and window <= 0 and \
                pre.shape == (q.shape[0], q.shape[2], q.shape[1], k.shape[1], bool(causal), float(dropout_p)):
            seed, off = pre.seed, pre.off
            bits_in = pre.consume()
        else:
            seed, off = dropout_seed_offset(qkv.device) if dropout_p > 0.0 else (0, 0)
        bias = kb.bias if kb is not None else None
        o, lse, bits = ext().attention_fwd(q, k, v, scale, causal, window, bias, dropout_p, seed, off,
                                           _store_bits(q, k, dropout_p), bits_in)
        ctx.save_for_backward(qkv, o, lse, bits)
        ctx.kb = kb
        ctx.scale, ctx.causal, ctx.window = scale, causal, window
        ctx.drop = (dropout_p, seed, off)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, bits = ctx.saved_tensors
        dqkv = torch.empty_like(qkv)
        p, seed, off = ctx.drop
        kb = ctx.kb
        bias = kb.bias if kb is not None else None
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        bits = _keep_bits(bits, q, k, v, ctx.causal, ctx.window, p, seed, off)
        ext().attention_bwd_into(do.contiguous(), q, k, v, o, lse, dqkv[:, :, 0],
                                 dqkv[:, :, 1], dqkv[:, :, 2], ctx.scale, ctx.causal, ctx.window, bias, p, seed, off,
                                 bits)
        # a fresh buffer no one else holds: the packed rotary's backward may rotate it in place
        dqkv._smp_fresh_grad = True
        return dqkv, None, None, None, None, None, None


def attention_packed(qkv, causal=True, scale=None, dropout_p=0.0, window=None, training=True, use_flash=True,
                     mask=None, mask_value=-1e4, keep_bits=None):
    """qkv: [b, s, 3, h, d] -> [b, s, h, d].  mask: optional [b|1, 1, s, s] bool (True = masked).
    keep_bits: a ``prefetch_keep_bits`` result for this attention (used by the flash path)."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    q = qkv[:, :, 0]
    p = dropout_p if training else 0.0
    kbias = key_padding_bias(mask, q.shape[1], q.shape[1], mask_value) if mask is not None else None
    if use_flash and flash_supported(q, p, mask, kbias):
        _count_flash(kbias)
        return _FlashAttentionPacked.apply(qkv, float(scale), bool(causal), int(window or 0), kbias, float(p),
                                           keep_bits)
    return attention(q, qkv[:, :, 1], qkv[:, :, 2], causal=causal, mask=mask, scale=scale, dropout_p=dropout_p,
                     window=window, training=training, use_flash=use_flash, mask_value=mask_value)


# Score elements per materialised chunk.  Root cause of the round-1 GPT-J fault
# (profiles/r2/gptj_fault_root_cause.md): torch's bundled hipBLASLt picks a stream-K solution
# (Custom_Cijk_Alik_Bljk_..._SK3_..._MT256x256x64_..._shortname0_gfx950) for the batched
# "A @ B^T" product [bh, s, s] x [bh, d, s]^T -> [bh, s, d], and that kernel faults from
# bh = 32, s = 2048, d = 256 (A = 2^27 elements); the same product with B contiguous
# [bh, s, d] ("A @ B") runs at every size tried (up to 2^28).  That layout arises when the
# score GEMM's K^T operand is a materialised copy (packed-QKV views); this path feeds the GEMMs
# contiguous [b, h, s, d] q/k/v, so every score GEMM and its backward run as NN / TN / "Q K^T
# on a K view" (tests/test_attention_chunking.py checks the layouts).  Chunking over the
# batch additionally bounds the [b, h, sq, sk] score memory.
_MAX_SCORE_ELEMS = 1 << 26


def _materialised(q, k, v, scale, causal, mask, dropout_p, window, training, fp32):
    b, sq, h = q.shape[0], q.shape[1], q.shape[2]
    per_b = h * sq * k.shape[1]
    if b > 1 and b * per_b > _MAX_SCORE_ELEMS:
        cb = max(1, _MAX_SCORE_ELEMS // per_b)
        # split(), not slicing: its backward is one concatenation of the chunk grads, where a
        # slice's backward zero-fills a full-size gradient per chunk and adds them up
        qs, ks, vs = q.split(cb), k.split(cb), v.split(cb)
        ms = [mask] * len(qs) if mask is None or mask.shape[0] == 1 else mask.split(cb)
        outs = [_chunk(qi, ki, vi, scale, causal, mi, dropout_p, window, training, fp32)
                for qi, ki, vi, mi in zip(qs, ks, vs, ms)]
        return torch.cat(outs, 0)
    return _chunk(q, k, v, scale, causal, mask, dropout_p, window, training, fp32)


def _checkpoint_attentions():
    from ..torch.state_mod import state

    return state.cfg is not None and bool(getattr(state.cfg, "checkpoint_attentions", False))


def _chunk(q, k, v, scale, causal, mask, dropout_p, window, training, fp32):
    """``checkpoint_attentions`` (reference `nn/transformer.py:1487-1496`): the materialised
    path keeps no [b, h, sq, sk] scores / probabilities for backward -- they are recomputed
    (same dropout decisions: the RNG state is replayed).  The flash kernels need no such
    option: they only ever keep the output and the per-row log-sum-exp."""
    if _checkpoint_attentions() and torch.is_grad_enabled() and any(t.requires_grad for t in (q, k, v)):
        from torch.utils.checkpoint import checkpoint

        return checkpoint(_materialised_chunk, q, k, v, scale, causal, mask, dropout_p, window, training, fp32,
                          use_reentrant=False, preserve_rng_state=True)
    return _materialised_chunk(q, k, v, scale, causal, mask, dropout_p, window, training, fp32)


def _materialised_chunk(q, k, v, scale, causal, mask, dropout_p, window, training, fp32):
    # q,k,v: [b, s, h, d] -> contiguous [b, h, s, d]: the score GEMMs then run as plain
    # batched GEMMs.  Strided views of a packed QKV reach library solutions that fault
    # (TunableOp tuning of GPT-J's score GEMM: profiles/r1_gptj6b_1gpu.md).
    qh, kh, vh = (t.transpose(1, 2).contiguous() for t in (q, k, v))
    if fp32:
        qh, kh, vh = qh.float(), kh.float(), vh.float()
    scores = torch.matmul(qh, kh.transpose(-1, -2))
    b, h, sq, sk = scores.shape
    if window is not None and window > 0:
        i = torch.arange(sq, device=q.device).view(-1, 1) + (sk - sq)
        j = torch.arange(sk, device=q.device).view(1, -1)
        # same semantics as the flash kernel: keys older than the window are masked, future
        # keys only when the attention is causal
        local = j <= i - window
        if causal:
            local = local | (j > i)
        mask = local.view(1, 1, sq, sk) if mask is None else (mask.bool() | local.view(1, 1, sq, sk))
        causal = False
    if fused_ok(scores) and scores.dtype in (torch.float16, torch.bfloat16):
        if causal and mask is None:
            probs = _sm.scaled_causal_softmax(scores, scale)
        else:
            m = mask
            if causal:
                tri = torch.ones(sq, sk, dtype=torch.bool, device=q.device).tril(diagonal=sk - sq)
                m = (~tri).view(1, 1, sq, sk) if m is None else (m.bool() | (~tri).view(1, 1, sq, sk))
            if m is not None:
                m = m.expand(m.shape[0], 1, sq, sk).to(torch.uint8).contiguous()
            probs = _sm.scaled_masked_softmax(scores, m, scale)
    else:
        probs = _sm._ref_softmax(scores, mask, scale, causal) if mask is None or mask.dtype == torch.bool or \
            mask.dtype == torch.uint8 else torch.softmax(scores.float() * scale + mask.float(), dim=-1).to(scores.dtype)
    if dropout_p > 0.0 and training:
        probs = torch.nn.functional.dropout(probs, p=dropout_p, training=True)
    ctx = torch.matmul(probs, vh)
    return ctx.transpose(1, 2).to(q.dtype)


def attention(q, k, v, causal=True, mask=None, scale=None, dropout_p=0.0, window=None, training=True,
              attention_in_fp32=False, use_flash=True, mask_value=-1e4):
    """q, k, v: [b, s, h, d]. mask: bool/uint8 [b|1, 1, sq, sk] with True = masked (applied
    together with the causal / window masks)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    p = dropout_p if training else 0.0
    if use_flash and not attention_in_fp32 and fused_ok(q):
        kbias = key_padding_bias(mask, q.shape[1], k.shape[1], mask_value) if mask is not None else None
        if flash_supported(q, p, mask, kbias):
            _count_flash(kbias)
            return _FlashAttention.apply(q, k, v, float(scale), bool(causal), int(window or 0), kbias, float(p))
    return _materialised(q, k, v, scale, causal, mask, dropout_p, window, training, attention_in_fp32)
