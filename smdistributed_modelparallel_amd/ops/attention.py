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

import torch

from . import softmax as _sm
from ._ext import ext

_FLASH_OK = None


def flash_supported(q, dropout_p, mask):
    global _FLASH_OK
    if not q.is_cuda or dropout_p > 0.0 or mask is not None:
        return False
    if q.dtype not in (torch.bfloat16, torch.float16):
        return False
    if q.shape[-1] not in (64, 128):
        return False
    if _FLASH_OK is None:
        _FLASH_OK = hasattr(ext(), "attention_fwd")
    return _FLASH_OK


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, window):
        o, lse = ext().attention_fwd(q, k, v, scale, causal, window)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale, ctx.causal, ctx.window = scale, causal, window
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = ext().attention_bwd(do.contiguous(), q, k, v, o, lse, ctx.scale, ctx.causal, ctx.window)
        return dq, dk, dv, None, None, None


def _materialised(q, k, v, scale, causal, mask, dropout_p, window, training, fp32):
    # q,k,v: [b, s, h, d] -> [b, h, s, d]
    qh, kh, vh = (t.transpose(1, 2) for t in (q, k, v))
    if fp32:
        qh, kh, vh = qh.float(), kh.float(), vh.float()
    scores = torch.matmul(qh, kh.transpose(-1, -2))
    b, h, sq, sk = scores.shape
    if window is not None and window > 0:
        i = torch.arange(sq, device=q.device).view(-1, 1) + (sk - sq)
        j = torch.arange(sk, device=q.device).view(1, -1)
        local = (j > i) | (j <= i - window)
        mask = local.view(1, 1, sq, sk) if mask is None else (mask.bool() | local.view(1, 1, sq, sk))
        causal = False
    if scores.is_cuda and scores.dtype in (torch.float16, torch.bfloat16):
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
              attention_in_fp32=False, use_flash=True):
    """q, k, v: [b, s, h, d]. mask: bool/uint8 [b|1, 1, sq, sk] with True = masked."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if use_flash and not attention_in_fp32 and flash_supported(q, dropout_p if training else 0.0, mask):
        return _FlashAttention.apply(q, k, v, float(scale), bool(causal), int(window or 0))
    return _materialised(q, k, v, scale, causal, mask, dropout_p, window, training, attention_in_fp32)
