"""LM head + cross entropy over a 64-aligned padded vocabulary.

GPT-2's vocabulary (50257) is odd: the logits rows of ``hidden @ E^T`` are then not
16-byte aligned and all three LM-head GEMMs run in hipBLASLt's unaligned variants
(GPT-2 XL at mbs 16 x 2048: 3.0 ms forward, 5.2 ms input-gradient in the strided NN
layout, 5.9 ms weight-gradient per step).  Here the [V, h] weight is viewed through a
zero-padded [Vp, h] copy (Vp = V rounded up to 64; refreshed once per step like the
W^T copies of ``ops/linear.py``), so

* the logits are [T, Vp] with aligned rows (forward GEMM in the fast TN layout);
* the cross-entropy kernels read only the first V columns of each row (``vocab`` < row
  stride) and the backward writes the padding columns of dlogits as zeros, so the loss
  and every gradient equal the unpadded model's exactly (the padding rows never
  receive gradient and never influence the logits that are read);
* the input gradient ``dlogits @ E`` runs as ``F.linear(dlogits, E_pad^T)`` (TN, aligned);
* the weight gradient is one aligned GEMM -- the split-K MFMA kernel of ``ops/linear.py``
  for bf16 -- into a [Vp, h] temporary whose first V rows are added to the (flat-buffer)
  gradient.

The user still receives [.., V] logits (a view) and can backpropagate through them.

Measured on MI355X for GPT-2 XL (TunableOp-selected GEMMs, mbs 16, round 2): forward 3.50 ms
padded vs 3.03 ms unpadded, input gradient 3.90 vs 4.74 ms, weight gradient 5.30 vs 4.91 ms --
a wash then.  With the round-5 ping-pong weight-gradient kernel at the bench's mbs 32 the
padded path wins: 748.38 / 748.56 vs 750.73 / 752.94 ms per step, same box alternating, same
loss (tools/gpu_r5w.sh) -- so it is ON by default (``SMP_PADDED_LM_HEAD=0`` disables it).
Reference behaviour being reproduced: the LM head + CE of ``DistributedTransformerLMHead``
(`smp/torch/nn/transformer.py:455-548`).
"""
import os

import torch
import torch.nn.functional as F

from ._ext import ext, fused_ok
from .linear import _WT_EPOCH, _fusable

# LM-head weight gradient on the MFMA weight-gradient kernel (bf16 operands)
_WGRAD_KERNEL = True

_ALIGN = 64
_ENABLED = os.environ.get("SMP_PADDED_LM_HEAD", "1") == "1"


def _padded(w, vp):
    """(W_pad [vp, h], W_pad^T [h, vp]) cached per (epoch, storage, version)."""
    key = (_WT_EPOCH[0], w.data_ptr(), w._version, vp)
    ent = w.__dict__.get("_smp_wpad")
    if ent is not None and ent[0] == key:
        return ent[1], ent[2]
    V, H = w.shape
    if ent is not None and ent[1].shape == (vp, H) and ent[1].dtype == w.dtype:
        wp, wpt = ent[1], ent[2]
    else:
        wp = torch.zeros(vp, H, dtype=w.dtype, device=w.device)
        wpt = torch.empty(H, vp, dtype=w.dtype, device=w.device)
    with torch.no_grad():
        wp[:V].copy_(w.detach())
        ext().transpose_into(wp, wpt)
    w.__dict__["_smp_wpad"] = (key, wp, wpt)
    return wp, wpt


def usable(weight, hidden):
    """The padded path applies to an odd-sized bf16/fp16 CUDA LM head inside a step (the
    cached copies are refreshed per step)."""
    if not (_ENABLED and fused_ok(hidden) and weight.is_cuda and weight.dim() == 2):
        return False
    if weight.shape[0] % _ALIGN == 0 or weight.dtype not in (torch.bfloat16, torch.float16):
        return False
    if hidden.dtype != weight.dtype or not weight.is_contiguous():
        return False
    from ..torch.state_mod import state

    return bool(getattr(state, "in_step_func", False))


class _PaddedLMHeadCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight, labels, ignore_index):
        V, H = weight.shape
        vp = (V + _ALIGN - 1) // _ALIGN * _ALIGN
        wp, wpt = _padded(weight, vp)
        h2 = hidden.reshape(-1, H)
        t = labels.reshape(-1).contiguous()
        logits = F.linear(h2, wp)  # [T, vp]
        mx, se, tl = ext().xent_fwd(logits, t, 0, ignore_index, V)
        lse = mx + torch.log(se)
        rows = torch.where(t == ignore_index, torch.zeros_like(lse), lse - tl)
        ctx.save_for_backward(h2, logits, t, lse)
        # an unused logits output must stay None in backward: materialised, it is a [T, Vp]
        # zero tensor plus a full read-modify-write of dlogits (~3.4 ms per GPT-2 XL b32 step)
        ctx.set_materialize_grads(False)
        ctx.weight, ctx.wpt, ctx.V, ctx.ignore, ctx.hshape = weight, wpt, V, ignore_index, hidden.shape
        out_logits = logits.view(*hidden.shape[:-1], vp)[..., :V]
        return rows.view(labels.shape), out_logits

    @staticmethod
    def backward(ctx, g_rows, g_logits):
        h2, logits, t, lse = ctx.saved_tensors
        V = ctx.V
        gr = g_rows.reshape(-1).float().contiguous() if g_rows is not None else torch.zeros_like(lse)
        dl = ext().xent_bwd(logits, t, lse, gr, 0, ctx.ignore, V)  # [T, vp]; padding columns zero
        if g_logits is not None:
            dl[:, :V] += g_logits.reshape(-1, V).to(dl.dtype)
        dx = F.linear(dl, ctx.wpt).view(ctx.hshape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if _WGRAD_KERNEL and dl.is_cuda and dl.dtype == torch.bfloat16 and h2.dtype == torch.bfloat16 \
                    and h2.shape[1] % 8 == 0 and h2.is_contiguous():
                # the split-K MFMA weight-gradient kernel (csrc/kernels/wgrad.hip): 9.99 vs
                # 10.9-11.1 ms for hipBLASLt at GPT-2 XL's [50304, 1600] x 65536 tokens
                # (profiles/r2/wgrad_kernel.md)
                gp = torch.empty(dl.shape[1], h2.shape[1], dtype=h2.dtype, device=h2.device)
                ext().wgrad_(gp, dl, h2, False, 0)
            else:
                gp = torch.mm(dl.t(), h2)  # [vp, h], aligned
            w = ctx.weight
            if _fusable(w):
                w.grad.add_(gp[:V])  # flat-buffer view: accumulate in place (hooks still fire)
            else:
                dw = gp[:V]
        return dx, dw, None, None


def padded_lm_head_cross_entropy(hidden, weight, labels, ignore_index=-100):
    """(per-token loss rows [...], logits [..., V]) of ``hidden @ weight^T`` against
    ``labels`` (ignore_index rows contribute 0)."""
    return _PaddedLMHeadCE.apply(hidden, weight, labels, ignore_index)
