"""Independent plain-torch GPT forward for equivalence tests.

Written only with torch functional ops (F.embedding / F.layer_norm / F.linear, a materialised
softmax(Q K^T * scale) V, the GeLU formulas, HF-style rotary) on a FULL (unsharded) state dict
of a ``DistributedTransformerLMHead`` -- it never calls this package's modules or kernels, so
it can serve as the reference the reference harness (`test/torch/smp_test_base.py:731-788`)
compares against.

Covered layouts: GPT-2 (pre-LN, learned positions, tied head), GPT-J (single pre-LN, parallel
attention + MLP, interleaved rotary, untied head with bias) and GPT-NeoX (two pre-LNs, parallel
attention + MLP, half rotary).  ``dtype`` is the compute dtype of the weights and branch
activations; ``fp32_residual`` keeps the residual stream in fp32 with the LayerNorms computed in
fp32 and rounded once to ``dtype`` (reference `torch/nn/transformer.py:890-894` +
MixedFusedLayerNorm).
"""
import math
import os

import torch
import torch.nn.functional as F


def _ln(x, w, b, eps, out_dtype):
    y = F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(out_dtype)


def _rotary(x, rd, base, neox):
    """x [B, s, nh, d]; rotate the first rd channels (HF GPT-J / GPT-NeoX formulas)."""
    s = x.shape[1]
    inv = 1.0 / (base ** (torch.arange(0, rd, 2, dtype=torch.float64, device=x.device) / rd))
    f = torch.arange(s, dtype=torch.float64, device=x.device)[:, None] * inv[None]
    cos, sin = f.cos().float(), f.sin().float()
    r, rest = x[..., :rd].float(), x[..., rd:]
    if neox:
        c = torch.cat((cos, cos), -1)[None, :, None]
        sn = torch.cat((sin, sin), -1)[None, :, None]
        half = rd // 2
        rot = torch.cat((-r[..., half:], r[..., :half]), -1)
    else:
        c = cos.repeat_interleave(2, -1)[None, :, None]
        sn = sin.repeat_interleave(2, -1)[None, :, None]
        rot = torch.stack((-r[..., 1::2], r[..., ::2]), -1).flatten(-2)
    return torch.cat(((r * c + rot * sn).to(x.dtype), rest), -1)


def _gelu(x, tanh):
    if tanh:
        xf = x.float()
        return (0.5 * xf * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (xf + 0.044715 * xf ** 3)))).to(x.dtype)
    return F.gelu(x.float()).to(x.dtype)


def gpt_logits(sd, ids, cfg, dtype=torch.float32, fp32_residual=False):
    """Logits [B, s, V] of the model described by ``cfg`` (a GPT_CONFIGS-style dict with the
    overrides applied) for weights ``sd`` (name -> tensor, any dtype/device; cast to ``dtype``)."""
    p = {k: v.to(dtype) for k, v in sd.items()}
    H, nh, d = cfg["hidden_size"], cfg["num_attention_heads"], cfg["attention_head_size"]
    eps = cfg.get("layernorm_epsilon", 1e-5)
    rd = cfg.get("rotary_dim") or 0
    neox = bool(cfg.get("gpt_neox_type_rotary"))
    base = cfg.get("rotary_emb_base") or 10000
    parallel = bool(cfg.get("parallel_attn_output"))
    single = bool(cfg.get("single_pre_layernorm"))
    tanh = bool(cfg.get("fused_bias_gelu")) or os.environ.get("SMP_USE_HF_GELU") == "1"
    B, s = ids.shape
    x = F.embedding(ids, p["word_embedding.weight"])
    if cfg.get("use_positional_embedding", True):
        x = x + F.embedding(torch.arange(s, device=ids.device), p["position_embedding.weight"])[None]
    if fp32_residual:
        x = x.float()
    causal = torch.ones(s, s, dtype=torch.bool, device=ids.device).triu(1)
    for i in range(cfg["num_layers"]):
        q_ = f"transformer.seq_layers.{i}."
        a = _ln(x, p[q_ + "attention.pre_layernorm_module.weight"], p[q_ + "attention.pre_layernorm_module.bias"],
                eps, dtype)
        qkv = F.linear(a, p[q_ + "attention.qkv_weight"], p.get(q_ + "attention.qkv_bias")).view(B, s, 3, nh, d)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if rd:
            q, k = _rotary(q, rd, base, neox), _rotary(k, rd, base, neox)
        scale = 1.0 / math.sqrt(d) if cfg.get("scale_attention_scores", True) else 1.0
        if cfg.get("scale_attn_by_layer_idx") and not cfg.get("query_key_layer_scaling"):
            scale /= i + 1
        sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
        att = torch.softmax(sc.masked_fill(causal, float("-inf")), dim=-1)
        ctx = torch.einsum("bhqk,bkhd->bqhd", att.to(dtype).float(), v.float()).to(dtype).reshape(B, s, nh * d)
        attn = F.linear(ctx, p[q_ + "attention.dense_weight"], p.get(q_ + "attention.dense_bias"))
        if parallel:
            m = a if single else _ln(x, p[q_ + "output.pre_layernorm_module.weight"],
                                     p[q_ + "output.pre_layernorm_module.bias"], eps, dtype)
        else:
            x = x + attn
            m = _ln(x, p[q_ + "output.pre_layernorm_module.weight"], p[q_ + "output.pre_layernorm_module.bias"], eps,
                    dtype)
        h = _gelu(F.linear(m, p[q_ + "output.dense1_weight"], p[q_ + "output.dense1_bias"]), tanh)
        mlp = F.linear(h, p[q_ + "output.dense2_weight"], p.get(q_ + "output.dense2_bias"))
        x = (x + attn + mlp) if parallel else (x + mlp)
    x = _ln(x, p["layernorm.weight"], p["layernorm.bias"], eps, dtype)
    if cfg.get("tie_input_output_embedding", True):
        return F.linear(x, p["word_embedding.weight"])
    return F.linear(x, p["lm_head.weight"], p.get("lm_head.bias"))


def gpt_loss(sd, ids, labels, cfg, dtype=torch.float32, fp32_residual=False):
    logits = gpt_logits(sd, ids, cfg, dtype, fp32_residual)
    return F.cross_entropy(logits[:, :-1].float().reshape(-1, logits.shape[-1]), labels[:, 1:].reshape(-1))
