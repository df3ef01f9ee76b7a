"""GPT-family configurations on ``smp.nn.DistributedTransformerLMHead``.

The configs mirror the public architectures used by BASELINE.json (GPT-2 small/XL,
GPT-J 6B, GPT-NeoX 20B, a GPT-3 175B shape) and the reference's HF translations
(`smp/torch/nn/huggingface/gpt2.py:41-81`, `gptj.py:34-80`, `gptneox.py:35-90`).
"""
import torch

from ..nn.transformer import DistributedTransformerLMHead

_GPT2_COMMON = dict(
    activation="gelu", layernorm_epsilon=1e-5, pre_layernorm=True, post_layernorm=False, final_layernorm=True,
    use_positional_embedding=True, tie_input_output_embedding=True, use_qkv_bias=True, use_attn_dense_bias=True,
    initializer_range=0.02, fused_bias_gelu=True,
)

GPT_CONFIGS = {
    "gpt2-tiny": dict(_GPT2_COMMON, num_layers=2, num_attention_heads=4, attention_head_size=16, hidden_size=64,
                      intermediate_size=256, vocab_size=512, num_positions=128),
    "gpt2-small": dict(_GPT2_COMMON, num_layers=12, num_attention_heads=12, attention_head_size=64, hidden_size=768,
                       intermediate_size=3072, vocab_size=50257, num_positions=1024),
    "gpt2-xl": dict(_GPT2_COMMON, num_layers=48, num_attention_heads=25, attention_head_size=64, hidden_size=1600,
                    intermediate_size=6400, vocab_size=50257, num_positions=2048),
    "gptj-6b": dict(activation="gelu", layernorm_epsilon=1e-5, pre_layernorm=True, post_layernorm=False,
                    single_pre_layernorm=True, parallel_attn_output=True, final_layernorm=True,
                    use_positional_embedding=False, rotary_dim=64, tie_input_output_embedding=False,
                    use_lm_head_bias=True, use_qkv_bias=False, use_attn_dense_bias=False, num_layers=28,
                    num_attention_heads=16, attention_head_size=256, hidden_size=4096, intermediate_size=16384,
                    vocab_size=50400, num_positions=2048),
    "gptneox-20b": dict(activation="gelu", layernorm_epsilon=1e-5, pre_layernorm=True, post_layernorm=False,
                        parallel_attn_output=True, final_layernorm=True, use_positional_embedding=False,
                        rotary_dim=24, gpt_neox_type_rotary=True, rotary_emb_base=10000,
                        tie_input_output_embedding=False, num_layers=44, num_attention_heads=64,
                        attention_head_size=96, hidden_size=6144, intermediate_size=24576, vocab_size=50432,
                        num_positions=2048),
    "gpt3-175b": dict(_GPT2_COMMON, num_layers=96, num_attention_heads=96, attention_head_size=128, hidden_size=12288,
                      intermediate_size=49152, vocab_size=50257, num_positions=2048),
}


def build_gpt(name, dropout=0.1, **overrides):
    cfg = dict(GPT_CONFIGS[name])
    cfg.update(attention_dropout_prob=dropout, hidden_dropout_prob=dropout, embedding_dropout_prob=dropout)
    cfg.update(overrides)
    cfg.setdefault("causal_mask_size", cfg["num_positions"])  # follows a num_positions override
    return DistributedTransformerLMHead(**cfg)


def gpt_inputs(batch, seq, vocab, device, generator=None):
    """Synthetic (input_ids, attention_mask, token_type_ids, position_ids, labels)."""
    ids = torch.randint(0, vocab, (batch, seq), device=device, generator=generator)
    mask = torch.ones(batch, seq, dtype=torch.long, device=device)
    return ids, mask, None, None, ids


def num_params(name):
    c = GPT_CONFIGS[name]
    h, L, V, i = c["hidden_size"], c["num_layers"], c["vocab_size"], c["intermediate_size"]
    att = c["num_attention_heads"] * c["attention_head_size"]
    per_layer = 3 * h * att + 3 * att + att * h + h + h * i + i + i * h + h + 4 * h
    emb = V * h + (c["num_positions"] * h if c.get("use_positional_embedding", True) else 0)
    head = 0 if c.get("tie_input_output_embedding", True) else V * h
    return L * per_layer + emb + head + 2 * h


def train_flops_per_token(name, seq):
    """6N + 12 L h s (attention), no recompute."""
    c = GPT_CONFIGS[name]
    return 6 * num_params(name) + 12 * c["num_layers"] * c["num_attention_heads"] * c["attention_head_size"] * seq
