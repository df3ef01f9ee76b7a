"""GPT-NeoX (HF ``GPTNeoXForCausalLM``) <-> ``DistributedTransformerLMHead``.

Reference: `smp/torch/nn/huggingface/gptneox.py:35-90`.  Parallel residual with two
LayerNorms (input / post-attention), NeoX half-rotation rotary on
``partial_rotary_factor * head_dim`` channels, exact-erf GeLU, untied bias-free LM head.
HF stores query_key_value per head as [heads][3][d]; the fused smp layout is [3][heads][d].
"""
import re

from ._common import KeyMap, lm_forward_hook, lm_return_hook

_L = r"gpt_neox\.layers\.(\d+)\."
_S = "transformer.seq_layers.{}."
RULES = KeyMap([
    (r"gpt_neox\.embed_in\.weight", "word_embedding.weight", "copy"),
    (_L + r"input_layernorm\.weight", _S + "attention.pre_layernorm_module.weight", "copy"),
    (_L + r"input_layernorm\.bias", _S + "attention.pre_layernorm_module.bias", "copy"),
    (_L + r"post_attention_layernorm\.weight", _S + "output.pre_layernorm_module.weight", "copy"),
    (_L + r"post_attention_layernorm\.bias", _S + "output.pre_layernorm_module.bias", "copy"),
    (_L + r"attention\.dense\.weight", _S + "attention.dense_weight", "copy"),
    (_L + r"attention\.dense\.bias", _S + "attention.dense_bias", "copy"),
    (_L + r"mlp\.dense_h_to_4h\.weight", _S + "output.dense1_weight", "copy"),
    (_L + r"mlp\.dense_h_to_4h\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"mlp\.dense_4h_to_h\.weight", _S + "output.dense2_weight", "copy"),
    (_L + r"mlp\.dense_4h_to_h\.bias", _S + "output.dense2_bias", "copy"),
    (r"gpt_neox\.final_layer_norm\.weight", "layernorm.weight", "copy"),
    (r"gpt_neox\.final_layer_norm\.bias", "layernorm.bias", "copy"),
    (r"lm_head\.weight", "lm_head.weight", "copy"),
    (r"embed_out\.weight", "lm_head.weight", "copy"),
])

_heads = {}


def _rope(config):
    rp = getattr(config, "rope_parameters", None) or {}
    frac = rp.get("partial_rotary_factor", getattr(config, "rotary_pct", 0.25))
    base = rp.get("rope_theta", getattr(config, "rotary_emb_base", 10000))
    return frac, base


def config_to_kwargs(config):
    h = config.hidden_size
    d = h // config.num_attention_heads
    frac, base = _rope(config)
    _heads["n"] = config.num_attention_heads
    return {
        "num_layers": config.num_hidden_layers,
        "num_attention_heads": config.num_attention_heads,
        "attention_head_size": d,
        "hidden_size": h,
        "intermediate_size": config.intermediate_size,
        "vocab_size": config.vocab_size,
        "num_positions": config.max_position_embeddings,
        "attention_dropout_prob": config.attention_dropout,
        "hidden_dropout_prob": config.hidden_dropout,
        "embedding_dropout_prob": 0.0,
        "activation": "gelu_exact" if config.hidden_act == "gelu" else "gelu",
        "layernorm_epsilon": config.layer_norm_eps,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "causal_mask_size": config.max_position_embeddings,
        "pre_layernorm": True,
        "post_layernorm": False,
        "parallel_attn_output": bool(config.use_parallel_residual),
        "final_layernorm": True,
        "rotary_dim": int(d * frac),
        "rotary_emb_base": base,
        "gpt_neox_type_rotary": True,
        "use_positional_embedding": False,
        "tie_input_output_embedding": False,
        "add_lm_head": True,
    }


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = lm_forward_hook
return_hook = lm_return_hook


def _reorder(t, heads, to_smp):
    shape = t.shape
    rest = shape[1:]
    d = shape[0] // (3 * heads)
    if to_smp:
        return t.reshape(heads, 3, d, *rest).transpose(0, 1).reshape(shape).contiguous()
    return t.reshape(3, heads, d, *rest).transpose(0, 1).reshape(shape).contiguous()


def hf_to_smp(sd, num_heads=None):
    heads = num_heads or _heads.get("n")
    out, rest = {}, {}
    for k, v in sd.items():
        m = re.match(r"^(.*?)" + _L + r"attention\.query_key_value\.(weight|bias)$", k)
        if m:
            if heads is None:
                raise ValueError("GPT-NeoX translation needs num_attention_heads")
            out[m.group(1) + _S.format(m.group(2)) + "attention.qkv_" + m.group(3)] = _reorder(v, heads, True)
        elif k.endswith(("attention.bias", "attention.masked_bias", "rotary_emb.inv_freq")):
            continue
        else:
            rest[k] = v
    rest = RULES.hf_to_smp(rest, out)
    out.update(rest)
    return out


def smp_to_hf(sd, num_heads=None):
    heads = num_heads or _heads.get("n")
    out, rest = {}, {}
    for k, v in sd.items():
        m = re.match(r"^(.*?)transformer\.seq_layers\.(\d+)\.attention\.qkv_(weight|bias)$", k)
        if m:
            out[f"{m.group(1)}gpt_neox.layers.{m.group(2)}.attention.query_key_value.{m.group(3)}"] = \
                _reorder(v, heads, False)
        else:
            rest[k] = v
    rest = RULES.smp_to_hf(rest, out)  # LM head: `lm_head` in transformers 5.x (older: `embed_out`)
    out.update(rest)
    return out


# ---- reference-named entry points (`torch/nn/huggingface/gptneox.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_gptneox_transformer_lm_head_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_gptneox(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_gptneox(state_dict, max_seq_len=None):
    """(max_seq_len: the reference re-creates HF attention-mask buffers of that length; the
    installed transformers keeps none in its state dicts, so it is accepted and unused.)"""
    return smp_to_hf(state_dict)
