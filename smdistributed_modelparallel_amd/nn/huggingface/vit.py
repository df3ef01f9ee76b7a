"""ViT (HF ``ViTLayer``) <-> ``DistributedTransformerLayer``.

Reference: `smp/torch/nn/huggingface/vit.py` (registered manually in its tests,
`test/torch/mpi_hybrid/test_vit_grad.py`), which replaced HF 4.x's ``ViTEncoder`` with a
``DistributedTransformer``.  transformers 5.x has no encoder module (``ViTModel`` loops
over ``layers``, a ModuleList of ``ViTLayer``), so the unit distributed here is the
layer: each ``ViTLayer`` becomes a pre-LayerNorm, bidirectional
``DistributedTransformerLayer`` (exact-erf GeLU for ``hidden_act="gelu"``, q/k/v fused
into one projection).  Keys: ``layers.{i}.attention.{q,k,v}_proj`` <->
``layers.{i}.attention.qkv_*``; embeddings, final LayerNorm, pooler and classifier stay HF.
Like the reference's, this mapping is opt-in: ``register_vit()`` (the process's registry,
``smp.state.tp_registry``; the predefined set covers the GPT/BERT families).
"""
from ._common import KeyMap, masked_from_hf, pack_qkv, unpack_qkv

# no layer prefix: the rules translate one layer's own state dict (``_match_weights``) as
# well as a whole model's (``layers.{i}.`` prefixes are carried through)
_L = ""
_S = ""
RULES = KeyMap([
    (_L + r"attention\.o_proj\.weight", _S + "attention.dense_weight", "copy"),
    (_L + r"attention\.o_proj\.bias", _S + "attention.dense_bias", "copy"),
    (_L + r"layernorm_before\.weight", _S + "attention.pre_layernorm_module.weight", "copy"),
    (_L + r"layernorm_before\.bias", _S + "attention.pre_layernorm_module.bias", "copy"),
    (_L + r"layernorm_after\.weight", _S + "output.pre_layernorm_module.weight", "copy"),
    (_L + r"layernorm_after\.bias", _S + "output.pre_layernorm_module.bias", "copy"),
    (_L + r"mlp\.fc1\.weight", _S + "output.dense1_weight", "copy"),
    (_L + r"mlp\.fc1\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"mlp\.fc2\.weight", _S + "output.dense2_weight", "copy"),
    (_L + r"mlp\.fc2\.bias", _S + "output.dense2_bias", "copy"),
])

_ACT = {"gelu": "gelu_exact", "gelu_new": "gelu", "gelu_pytorch_tanh": "gelu", "relu": "relu"}


def config_to_kwargs(config):
    h = config.hidden_size
    if config.hidden_act not in _ACT:
        from ...backend.exceptions import HFViTConfigError

        raise HFViTConfigError(f"unsupported ViT activation {config.hidden_act!r}")
    return {
        "num_attention_heads": config.num_attention_heads,
        "attention_head_size": h // config.num_attention_heads,
        "hidden_size": h,
        "intermediate_size": config.intermediate_size,
        "attention_dropout_prob": config.attention_probs_dropout_prob,
        "hidden_dropout_prob": config.hidden_dropout_prob,
        "activation": _ACT[config.hidden_act],
        "fused_bias_gelu": config.hidden_act != "gelu",
        "layernorm_epsilon": config.layer_norm_eps,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "causal_mask_size": None,
        "pre_layernorm": True,
        "post_layernorm": False,
        "use_qkv_bias": bool(getattr(config, "qkv_bias", True)),
    }


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


def forward_hook(hidden_states, attention_mask=None, *args, **kwargs):
    if kwargs.get("output_attentions") or kwargs.get("output_hidden_states"):
        from ...backend.exceptions import HFViTConfigError

        raise HFViTConfigError("output_attentions / output_hidden_states are not supported by the distributed ViT layer")
    return ((hidden_states, masked_from_hf(attention_mask)),), {}


def return_hook(out):
    return out[0]


def hf_to_smp(sd):
    out = {}
    rest = pack_qkv(sd, out, _L + r"attention\.q_proj\.weight", _L + r"attention\.k_proj\.weight",
                    _L + r"attention\.v_proj\.weight", _S + "attention.qkv_weight")
    rest = pack_qkv(rest, out, _L + r"attention\.q_proj\.bias", _L + r"attention\.k_proj\.bias",
                    _L + r"attention\.v_proj\.bias", _S + "attention.qkv_bias")
    rest = RULES.hf_to_smp(rest, out)
    out.update(rest)
    return out


def smp_to_hf(sd):
    out = {}
    rest = unpack_qkv(sd, out, r"attention\.qkv_weight", "attention.q_proj.weight", "attention.k_proj.weight",
                      "attention.v_proj.weight")
    rest = unpack_qkv(rest, out, r"attention\.qkv_bias", "attention.q_proj.bias", "attention.k_proj.bias",
                      "attention.v_proj.bias")
    rest = RULES.smp_to_hf(rest, out)
    out.update(rest)
    return out


def register_vit(registry=None):
    """Opt-in registration of ViTLayer -> DistributedTransformerLayer (reference tests
    register their ViT translation by hand the same way); default: the process's registry
    (``smp.state.tp_registry``), so ViT models created under ``smp.model_creation(
    tensor_parallelism=True)`` afterwards get distributed layers."""
    from transformers.models.vit.modeling_vit import ViTLayer

    if registry is None:
        from ...torch.state_mod import state

        registry = state.tp_registry

    from ..transformer import DistributedTransformerLayer

    registry.register(ViTLayer, DistributedTransformerLayer, init_hook=init_hook, forward_hook=forward_hook,
                      return_hook=return_hook, translate_functions=(smp_to_hf, hf_to_smp))


# ---- reference-named entry points (`torch/nn/huggingface/vit.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_vit_encoder_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_vit(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_vit(state_dict):
    return smp_to_hf(state_dict)


translate_hf_state_dict_to_smdistributed = translate_hf_state_dict_to_smdistributed_vit
