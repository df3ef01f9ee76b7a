"""RoBERTa encoder (HF ``RobertaEncoder``) <-> ``DistributedTransformer``.

Reference: `smp/torch/nn/huggingface/roberta.py`.  The encoder layers are BERT's (post-LN,
exact-erf GeLU, ``encoder.layer.{i}.*`` keys, optional cross-attention), so the key rules and
the layer translation are `bert.py`'s; what is RoBERTa's own is the validation, raised as
``HFRobertaConfigError`` as the reference does.  RoBERTa's padding-offset position ids are
computed by the HF embeddings module, which stays outside the distributed stack.
"""
from functools import partial

from ...backend.exceptions import HFRobertaConfigError
from . import bert
from ._common import encoder_forward_hook, encoder_return_hook

hf_to_smp = bert.hf_to_smp
smp_to_hf = bert.smp_to_hf


def config_to_kwargs(config):
    return bert.config_to_kwargs(config, error=HFRobertaConfigError, family="RoBERTa")


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = partial(encoder_forward_hook, error=HFRobertaConfigError, family="RoBERTa")
return_hook = encoder_return_hook


# ---- reference-named entry points (`torch/nn/huggingface/roberta.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_roberta_transformer_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_roberta(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_roberta(state_dict):
    return smp_to_hf(state_dict)


translate_hf_state_dict_to_smdistributed = translate_hf_state_dict_to_smdistributed_roberta
