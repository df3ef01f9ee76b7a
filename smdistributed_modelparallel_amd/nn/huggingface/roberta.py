"""RoBERTa encoder: same layer structure and key names as BERT (`bert.py`)."""
from .bert import config_to_kwargs, forward_hook, hf_to_smp, init_hook, return_hook, smp_to_hf  # noqa: F401
