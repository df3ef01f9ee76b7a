"""Model zoo: GPT-2 / GPT-J / GPT-Neo / GPT-NeoX / BERT configurations built on smp.nn."""
from .gpt import GPT_CONFIGS, build_gpt, gpt_inputs  # noqa: F401
