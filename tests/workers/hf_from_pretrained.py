"""Worker: the reference's pretrained-load flow (`test/torch/mpi/test_translate_state_dict.py:
103-160`): rank 0 writes an HF model with save_pretrained, every rank re-creates it with
from_pretrained under smp.tensor_parallelism (swapped for smp.nn at DistributedModel), the
saved weights are loaded with the family's translator (argv[3] "auto": no translate_function,
the registered one applies), and the TP=2 model's logits equal the HF model's.
argv: family(gpt2|gptj|gpt_neo|gpt_neox) dir auto|explicit"""
import os
import sys

import torch
import transformers as tf
from safetensors.torch import load_file

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import DistributedTransformerLMHead
from smdistributed_modelparallel_amd.nn.huggingface import gpt2, gptj, gptneo, gptneox

FAMILIES = {
    "gpt2": (tf.GPT2Config, tf.GPT2LMHeadModel, gpt2.translate_hf_state_dict_to_smdistributed_gpt2,
             dict(n_layer=2, n_embd=64, n_head=4, n_positions=32, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)),
    "gptj": (tf.GPTJConfig, tf.GPTJForCausalLM, gptj.translate_hf_state_dict_to_smdistributed_gptj,
             dict(n_layer=2, n_embd=64, n_head=4, n_positions=32, rotary_dim=8, resid_pdrop=0.0, embd_pdrop=0.0,
                  attn_pdrop=0.0)),
    "gpt_neo": (tf.GPTNeoConfig, tf.GPTNeoForCausalLM, gptneo.translate_hf_state_dict_to_smdistributed_gptneo,
                dict(num_layers=2, hidden_size=64, num_heads=4, max_position_embeddings=32,
                     attention_types=[[["global", "local"], 1]], window_size=8, resid_dropout=0.0,
                     embed_dropout=0.0, attention_dropout=0.0)),
    "gpt_neox": (tf.GPTNeoXConfig, tf.GPTNeoXForCausalLM, gptneox.translate_hf_state_dict_to_smdistributed_gptneox,
                 dict(num_hidden_layers=2, hidden_size=64, num_attention_heads=4, intermediate_size=256,
                      max_position_embeddings=32)),
}

TRANSLATOR_MODULES = {"gpt2": gpt2, "gptj": gptj, "gpt_neo": gptneo, "gpt_neox": gptneox}


def main():
    fam, d, how = sys.argv[1], sys.argv[2], sys.argv[3]
    cfg_cls, model_cls, translate, kw = FAMILIES[fam]
    cfg = cfg_cls(vocab_size=97, bos_token_id=0, eos_token_id=0, **kw)
    smp.init({"tensor_parallel_degree": 2, "ddp": True})
    torch.manual_seed(0)
    hf = model_cls(cfg).eval()
    if smp.rank() == 0:
        hf.save_pretrained(d)
    smp.barrier()
    with smp.tensor_parallelism(enabled=True):
        net = model_cls.from_pretrained(d)
    model = smp.DistributedModel(net)
    assert isinstance(model.get_module(), DistributedTransformerLMHead), type(model.get_module())
    sd = load_file(os.path.join(d, "model.safetensors"))
    model.load_state_dict(sd, strict=True, translate_function=translate if how == "explicit" else None)

    @smp.step
    def logits(model, ids):
        return model(input_ids=ids)["logits"]

    model.eval()
    ids = torch.randint(0, 97, (2, 16), generator=torch.Generator().manual_seed(1))
    out = logits(model, ids).concat()
    with torch.no_grad():
        ref = hf(input_ids=ids).logits
    err = (out.float() - ref.float()).abs().max().item()
    assert err < 1e-4, err
    # and back out (reference test_translate_state_dict_to_hf_*): the gathered state dict through
    # translate_state_dict_to_hf_<family> loads strictly into a fresh HF model with equal logits
    to_hf = getattr(TRANSLATOR_MODULES[fam], "translate_state_dict_to_hf_" + TRANSLATOR_MODULES[fam].__name__.rsplit(".", 1)[1])
    full = model.state_dict(gather_to_rank0=False)
    fresh = model_cls(cfg).eval()
    fresh.load_state_dict(to_hf(full, cfg.max_position_embeddings if hasattr(cfg, "max_position_embeddings") else 32),
                          strict=True)
    with torch.no_grad():
        err2 = (fresh(input_ids=ids).logits.float() - ref.float()).abs().max().item()
    assert err2 < 1e-5, err2
    print(f"rank {smp.rank()} OK {fam} {how} err={err:.2e}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
