"""Worker: HF causal LMs (argv: family pp tp) created under smp.model_creation(tensor_parallelism=
tp > 1) -- smp.nn's DistributedTransformerLMHead when tp > 1 -- optionally auto-partitioned
over pp stages, trained on right-padded batches (attention_mask) in step with the plain HF
model: same loss every step."""
import os
import sys

import torch
import transformers as tf

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn.huggingface import gpt2, gptj, gptneo, gptneox


def build(family):
    common = dict(vocab_size=97, bos_token_id=0, eos_token_id=0)
    if family == "gpt2":
        return tf.GPT2LMHeadModel(tf.GPT2Config(n_layer=4, n_embd=64, n_head=4, n_positions=64, resid_pdrop=0.0,
                                                embd_pdrop=0.0, attn_pdrop=0.0, **common)), gpt2
    if family == "gptj":
        return tf.GPTJForCausalLM(tf.GPTJConfig(n_layer=4, n_embd=64, n_head=4, n_positions=64, rotary_dim=8,
                                                resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0, **common)), gptj
    if family == "gptneo":
        return tf.GPTNeoForCausalLM(tf.GPTNeoConfig(num_layers=4, hidden_size=64, num_heads=4, max_position_embeddings=64,
                                                    attention_types=[[["global", "local"], 2]], window_size=8,
                                                    resid_dropout=0.0, embed_dropout=0.0, attention_dropout=0.0,
                                                    **common)), gptneo
    return tf.GPTNeoXForCausalLM(tf.GPTNeoXConfig(num_hidden_layers=4, hidden_size=64, num_attention_heads=4,
                                                  intermediate_size=256, max_position_embeddings=64,
                                                  hidden_dropout=0.0, attention_dropout=0.0, **common)), gptneox


def main():
    family, pp, tp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    torch.manual_seed(0)
    ref, mod = build(family)
    bf16 = os.environ.get("HF_MASK_BF16") == "1"  # GPU variant: bf16 smp model (flash key-bias path)
    extra = {}
    for kv in filter(None, os.environ.get("HF_MASK_CFG", "").split(",")):  # e.g. optimize=memory
        k, v = kv.split("=")
        extra[k] = {"true": True, "false": False}.get(v.lower(), v)
    smp.init(dict({"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2,
                   "auto_partition": True, "ddp": True, "bf16": bf16}, **extra))
    torch.manual_seed(0)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net, _ = build(family)
    model = smp.DistributedModel(net)
    if tp > 1:
        model.load_state_dict(ref.state_dict(), translate_function=mod.hf_to_smp)
    else:
        model.load_state_dict(ref.state_dict())
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.5))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.5)

    dev = smp.state.device

    @smp.step
    def train(model, ids, mask, labels):
        out = model(input_ids=ids, attention_mask=mask, labels=labels)
        model.backward(out.loss)
        return out.loss

    g = torch.Generator().manual_seed(5)
    for it in range(3):
        ids = torch.randint(1, 97, (4, 24), generator=g)
        mask = torch.ones(4, 24, dtype=torch.long)
        mask[1, 17:] = 0
        mask[3, 9:] = 0
        labels = ids.masked_fill(mask == 0, -100)
        opt.zero_grad()
        loss = float(train(model, ids.to(dev), mask.to(dev), labels.to(dev)).reduce_mean())
        opt.step()
        ropt.zero_grad()
        rl = torch.stack([ref(input_ids=ids[i:i + 2], attention_mask=mask[i:i + 2], labels=labels[i:i + 2]).loss
                          for i in (0, 2)]).mean()
        rl.backward()
        ropt.step()
        if smp.pp_rank() == 0:
            tol = 3e-2 * abs(rl.item()) if bf16 else 2e-4
            assert abs(loss - rl.item()) < tol, (family, it, loss, rl.item())
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
