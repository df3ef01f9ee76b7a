"""Worker: an HF GPT2LMHeadModel created under smp.model_creation(tensor_parallelism=True)
is replaced by DistributedTransformerLMHead (TP=2), loads the HF weights through the
translator, and trains in step with the HF model (scaled-batch TP: each rank its batch)."""
import torch
from transformers import GPT2Config, GPT2LMHeadModel

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import DistributedTransformerLayer, DistributedTransformerLMHead
from smdistributed_modelparallel_amd.nn.huggingface import gpt2


def main():
    import sys

    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    match = mode in ("match", "layer")
    cfg = GPT2Config(n_layer=2, n_embd=64, n_head=4, vocab_size=97, n_positions=32, bos_token_id=0, eos_token_id=0,
                     resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    torch.manual_seed(0)
    ref = GPT2LMHeadModel(cfg)
    smp.init({"tensor_parallel_degree": 2, "ddp": True, "_match_weights": match})
    torch.manual_seed(0)
    if mode == "layer":
        # "huggingface-gpt-2-layer": only the GPT2Blocks are distributed (embeddings, ln_f
        # and the tied head stay HF modules), their weights matched from the HF blocks
        net = GPT2LMHeadModel(cfg)
        for block in net.transformer.h:
            smp.set_tensor_parallelism(block, True)
        model = smp.DistributedModel(net)
        assert all(isinstance(b, DistributedTransformerLayer) for b in model.get_module().transformer.h)
    else:
        with smp.model_creation(tensor_parallelism=True):
            net = GPT2LMHeadModel(cfg)  # same seed: the same initial weights as ref
        model = smp.DistributedModel(net)
        assert isinstance(model.get_module(), DistributedTransformerLMHead), type(model.get_module())
    if not match:
        model.load_state_dict(ref.state_dict(), translate_function=gpt2.hf_to_smp)
    # (match: _match_weights already gave every TP rank its slices of the HF weights)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)

    @smp.step
    def train(model, ids):
        out = model(input_ids=ids, labels=ids)
        model.backward(out.loss)
        return out.loss

    g = torch.Generator().manual_seed(3)
    for it in range(2):
        ids_all = torch.randint(0, 97, (4, 16), generator=g)
        ids = ids_all[smp.rank() * 2:(smp.rank() + 1) * 2]
        opt.zero_grad()
        loss = train(model, ids).reduce_mean().item()
        opt.step()
        ropt.zero_grad()
        rl = [ref(input_ids=ids_all[r * 2:(r + 1) * 2], labels=ids_all[r * 2:(r + 1) * 2]).loss for r in range(2)]
        torch.stack(rl).mean().backward()
        ropt.step()
        assert abs(loss - rl[smp.rank()].item()) < 1e-4, (it, loss, rl[smp.rank()].item())
    # full state dict comes back in HF key space
    sd = model.state_dict(gather_to_rank0=False)
    hf_sd = gpt2.layer_smp_to_hf(sd) if mode == "layer" else gpt2.smp_to_hf(sd)
    worst = max((hf_sd[k].float() - v.detach().float()).abs().max().item() for k, v in ref.state_dict().items())
    assert worst < 2e-4, worst
    if len(sys.argv) > 2:
        # full checkpoint in HF key space (translate_if_full): a plain transformers model loads
        # it strictly and computes the trained model's loss
        import os

        ckpt = sys.argv[2]
        smp.save_checkpoint(ckpt, tag="hf", partial=False, model=model, translate_if_full=True)
        if smp.rank() == 0:
            saved = torch.load(os.path.join(ckpt, "hf"), weights_only=True)
            fresh = GPT2LMHeadModel(cfg)
            fresh.load_state_dict(saved, strict=True)
            ids = torch.randint(0, 97, (2, 16), generator=g)
            with torch.no_grad():
                a, b = fresh(input_ids=ids, labels=ids).loss.item(), ref(input_ids=ids, labels=ids).loss.item()
            assert abs(a - b) < 1e-4, (a, b)
            print("full HF checkpoint OK", flush=True)
        # and it resumes into the TP model: HF keys go back through hf_to_smp
        with torch.no_grad():
            for p in model.parameters():
                p.zero_()
        smp.resume_from_checkpoint(ckpt, tag="hf", partial=False, load_optimizer=False)
        back = gpt2.smp_to_hf(model.state_dict(gather_to_rank0=False))
        worst = max((back[k].float() - v.detach().float()).abs().max().item() for k, v in ref.state_dict().items())
        assert worst < 2e-4, worst
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
