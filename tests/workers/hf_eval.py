"""Worker (argv: pp tp): an HF GPT-2 trained, then evaluated under torch.no_grad() by a second
@smp.step function that returns (loss, logits) -- a tuple of StepOutputs, as in the reference --
then trained again; logits come back full-vocabulary on the first stage."""
import sys

import torch
import transformers as tf

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.split import StepOutput


def main():
    pp, tp = int(sys.argv[1]), int(sys.argv[2])
    smp.init({"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2,
              "auto_partition": True, "ddp": True})
    cfg = tf.GPT2Config(n_layer=4, n_embd=64, n_head=4, n_positions=64, vocab_size=97, bos_token_id=0, eos_token_id=0)
    torch.manual_seed(0)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net = tf.GPT2LMHeadModel(cfg)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-3))

    @smp.step
    def train_step(model, ids):
        out = model(input_ids=ids, labels=ids)
        model.backward(out.loss)
        return out.loss

    @smp.step
    def eval_step(model, ids):
        out = model(input_ids=ids, labels=ids)
        return out.loss, {"logits": out.logits}

    g = torch.Generator().manual_seed(1)
    for _ in range(2):
        opt.zero_grad()
        train_step(model, torch.randint(0, 97, (4, 16), generator=g))
        opt.step()
    model.eval()
    with torch.no_grad():
        res = eval_step(model, torch.randint(0, 97, (4, 16), generator=g))
    if smp.pp_rank() == 0:
        loss, extra = res
        assert isinstance(loss, StepOutput) and isinstance(extra["logits"], StepOutput)
        assert tuple(extra["logits"].concat().shape) == (4, 16, 97)
        assert 3.0 < float(loss.reduce_mean()) < 6.0
    model.train()
    opt.zero_grad()
    out = train_step(model, torch.randint(0, 97, (4, 16), generator=g))
    opt.step()
    if smp.pp_rank() == 0:
        assert isinstance(out, StepOutput) and torch.isfinite(out.reduce_mean())
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
