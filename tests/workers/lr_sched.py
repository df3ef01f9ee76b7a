"""Worker (argv: pp tp): torch.optim.lr_scheduler on smp.DistributedOptimizer (an Optimizer by
type), with gradient accumulation over two @smp.step calls (backward_passes_per_step=2): the
inner optimizer's groups carry the scheduled learning rate and the model trains."""
import sys

import torch
import transformers as tf

import smdistributed_modelparallel_amd.torch as smp


def main():
    pp, tp = int(sys.argv[1]), int(sys.argv[2])
    smp.init({"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2,
              "auto_partition": True, "ddp": True})
    torch.manual_seed(0)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net = tf.GPT2LMHeadModel(tf.GPT2Config(n_layer=4, n_embd=64, n_head=4, n_positions=64, vocab_size=97,
                                               resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0))
    model = smp.DistributedModel(net, backward_passes_per_step=2)
    inner = torch.optim.AdamW(model.parameters(), lr=1e-2)
    opt = smp.DistributedOptimizer(inner)
    assert isinstance(opt, torch.optim.Optimizer)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))

    @smp.step
    def step(model, ids):
        out = model(input_ids=ids, labels=ids)
        model.backward(out.loss)
        return out.loss

    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 97, (4, 16), generator=g)
    first = last = None
    for it in range(4):
        for _ in range(2):
            loss = step(model, ids)
        opt.step()
        sched.step()
        opt.zero_grad()
        assert abs(inner.param_groups[0]["lr"] - 1e-2 / (2 + it)) < 1e-12, inner.param_groups[0]["lr"]
        if smp.pp_rank() == 0:
            v = float(loss.reduce_mean())
            first = v if first is None else first
            last = v
    if smp.pp_rank() == 0:
        assert last < first, (first, last)  # same batch every step: the loss must fall
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
