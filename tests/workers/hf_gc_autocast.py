"""Worker (argv: pp tp mode): an HF GPT-2 through smp with (mode "gc") Hugging Face gradient
checkpointing enabled -- under PP its layers switch to smp activation checkpointing -- or
(mode "autocast") the step run under torch.autocast(bf16) with fp32 parameters (the TP linear's
backward handles the mixed dtypes).  The same fixed batch every step: the loss must fall."""
import sys

import torch
import transformers as tf

import smdistributed_modelparallel_amd.torch as smp


def main():
    pp, tp, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    smp.init({"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2,
              "auto_partition": True, "ddp": True})
    torch.manual_seed(0)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net = tf.GPT2LMHeadModel(tf.GPT2Config(n_layer=4, n_embd=64, n_head=4, n_positions=64, vocab_size=97,
                                               resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0))
    if mode == "gc":
        net.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
    net.train()
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=3e-3))
    dev = smp.state.device

    @smp.step
    def step(model, ids):
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=mode == "autocast"):
            out = model(input_ids=ids, labels=ids)
        model.backward(out.loss)
        return out.loss

    ids = torch.randint(0, 97, (4, 16), generator=torch.Generator().manual_seed(1)).to(dev)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        losses.append(step(model, ids))
        opt.step()
    if smp.pp_rank() == 0:
        v = [float(x.reduce_mean()) for x in losses]
        assert all(torch.isfinite(torch.tensor(v))) and v[-1] < v[0], v
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
