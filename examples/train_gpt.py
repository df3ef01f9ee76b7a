#!/usr/bin/env python
"""End-to-end training script on the smp API (the reference's usage pattern, unchanged).

One process per GPU (torchrun), any mix of pipeline / tensor / data parallelism:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        examples/train_gpt.py --model gpt2-xl --pp 2 --tp 2 --microbatches 4 --steps 100 \
        --ckpt-dir /tmp/ckpt --ckpt-every 50

BASELINE.json configurations map to:
    GPT-2 XL PP=4 interleaved       --model gpt2-xl --pp 4 --microbatches 8
    GPT-J 6B TP=4                   --model gptj-6b --tp 4
    GPT-NeoX 20B PP=2 x TP=4        --model gptneox-20b --pp 2 --tp 4 --shard-optimizer-state
    GPT-3 175B-shape PP=4 x TP=2    --model gpt3-175b --pp 4 --tp 2 --activation-checkpointing
                                    --offload-activations --delayed-init
CPU smoke (gloo): add --cpu and a tiny --model gpt2-tiny (tests/test_examples_cpu.py).
Synthetic data; resumes from the newest partial checkpoint in --ckpt-dir when present.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--layers", type=int, default=None, help="override the depth (smoke runs)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--mbs", type=int, default=2, help="micro-batch size per data-parallel rank")
    ap.add_argument("--microbatches", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--clip", type=float, default=1.0)
    ap.add_argument("--activation-checkpointing", action="store_true")
    ap.add_argument("--offload-activations", action="store_true")
    ap.add_argument("--shard-optimizer-state", action="store_true")
    ap.add_argument("--delayed-init", action="store_true")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--cpu", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    if args.cpu:
        os.environ["SMP_FORCE_CPU"] = "1"
    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt, gpt_inputs

    world = int(os.environ.get("WORLD_SIZE", 1))
    smp.init({
        "pipeline_parallel_degree": args.pp,
        "tensor_parallel_degree": args.tp,
        "microbatches": args.microbatches,
        "pipeline": "interleaved",
        "auto_partition": args.pp > 1,
        "ddp": world > 1,
        "bf16": not args.cpu,
        "shard_optimizer_state": args.shard_optimizer_state,
        "offload_activations": args.offload_activations,
        "delayed_parameter_initialization": args.delayed_init,
    })
    mc = GPT_CONFIGS[args.model]
    over = {"num_positions": max(args.seq, mc["num_positions"])}
    if args.layers:
        over["num_layers"] = args.layers
    torch.manual_seed(1234)
    with smp.delay_param_initialization(enabled=args.delayed_init):
        with smp.model_creation(tensor_parallelism=args.tp > 1):
            net = build_gpt(args.model, dropout=0.0, **over)
    model = smp.DistributedModel(net)
    if args.activation_checkpointing:
        for layer in model.get_module().transformer.seq_layers:
            smp.set_activation_checkpointing(layer)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=args.lr, betas=(0.9, 0.95),
                                                     weight_decay=0.1))

    start = 0
    if args.ckpt_dir and os.path.isfile(os.path.join(args.ckpt_dir, "newest")):
        user = smp.resume_from_checkpoint(args.ckpt_dir, partial=True)
        start = int((user or {}).get("step", 0))
        if smp.rank() == 0:
            print(f"resumed from {args.ckpt_dir} at step {start}", flush=True)

    @smp.step
    def train_step(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    dev = smp.state.device
    g = torch.Generator(device=dev)
    g.manual_seed(7 + smp.dp_rank())
    batch = args.mbs * args.microbatches
    t0 = time.time()
    for step in range(start, args.steps):
        ids, mask, _, _, labels = gpt_inputs(batch, args.seq, mc["vocab_size"], dev, generator=g)
        opt.zero_grad()
        out = train_step(model, ids, mask, labels)
        if args.clip > 0:
            opt.clip_master_grads(args.clip)
        opt.step()
        if smp.pp_rank() == 0 and smp.tp_rank() == 0 and smp.rdp_rank() == 0:
            loss = float(out.reduce_mean())
            print(f"step {step + 1} loss {loss:.4f} ({time.time() - t0:.1f}s)", flush=True)
        if args.ckpt_dir and args.ckpt_every and (step + 1) % args.ckpt_every == 0:
            smp.save_checkpoint(args.ckpt_dir, tag=f"step{step + 1}", partial=True, model=model, optimizer=opt,
                                user_content={"step": step + 1})
    smp.barrier()
    if smp.rank() == 0:
        print("TRAIN_DONE", flush=True)


if __name__ == "__main__":
    main()
