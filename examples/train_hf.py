#!/usr/bin/env python
"""Hugging Face causal-LM training on the smp API: the pattern SageMaker model-parallel users run,
unchanged apart from the import.

A `transformers` model built from its config (random init; no hub access needed) is handed to
smp.DistributedModel.  Pipeline parallelism partitions the HF module tree (auto-partition);
tensor parallelism replaces supported HF models (GPT-2, GPT-J, GPT-Neo, GPT-NeoX) with smp.nn's
DistributedTransformerLMHead when they are created under `smp.model_creation(tensor_parallelism=
True)`, with the HF weights translated in (`nn/huggingface/*`).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        examples/train_hf.py --family gpt2 --layers 48 --hidden 1600 --heads 25 --pp 4 \\
        --microbatches 8 --steps 50 --ckpt-dir /tmp/hf_ckpt --ckpt-every 25

CPU smoke (gloo): --cpu with a tiny shape (tests/test_examples_cpu.py).  Synthetic tokens;
resumes from the newest partial checkpoint in --ckpt-dir when present.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", choices=["gpt2", "gptj", "gpt_neox"], default="gpt2")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--mbs", type=int, default=2, help="micro-batch size per data-parallel rank")
    ap.add_argument("--microbatches", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--activation-checkpointing", action="store_true", help="checkpoint every transformer block")
    ap.add_argument("--shard-optimizer-state", action="store_true")
    ap.add_argument("--delayed-init", action="store_true")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--cpu", action="store_true")
    return ap.parse_args()


def hf_model(args):
    """A transformers causal LM of the requested family and shape, random init."""
    import transformers as tf

    common = dict(vocab_size=args.vocab, bos_token_id=0, eos_token_id=0)
    if args.family == "gpt2":
        cfg = tf.GPT2Config(n_layer=args.layers, n_embd=args.hidden, n_head=args.heads,
                            n_positions=max(args.seq, 1024), **common)
        return tf.GPT2LMHeadModel(cfg)
    if args.family == "gptj":
        cfg = tf.GPTJConfig(n_layer=args.layers, n_embd=args.hidden, n_head=args.heads, n_positions=args.seq,
                            rotary_dim=max(8, args.hidden // args.heads // 4), **common)
        return tf.GPTJForCausalLM(cfg)
    cfg = tf.GPTNeoXConfig(num_hidden_layers=args.layers, hidden_size=args.hidden, num_attention_heads=args.heads,
                           intermediate_size=4 * args.hidden, max_position_embeddings=args.seq, **common)
    return tf.GPTNeoXForCausalLM(cfg)


def main():
    args = parse()
    if args.cpu:
        os.environ["SMP_FORCE_CPU"] = "1"
    import smdistributed_modelparallel_amd.torch as smp

    world = int(os.environ.get("WORLD_SIZE", 1))
    smp.init({
        "pipeline_parallel_degree": args.pp,
        "tensor_parallel_degree": args.tp,
        "microbatches": args.microbatches,
        "pipeline": "interleaved",
        "auto_partition": True,
        "ddp": world > 1,
        "bf16": not args.cpu,
        "shard_optimizer_state": args.shard_optimizer_state,
        "delayed_parameter_initialization": args.delayed_init,
    })
    torch.manual_seed(1234)
    with smp.delay_param_initialization(enabled=args.delayed_init):
        with smp.model_creation(tensor_parallelism=args.tp > 1,
                                dtype=torch.float32 if args.cpu else torch.bfloat16):
            net = hf_model(args)
    model = smp.DistributedModel(net)
    if args.activation_checkpointing:
        # the transformer blocks: HF ModuleList children, or smp.nn's layer stack after the TP swap
        inner = model.get_module()
        stack = getattr(getattr(inner, "transformer", None), "seq_layers", None)
        if stack is None:
            body = getattr(inner, "transformer", None) or getattr(inner, "gpt_neox", None)
            stack = getattr(body, "h", None) or getattr(body, "layers", None)
        for block in stack:
            smp.set_activation_checkpointing(block)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=0.01))

    start = 0
    if args.ckpt_dir and os.path.isfile(os.path.join(args.ckpt_dir, "newest")):
        user = smp.resume_from_checkpoint(args.ckpt_dir, partial=True)
        start = int((user or {}).get("step", 0))
        if smp.rank() == 0:
            print(f"resumed from {args.ckpt_dir} at step {start}", flush=True)

    @smp.step
    def train_step(model, ids):
        out = model(input_ids=ids, labels=ids)
        model.backward(out.loss)
        return out.loss

    dev = smp.state.device
    g = torch.Generator(device=dev)
    batch = args.mbs * args.microbatches
    t0 = time.time()
    for step in range(start, args.steps):
        g.manual_seed(7 + smp.dp_rank() + 1000 * step)  # per-step batches: a resumed run sees the same data
        ids = torch.randint(0, args.vocab, (batch, args.seq), device=dev, generator=g)
        opt.zero_grad()
        out = train_step(model, ids)
        opt.step()
        if smp.pp_rank() == 0 and smp.tp_rank() == 0 and smp.rdp_rank() == 0:
            print(f"step {step + 1} loss {float(out.reduce_mean()):.4f} ({time.time() - t0:.1f}s)", flush=True)
        if args.ckpt_dir and args.ckpt_every and (step + 1) % args.ckpt_every == 0:
            smp.save_checkpoint(args.ckpt_dir, tag=f"step{step + 1}", partial=True, model=model, optimizer=opt,
                                user_content={"step": step + 1})
    smp.barrier()
    if smp.rank() == 0:
        print("TRAIN_DONE", flush=True)


if __name__ == "__main__":
    main()
