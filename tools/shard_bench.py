#!/usr/bin/env python
"""Heaviest-rank shards of BASELINE configs 3 and 4 on one MI355X.

One tensor-parallel rank computes the whole model's layers at its TP-sliced shapes: every
attention block holds heads / tp heads, every MLP intermediate / tp channels and the LM head
vocab / tp rows.  The shard is built at tp = 1 with those shapes, so the per-rank compute of a
step is measured exactly; the TP all-reduces of the layer outputs are not (their cost is
estimated separately in the profile, see `comm_estimate`).

    gptj_tp4      config 3, GPT-J 6B at TP=4: 28 layers, 4 of 16 heads x 256, 4096 of 16384
                  MLP channels, rotary 64, parallel attention + MLP, 12600 of 50400 vocab rows
    neox_pp2tp4   config 4, GPT-NeoX 20B at PP=2 x TP=4, the last stage (heavier: LM head):
                  22 of 44 layers, 16 of 64 heads x 96, 6144 of 24576 MLP channels, NeoX
                  rotary 24, 12608 of 50432 vocab rows

    python tools/shard_bench.py gptj_tp4 --mbs 8 --steps 5 --warmup 3

bf16 params / grads, fp32 master weights + AdamW in HBM, no activation checkpointing, no
dropout (the GPT-J / NeoX training configs use none), synthetic tokens, seq 2048.  Prints one
JSON line: ms/step, tokens/s of the shard, model TFLOP/s of the shard's work (6 N_shard + the
shard's attention per token), peak HBM, and the TP all-reduce estimate.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHARDS = {
    "gptj_tp4": dict(base="gptj-6b", tp=4, layers=28),
    "neox_pp2tp4": dict(base="gptneox-20b", tp=4, layers=22),
}


def shard_overrides(name, seq):
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS

    s = SHARDS[name]
    c = GPT_CONFIGS[s["base"]]
    tp = s["tp"]
    return s["base"], dict(num_layers=s["layers"], num_attention_heads=c["num_attention_heads"] // tp,
                           intermediate_size=c["intermediate_size"] // tp,
                           vocab_size=(c["vocab_size"] + tp - 1) // tp, num_positions=max(seq, c["num_positions"]))


def comm_estimate(h, tokens, layers, tp, link_gbs=64.0, links=None):
    """TP all-reduce estimate (NOT measured): per layer with parallel attention + MLP one
    forward and one backward all-reduce of [tokens, h] bf16 (the reference's
    DistributedTransformer reduces the summed attention + MLP output once).  A ring over tp
    ranks moves 2 (tp - 1) / tp of the message per rank; with one xGMI link per peer
    (7 links x ~64 GB/s per direction on a fully connected 8-GPU node) a tp-rank ring uses
    tp - 1 links per rank in parallel when the collective is split per link (RCCL's
    multi-ring), so the per-rank time is bytes * 2 (tp - 1) / tp / ((tp - 1) * link_gbs)."""
    links = tp - 1 if links is None else links
    msg = tokens * h * 2
    per_ar = msg * 2 * (tp - 1) / tp / (links * link_gbs * 1e9)
    return {"all_reduces_per_step": 2 * layers, "message_mb": round(msg / 1e6, 1),
            "per_all_reduce_ms": round(per_ar * 1e3, 3), "per_step_ms": round(2 * layers * per_ar * 1e3, 1),
            "model": f"ring over {tp} ranks, {links} xGMI links x {link_gbs} GB/s per rank, no overlap"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shard", choices=sorted(SHARDS))
    ap.add_argument("--mbs", type=int, default=8)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=None, help="override the layer count (smoke tests)")
    ap.add_argument("--tunableop", choices=["auto", "off", "use", "tune"], default="auto",
                    help="per-shape GEMM solutions (configs/tunableop/<shard>_mbs<m>_s<s>.csv): 'tune' measures "
                         "them during warmup and writes the file, auto = use when the file exists")
    args = ap.parse_args()

    import torch

    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt, gpt_inputs

    os.environ.setdefault("SMP_STEP_TIMEOUT_S", "3600" if args.tunableop == "tune" else "600")
    import bench  # the repo-root benchmark's TunableOp helpers

    tfile = os.path.join(ROOT, "configs", "tunableop", f"{args.shard}_mbs{args.mbs}_s{args.seq}.csv")
    os.environ["SMP_TUNABLEOP_FILE"] = tfile
    tmode = bench.setup_tunableop(argparse.Namespace(tunableop=args.tunableop))
    smp.init({"bf16": True, "ddp": False})
    base, ov = shard_overrides(args.shard, args.seq)
    if args.layers:
        ov["num_layers"] = args.layers
    with smp.model_creation(dtype=torch.float32):
        net = build_gpt(base, dropout=0.0, **ov)
    model = smp.DistributedModel(net)
    decay, no_decay = [], []
    for n, p in model.get_module().named_parameters():
        (no_decay if (p.dim() < 2 or "bias" in n or "norm" in n) else decay).append(p)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(
        [{"params": decay, "weight_decay": 0.1}, {"params": no_decay, "weight_decay": 0.0}], lr=1e-4,
        betas=(0.9, 0.95), eps=1e-8))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    dev = smp.state.device
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    ids, mask, _, _, labels = gpt_inputs(args.mbs, args.seq, ov["vocab_size"], dev, generator=g)

    def one():
        opt.zero_grad()
        out = train(model, ids, mask, labels)
        opt.step()
        return out

    if tmode == "tune":  # tuning steps can run for minutes: keep printing
        import threading

        t_start = time.time()
        done = threading.Event()

        def beat():
            while not done.wait(30):
                print(f"tunableop: tuning in progress, {time.time() - t_start:.0f} s", flush=True)

        threading.Thread(target=beat, daemon=True).start()
    for i in range(args.warmup):
        out = one()
        print(f"warmup {i}: loss {float(out.reduce_mean()):.4f}", flush=True)
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    sync()
    if tmode == "tune":
        done.set()
        torch.cuda.tunable.tuning_enable(False)
        bench.write_tunableop_results(tfile)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one()
    sync()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    n = sum(p.numel() for p in model.get_module().parameters())
    c = dict(ov)
    att = c["num_attention_heads"] * GPT_CONFIGS[base]["attention_head_size"]
    tokens = args.mbs * args.seq
    flops_tok = 6 * n + 12 * c["num_layers"] * att * args.seq
    h = GPT_CONFIGS[base]["hidden_size"]
    rec = {"shard": args.shard, "base": base, "tp": SHARDS[args.shard]["tp"], "params_shard": n, "mbs": args.mbs,
           "seq": args.seq, "ms_per_step": round(ms, 1), "tokens_per_s": round(tokens / ms * 1e3, 1),
           "samples_per_s": round(args.mbs / ms * 1e3, 3),
           "model_tflops_shard": round(flops_tok * tokens / ms / 1e9, 1),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2) if torch.cuda.is_available() else None,
           "final_loss": round(float(out.reduce_mean()), 4), "gemm_selection": tmode,
           "comm_estimate": comm_estimate(h, tokens, c["num_layers"], SHARDS[args.shard]["tp"])}
    print("SHARD " + json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
