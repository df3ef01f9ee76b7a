#!/usr/bin/env python
"""Max trainable parameter count (second BASELINE.json metric) -- measured on 1 MI355X,
projected to 8 with sharded data parallelism.

probe mode (one process, one model size):
    python tools/max_params.py probe --layers L [--hidden 6144]
builds a GPT (h=6144, 48 heads x 128, 4h MLP, L layers) with delayed parameter
initialisation (materialised straight on the GPU), activation checkpointing on every
layer, bf16 params/grads + fp32 master weights + fused AdamW (16 B/param of model state),
runs two full training steps (fwd, recompute bwd, optimizer) at micro-batch 1 x seq 2048
and prints one JSON line {"ok", "params", "peak_mem_gb", ...}.

search mode:
    python tools/max_params.py search [--lo 20 --hi 40] [--out profiles/max_params.json]
binary-searches L with one probe subprocess per size (an OOM ends only that probe) and
writes the largest size that trained, its measured peak memory, and the 8-GPU projection:
with sharded data parallelism over 8 ranks (parallel/sharded_dp.py: params, grads,
master weights and optimizer state all sharded) the per-GPU model state is 16/8 B/param,
plus the non-shardable per-GPU part measured here (activations, one gathered layer of
bf16 params + grads, workspaces).  The projection is arithmetic on the measured numbers,
not an 8-GPU run (8-GPU runs belong to the driver).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def probe(args):
    import torch

    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs

    smp.init({"bf16": True, "delayed_parameter_initialization": True})
    h = args.hidden
    heads = h // 128
    with smp.delay_param_initialization():
        with smp.model_creation(dtype=torch.bfloat16):
            net = build_gpt("gpt2-xl", dropout=0.0, num_layers=args.layers, hidden_size=h, num_attention_heads=heads,
                            attention_head_size=128, intermediate_size=4 * h, num_positions=args.seq)
    model = smp.DistributedModel(net)
    for layer in model.get_module().transformer.seq_layers:
        smp.set_activation_checkpointing(layer)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-5, betas=(0.9, 0.95)))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    dev = smp.state.device
    ids, mask, _, _, labels = gpt_inputs(args.mbs, args.seq, 50257, dev)
    t0 = time.time()
    losses = []
    for _ in range(2):
        opt.zero_grad()
        out = train(model, ids, mask, labels)
        opt.step()
        losses.append(float(out.reduce_mean()))
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.synchronize()
    n = sum(p.numel() for p in model.get_module().parameters())
    rec = {"ok": all(l == l for l in losses), "layers": args.layers, "hidden": h, "params": n,
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2) if gpu else None,
           "peak_reserved_gb": round(torch.cuda.max_memory_reserved() / 1e9, 2) if gpu else None,
           "hbm_gb": round(torch.cuda.get_device_properties(dev).total_memory / 1e9, 2) if gpu else None,
           "step_s": round((time.time() - t0) / 2, 2), "losses": [round(l, 4) for l in losses]}
    print("MAXPARAMS " + json.dumps(rec), flush=True)


def _host_rss_gb():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmHWM:"):
                return int(line.split()[1]) / 1e6
    return None


def shard(args):
    """BASELINE config 5 (GPT-3 175B shape, PP=4 x TP=2) -- ONE rank's shard on one GPU: the
    heaviest stage (embedding + 24 of the 96 layers; --layers sets more per stage) with every tensor-parallel dimension
    halved (48 of the 96 heads x 128, 4h / 2 = 24576 MLP channels, half the vocabulary), built
    at tp=1 with those sliced shapes.  bf16 params / grads, AdamW with the fp32 state fields
    named by SMP_OFFLOAD_OPTIMIZER_FIELDS in pinned host memory (amd_offload_optimizer_state),
    activation checkpointing on every layer, micro-batch 1 x seq 2048, 3 full steps."""
    import torch

    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs

    smp.init({"bf16": True, "delayed_parameter_initialization": True, "amd_offload_optimizer_state": True})
    h, tp = 12288, 2
    vocab = (50257 + tp - 1) // tp
    with smp.delay_param_initialization():
        with smp.model_creation(dtype=torch.bfloat16):
            net = build_gpt("gpt3-175b", dropout=0.0, num_layers=args.layers, hidden_size=h,
                            num_attention_heads=96 // tp, attention_head_size=128, intermediate_size=4 * h // tp,
                            vocab_size=vocab, num_positions=args.seq)
    model = smp.DistributedModel(net)
    for layer in model.get_module().transformer.seq_layers:
        smp.set_activation_checkpointing(layer)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-5, betas=(0.9, 0.95)))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    dev = smp.state.device
    ids, mask, _, _, labels = gpt_inputs(args.mbs, args.seq, vocab, dev)
    losses, times = [], []
    for i in range(3):
        t0 = time.time()
        opt.zero_grad()
        out = train(model, ids, mask, labels)
        opt.step()
        losses.append(float(out.reduce_mean()))
        torch.cuda.synchronize()
        times.append(round(time.time() - t0, 2))
        print(f"shard step {i}: loss {losses[-1]:.4f} {times[-1]} s", flush=True)
    n = sum(p.numel() for p in model.get_module().parameters())
    host_state = sum(t.numel() * t.element_size() for d in opt.domains for t in (d.master, d.m, d.v)
                     if t is not None and not t.is_cuda)
    rec = {"ok": all(l == l for l in losses), "config": "GPT-3 175B shape, PP=4 x TP=2: one rank's shard "
           f"(embedding + {args.layers} layers, TP-sliced shapes at tp=1)", "layers": args.layers, "hidden": h,
           "heads_local": 96 // tp, "intermediate_local": 4 * h // tp, "vocab_local": vocab, "params": n,
           "offloaded_fields": sorted(opt._offload_fields), "host_state_gb": round(host_state / 1e9, 2),
           "host_peak_rss_gb": round(_host_rss_gb() or 0.0, 2),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2),
           "peak_reserved_gb": round(torch.cuda.max_memory_reserved() / 1e9, 2),
           "hbm_gb": round(torch.cuda.get_device_properties(dev).total_memory / 1e9, 2),
           "step_s": times, "losses": [round(l, 4) for l in losses]}
    print("MAXPARAMS " + json.dumps(rec), flush=True)


def run_probe(layers, args):
    cmd = [sys.executable, os.path.abspath(__file__), "probe", "--layers", str(layers), "--hidden", str(args.hidden),
           "--seq", str(args.seq), "--mbs", str(args.mbs)]
    print(f"probe L={layers} ...", flush=True)
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=args.probe_timeout)
    except subprocess.TimeoutExpired:
        print(f"probe L={layers}: timeout", flush=True)
        return None
    for line in r.stdout.splitlines():
        if line.startswith("MAXPARAMS "):
            rec = json.loads(line[len("MAXPARAMS "):])
            print(f"probe L={layers}: {rec}", flush=True)
            return rec if rec["ok"] else None
    tail = "\n".join(r.stdout.splitlines()[-4:])
    print(f"probe L={layers}: failed rc={r.returncode}\n{tail}", flush=True)
    return None


def search(args):
    lo, hi = args.lo, args.hi
    best = None
    while lo <= hi:
        mid = (lo + hi) // 2
        rec = run_probe(mid, args)
        if rec is not None:
            best, lo = rec, mid + 1
        else:
            hi = mid - 1
    if best is None:
        print("no size trained", flush=True)
        return 1
    h, p = best["hidden"], best["params"]
    state_b = 16.0  # bf16 param + bf16 grad + fp32 master + fp32 exp_avg + fp32 exp_avg_sq
    non_state = best["peak_mem_gb"] * 1e9 - state_b * p  # activations, workspaces, allocator slack
    layer_params = 12 * h * h
    gathered = 2 * 2 * layer_params  # one gathered layer: bf16 params + bf16 grads (sharded DP working set)
    usable = best["hbm_gb"] * 1e9 * 0.97
    per_gpu_fixed = max(non_state, 0.0) + gathered
    proj8 = int(8 * (usable - per_gpu_fixed) / state_b)
    out = {
        "metric": "max trainable params",
        "measured_1gpu": best,
        "bytes_per_param_model_state": state_b,
        "non_state_gb_measured": round(non_state / 1e9, 2),
        "projection_8gpu_sharded_dp8": {
            "params": proj8,
            "assumes": "sharded_data_parallel_degree=8 (params, grads, fp32 master and Adam state sharded 8 ways), "
                       "activation checkpointing, mbs 1 x seq 2048; per-GPU fixed part = measured non-state memory "
                       "+ one gathered layer (bf16 params + grads); 97% of HBM usable",
        },
        "note": "measured: one MI355X trains the 1-GPU model (2 steps, finite loss); 8-GPU value is a projection",
    }
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["probe", "search", "shard"])
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--hidden", type=int, default=6144)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--lo", type=int, default=20)
    ap.add_argument("--hi", type=int, default=40)
    ap.add_argument("--probe-timeout", type=int, default=300)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "max_params.json"))
    args = ap.parse_args()
    if args.mode == "probe":
        probe(args)
        return 0
    if args.mode == "shard":
        shard(args)
        return 0
    return search(args)


if __name__ == "__main__":
    sys.exit(main())
