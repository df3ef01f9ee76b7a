#!/usr/bin/env python
"""Headline benchmark: GPT-2 XL (1.5 B) training throughput at sequence length 2048.

Metric (BASELINE.json): samples/sec for the whole node.  Synthetic token data, random-init
weights, bf16 compute with fp32 master weights + fused AdamW, full training step
(forward, backward, gradient all-reduce over RCCL, optimizer step) through the smp API:
``smp.init`` -> ``smp.DistributedModel`` -> ``smp.DistributedOptimizer`` -> ``@smp.step``.

Single GPU:  python bench.py
N GPUs:      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
                 --master-port P bench.py --gpus N
Scaling is weak: the per-GPU micro-batch is fixed, global batch = mbs x microbatches x N/(pp*tp).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", 1)))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=None, help="override the model's layer count (tests only)")
    ap.add_argument("--layout", choices=["auto", "dp", "pp"], default="auto",
                    help="auto: N >= 4 GPUs (N %% 4 == 0) run BASELINE config 2 = GPT-2 XL PP=4 interleaved "
                         "x DP=N/4; fewer GPUs run data parallel.  dp: pure data parallel.  pp: PP=4 (x DP)")
    ap.add_argument("--mbs", type=int, default=None,
                    help="micro-batch size.  DP layout default 32 x 2048 tokens (GEMM M = 65536): amortises the "
                         "per-step optimizer / LM-head / transposition work and fills the chip with attention "
                         "blocks, ~190 GB of the 288 GB HBM3E (same-box A/B vs 16: +4.4 %% samples/s).  PP layout "
                         "default 16: one stage's work (12 layers + head) on one MI355X runs 117 / 134 / 142 samples/s "
                         "at mbs 4 / 8 / 16 (profiles/r3/pp_stage_mbs.md), the fastest measured; 16 x 32 "
                         "microbatches keeps the bubble at 8.6 %% and the in-flight activations of pp + 2 "
                         "microbatches (~33 GB per 16-sample microbatch set) well inside 288 GB")
    ap.add_argument("--microbatches", type=int, default=None,
                    help="DP default 1; PP default 32 (pipeline bubble (pp-1)/(m+pp-1) = 8.6 %% at PP=4; 16 x 32 = 512 "
                         "samples per pipeline per step)")
    ap.add_argument("--pp", type=int, default=None)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--head-cost", type=float, default=float(os.environ.get("SMP_BENCH_HEAD_COST", "2.4")),
                    help="PP layer split: cost of stage 0's tied embedding + LM head + loss in transformer-layer "
                         "units (2 h V vs 24 h^2 + attention FLOPs per token, plus the CE kernels)")
    ap.add_argument("--dropout", type=float, default=0.1,
                    help="attention / hidden / embedding dropout probability; default 0.1 = the GPT-2 XL and "
                         "smp.nn DistributedTransformer default (the reference trains with it on)")
    ap.add_argument("--no-flash", action="store_true")
    ap.add_argument("--activation-checkpointing", action="store_true")
    ap.add_argument("--shard-optimizer-state", action="store_true")
    ap.add_argument("--offload-optimizer-state", action="store_true",
                    help="fp32 master + Adam moments in pinned host memory (amd_offload_optimizer_state)")
    ap.add_argument("--tunableop", choices=["auto", "off", "use", "tune"], default="auto",
                    help="hipBLASLt/rocBLAS GEMM solution selection via PyTorch TunableOp: 'use' loads the "
                         "per-shape winners measured on MI355X (configs/tunableop), 'tune' re-measures them "
                         "during warmup; auto = use when a results file exists")
    return ap.parse_args()


def resolve_layout(args, world):
    """Fill pp / mbs / microbatches from the layout (explicit flags win)."""
    layout = args.layout
    if layout == "auto":
        layout = "pp" if (args.pp is None and world >= 4 and world % 4 == 0 and args.tp == 1) else "dp"
        if args.pp is not None and args.pp > 1:
            layout = "pp"
    if layout == "pp":
        args.pp = args.pp or 4
        args.mbs = args.mbs or 16
        args.microbatches = args.microbatches or 32
    else:
        args.pp = args.pp or 1
        args.mbs = args.mbs or 32
        args.microbatches = args.microbatches or 1
    args.layout = layout
    return args


def balanced_layer_split(num_layers, pp, head_cost):
    """Contiguous layer counts per stage minimising the most loaded stage, where stage 0 also
    runs the tied embedding + LM head + loss (cost `head_cost` layers): the main module and
    every module sharing the embedding weight stay on partition 0."""
    best = None

    def rec(i, left, counts):
        nonlocal best
        if i == pp - 1:
            counts = counts + [left]
            # most loaded stage first, then the next ones (prefer [10, 13, 13, 12] to [9, 13, 13, 13])
            key = sorted((c + (head_cost if j == 0 else 0.0) for j, c in enumerate(counts)), reverse=True)
            if best is None or key < best[0]:
                best = (key, counts)
            return
        for c in range(1, left - (pp - 1 - i) + 1):
            rec(i + 1, left - c, counts + [c])

    rec(0, num_layers, [])
    return best[1]


def tunableop_file(args):
    """Per-shape GEMM selections; the GEMM shapes depend on the micro-batch, sequence and TP
    degree but not on the pipeline degree, so a PP run falls back to the PP=1 file."""
    if os.environ.get("SMP_TUNABLEOP_FILE"):
        return os.environ["SMP_TUNABLEOP_FILE"]
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs", "tunableop")
    path = os.path.join(root, f"{args.model}_mbs{args.mbs}_s{args.seq}_pp{args.pp}_tp{args.tp}.csv")
    pp1 = os.path.join(root, f"{args.model}_mbs{args.mbs}_s{args.seq}_pp1_tp{args.tp}.csv")
    return path if (os.path.isfile(path) or not os.path.isfile(pp1) or args.tunableop == "tune") else pp1


def setup_tunableop(args):
    """GEMMs stay library GEMMs (hipBLASLt / rocBLAS): TunableOp picks, per shape, the
    fastest solution measured on this GPU instead of the library heuristic."""
    mode = args.tunableop
    path = tunableop_file(args)
    if mode == "auto":
        mode = "use" if os.path.isfile(path) else "off"
    if mode == "off" or not torch.cuda.is_available():
        return "off"
    tun = torch.cuda.tunable
    tun.enable(True)
    if mode == "use":
        tun.tuning_enable(False)
        tun.set_filename(path, insert_device_ordinal=False)
        if not tun.read_file(path):
            tun.enable(False)
            return "off"
    else:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(20)
        tun.set_max_tuning_iterations(30)
        # rotate operand copies through > the 256 MB MALL: pick solutions for cold caches,
        # as in the training step (operands arrive from HBM, not from a hot loop)
        tun.set_rotating_buffer_size(int(os.environ.get("SMP_TUNABLEOP_ROTATING_MB", "0")))
        tun.set_filename(path, insert_device_ordinal=False)
    return mode


def write_tunableop_results(path):
    """TunableOp results file: validator lines, then one line per tuned GEMM signature."""
    tun = torch.cuda.tunable
    lines = [f"Validator,{k},{v}" for k, v in tun.get_validators()]
    lines += [",".join(str(x) for x in r) for r in tun.get_results()]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def p2p_selfcheck():
    from smdistributed_modelparallel_amd.runtime.transport import SELFCHECK

    return SELFCHECK["verdict"]


def p2p_record(smp, args):
    """Pipeline transport facts for the record: mode, the init-time IPC self-check, and -- for
    IPC pulls -- the pull engine actually used (SDMA copies between distinct GPUs, a copy
    kernel within one) and how many exports went through the >1 GB staging pool."""
    tr = smp.state.transport if args.pp > 1 else None
    rec = {"mode": tr.mode if tr is not None else None, "ipc_selfcheck": p2p_selfcheck()}
    if tr is not None:
        st = tr.stats()
        for k in ("pull_engine", "pulls_sdma", "pulls_kernel", "mappings_remote_gpu", "staged_exports"):
            if k in st:
                rec[k] = st[k]
    return rec


def _lm_head_padded():
    from smdistributed_modelparallel_amd.ops import lm_head

    return bool(lm_head._ENABLED)


def device_record(smp, dev):
    """Every rank's (hostname, device index, GPU UUID): the record proves one rank per physical
    GPU.  Unless SMP_DEVICE_INDEX pins ranks on purpose (one-GPU rehearsals), two ranks of one
    host on the same GPU abort the bench."""
    import socket

    me = [socket.gethostname(), None, None]
    if dev.type == "cuda":
        me[1] = dev.index if dev.index is not None else torch.cuda.current_device()
        props = torch.cuda.get_device_properties(me[1])
        me[2] = str(getattr(props, "uuid", "")) or getattr(props, "pci_bus_id", None)
    allr = smp.allgather(me, smp.WORLD) if smp.size() > 1 else [me]
    if dev.type == "cuda" and not os.environ.get("SMP_DEVICE_INDEX"):
        seen = {}
        for r, (host, idx, uuid) in enumerate(allr):
            key = (host, uuid or idx)
            if key in seen:
                raise RuntimeError(f"ranks {seen[key]} and {r} share GPU {idx} ({uuid}) on {host}: the bench needs one "
                                   "rank per GPU")
            seen[key] = r
    return [{"rank": r, "device": idx, "uuid": uuid} for r, (host, idx, uuid) in enumerate(allr)]


def main():
    args = parse()
    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt, gpt_inputs
    from smdistributed_modelparallel_amd.models.gpt import train_flops_per_token
    from smdistributed_modelparallel_amd.ops.attention import FLASH_HEAD_DIMS

    world = int(os.environ.get("WORLD_SIZE", 1))
    resolve_layout(args, world)
    # an unattended multi-GPU run must not hang silently: a step running longer than this
    # dumps every thread's stack, ABORTs the peers and exits non-zero (backend/core.py
    # watchdog); TunableOp tuning steps run for minutes, so they get a longer budget
    os.environ.setdefault("SMP_STEP_TIMEOUT_S", "3600" if args.tunableop == "tune" else "600")
    cfg = {
        "pipeline_parallel_degree": args.pp,
        "tensor_parallel_degree": args.tp,
        "microbatches": args.microbatches,
        "ddp": world > 1 or args.tp > 1,
        "bf16": True,
        "amd_fused_attention": not args.no_flash,
        "shard_optimizer_state": args.shard_optimizer_state,
        "amd_offload_optimizer_state": args.offload_optimizer_state,
    }
    if os.environ.get("SMP_BENCH_ACTIVE_MB"):  # in-flight microbatches (default pp + 2)
        cfg["active_microbatches"] = int(os.environ["SMP_BENCH_ACTIVE_MB"])
    split = None
    if args.pp > 1:
        cfg["pipeline"] = "interleaved"
        # the step's module graph is identical every step: freeze and replay its schedule
        # (engine record-and-replay; the dynamic scheduler is the default otherwise)
        cfg["static_mode"] = os.environ.get("SMP_BENCH_STATIC", "1") != "0"
        if os.environ.get("SMP_BENCH_AUTO_PARTITION", "0") == "1":
            cfg["auto_partition"] = True
        else:
            cfg["auto_partition"] = False
            cfg["default_partition"] = 0
            split = balanced_layer_split(args.layers or GPT_CONFIGS[args.model]["num_layers"], args.pp,
                                         args.head_cost)
    smp.init(cfg)
    tmode = setup_tunableop(args)
    torch.manual_seed(1234 + smp.dp_rank())
    mc = GPT_CONFIGS[args.model]
    with smp.model_creation(tensor_parallelism=args.tp > 1, dtype=torch.float32):
        extra = {"num_layers": args.layers} if args.layers else {}
        model = build_gpt(args.model, dropout=args.dropout, num_positions=max(args.seq, mc["num_positions"]), **extra)
    if split is not None:
        layer_idx = 0
        for stage, cnt in enumerate(split):
            for _ in range(cnt):
                smp.set_partition(model.transformer.seq_layers[layer_idx], stage)
                layer_idx += 1
    model = smp.DistributedModel(model)
    if args.activation_checkpointing:
        for layer in model.get_module().transformer.seq_layers:
            smp.set_activation_checkpointing(layer)
    decay, no_decay = [], []
    for n, p in model.get_module().named_parameters():
        (no_decay if (p.dim() < 2 or "bias" in n or "norm" in n) else decay).append(p)
    inner = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1}, {"params": no_decay, "weight_decay": 0.0}],
                              lr=1e-4, betas=(0.9, 0.95), eps=1e-8)
    opt = smp.DistributedOptimizer(inner)

    @smp.step
    def train_step(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    dev = smp.state.device  # the device smp.init bound this rank to
    devices = device_record(smp, dev)
    batch = args.mbs * args.microbatches
    g = torch.Generator(device=dev)
    g.manual_seed(42 + smp.rank())
    data = [gpt_inputs(batch, args.seq, mc["vocab_size"], dev, generator=g) for _ in range(2)]

    def one(i):
        ids, mask, _, _, labels = data[i % len(data)]
        opt.zero_grad()
        out = train_step(model, ids, mask, labels)
        opt.step()
        return out

    if tmode == "tune" and smp.rank() == 0:
        # GEMM tuning runs silently for minutes: keep a heartbeat on stdout
        import threading

        t_start = time.time()

        def heartbeat():
            while True:
                time.sleep(60)
                print(f"tunableop: tuning in progress, {time.time() - t_start:.0f} s", flush=True)

        threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(args.warmup):
        out = one(i)
        if tmode == "tune" and smp.rank() == 0:
            print(f"tuning warmup step {i} done", flush=True)
    if tmode == "tune":
        torch.cuda.synchronize()
        torch.cuda.tunable.tuning_enable(False)
        if smp.rank() == 0:
            write_tunableop_results(tunableop_file(args))
    loss_val = float(out.reduce_mean()) if out is not None and smp.pp_rank() == 0 else float("nan")

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()

    from smdistributed_modelparallel_amd.parallel.comm_timer import timer as comm_timer

    from smdistributed_modelparallel_amd.ops.attention import FLASH_CALLS

    sync()
    fc0 = dict(FLASH_CALLS)
    comm_timer.reset()
    comm_timer.enabled = True  # two HIP events around each communication wait (no sync)
    t0 = time.perf_counter()
    step_times = os.environ.get("SMP_BENCH_STEP_TIMES") == "1"  # diagnostic: synchronises every step
    for i in range(args.steps):
        out = one(i)
        if step_times:
            torch.cuda.synchronize() if torch.cuda.is_available() else None
            print(f"rank {smp.rank()} timed step {i} ends at {1e3 * (time.perf_counter() - t0):.1f} ms",
                  file=sys.stderr, flush=True)
    sync()
    dt = time.perf_counter() - t0
    comm_timer.enabled = False
    exposed = comm_timer.collect()
    ex = torch.tensor([exposed["dp"], exposed["p2p"], exposed["tp"]], dtype=torch.float64, device=dev)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
    # flash-attention forward launches in the timed steps, summed over ranks
    fc = torch.tensor([FLASH_CALLS[k] - fc0[k] for k in ("plain", "key_bias")], dtype=torch.float64, device=dev)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(fc)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1000.0
    # scaled-batch TP: every data-parallel rank (TP ranks included) consumes its own batch
    global_batch = batch * smp.dp_size()
    samples_per_s = global_batch * args.steps / dt
    tokens_per_s = samples_per_s * args.seq
    flops = train_flops_per_token(args.model, args.seq) * tokens_per_s
    if smp.rank() == 0:
        par = f"pp{args.pp}xtp{args.tp}xdp{max(1, world // (args.pp * args.tp))}"
        rec = {
            "metric": ("samples/sec (whole node) GPT-2 XL seq2048" if (args.model, args.seq) == ("gpt2-xl", 2048)
                       else f"samples/sec (whole node) {args.model} seq{args.seq}"),
            "value": round(samples_per_s, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "model": args.model,
                "global_batch": global_batch,
                "seq_len": args.seq,
                "parallelism": par,
                "micro_batch_per_gpu": args.mbs,
                "microbatches": args.microbatches,
                "layout": args.layout,
                "pipeline": "interleaved" if args.pp > 1 else None,
                "layer_split": split,
                "p2p": smp.state.transport.mode if args.pp > 1 else None,
                "flash_attention": (not args.no_flash) and mc["attention_head_size"] in FLASH_HEAD_DIMS,
                "dropout": args.dropout,
                "gemm_selection": "tunableop" if tmode != "off" else "heuristic",
                # LM head + CE over the 64-padded vocabulary (ops/lm_head.py; same loss)
                "lm_head": "padded64" if _lm_head_padded() else "plain",
            },
            "dist_backend": dist.get_backend() if dist.is_initialized() else None,
            # world sizes of the process groups the backend actually formed (1: not created)
            "groups": {name: (dist.get_world_size(g) if g is not None else 1)
                       for name, g in (("world", smp.state.pgs.world), ("dp", smp.state.pgs.dp),
                                       ("pp", smp.state.pgs.pp), ("tp", smp.state.pgs.tp))},
            "p2p": p2p_record(smp, args),
            "devices": devices,
            # per-step compute-stream stall on communication (max over ranks): the DP bucket
            # all-reduces left after backward, pipeline activation / gradient pulls, and the
            # tensor-parallel collectives (the asynchronous dX all-reduce: its final wait only)
            "exposed_comm_ms": {"dp": round(float(ex[0]) / args.steps, 2), "p2p": round(float(ex[1]) / args.steps, 2),
                                "tp": round(float(ex[2]) / args.steps, 2)},
            "attention_calls": {"plain": int(fc[0]), "key_bias": int(fc[1])},
            "tokens_per_s": round(tokens_per_s, 1),
            "model_tflops_per_gpu": round(flops / world / 1e12, 1),
            "final_loss": round(loss_val, 4),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if torch.cuda.is_available() else None,
        }
        print(json.dumps(rec), flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
