"""Worker: GPT pipeline/data/tensor-parallel training vs an unpartitioned reference.

argv: pp tp microbatches pipeline(simple|interleaved) auto(0|1) steps [extra_json]
Each rank trains the smp model and an identical plain-PyTorch model on the same global
batch and checks loss and parameters after every step.

Gradient checks (reference `test/torch/smp_test_base.py:731-788`), on the first step, before
the optimizer update, per local (TP-sliced) parameter as a relative norm |g - g_ref| / |g_ref|:
* ``grad_tol``: against the same architecture run unpartitioned in the same dtype;
* ``fp32_ref_tol``: against the independent plain-torch fp32 model of tests/torch_ref.py on the
  initial weights (no smp module, no HIP kernel) -- a looser bound, since it also measures the
  reduced-precision rounding of the smp run.
``seq`` sets the sequence length (default 16); ``break_tp_bwd`` drops the column-parallel
input-gradient all-reduce on every rank (a mutation the gradient check must catch).
"""
import json
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    pp, tp, mbs, pipe, auto, steps = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                                      int(sys.argv[5]), int(sys.argv[6]))
    extra = json.loads(sys.argv[7]) if len(sys.argv) > 7 else {}
    world = int(__import__("os").environ["WORLD_SIZE"])
    cfg = {"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": mbs, "pipeline": pipe,
           "ddp": world > pp, "auto_partition": bool(auto)}
    if not auto:
        cfg["default_partition"] = 0
    cfg.update(extra.get("cfg", {}))
    torch.manual_seed(123)
    base = extra.get("base", "gpt2-tiny")
    if base == "gpt2-tiny":
        kw = dict(num_layers=4, hidden_size=64, num_attention_heads=4, attention_head_size=16, intermediate_size=128,
                  vocab_size=96, num_positions=32)
    else:  # a BASELINE architecture at full width, few layers, small vocabulary
        kw = dict(num_layers=2, vocab_size=1024, num_positions=64)
    kw.update(extra.get("model", {}))
    # learned position embeddings must cover the sequence (an out-of-range position id is an
    # out-of-bounds gather on the GPU)
    kw["num_positions"] = max(kw["num_positions"], int(extra.get("seq", 16)))
    # reduced precision (tests/test_hybrid_gpu.py): the smp model in bf16 / fp16 with fp32 master
    # weights against the SAME architecture run in that dtype without smp
    low = extra.get("dtype")
    ldt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(low)
    if low:
        cfg[low] = True
    ref = build_gpt(base, dropout=0.0, **kw)  # built before init: unsharded reference
    smp.init(cfg)
    dev = smp.state.device  # GPU runs (tests/test_hybrid_gpu.py): every rank on the box's one GPU
    ref.to(dev)
    if cfg.get("shard_optimizer_state") or cfg.get("sharded_data_parallel_degree", 1) > 1:
        # each rank holds only its shard of the reduced gradients: no per-parameter check
        extra.pop("grad_tol", None)
        extra.pop("fp32_ref_tol", None)
    fp32_tol = extra.get("fp32_ref_tol")
    sd0 = {k: v.detach().float().clone() for k, v in ref.state_dict().items()} if fp32_tol else None
    if ldt is not None:
        ref.to(ldt)
    if extra.get("break_tp_bwd"):
        import smdistributed_modelparallel_amd.nn.transformer as tr

        tr.dx_allreduce_async = lambda dx: None  # mutation: column-parallel dX never all-reduced
    delayed = bool(extra.get("delayed"))
    with smp.delay_param_initialization(enabled=delayed):
        with smp.model_creation(tensor_parallelism=tp > 1):
            net = build_gpt(base, dropout=0.0, **kw)
    if delayed:
        assert all(p.is_meta for p in net.parameters())
    elif tp == 1:
        net.load_state_dict({k: v.cpu() for k, v in ref.state_dict().items()})
    else:
        from smdistributed_modelparallel_amd.torch.checkpoint_utils import slice_for_param

        # distributed modules created under TP: copy the sliced reference weights
        rsd = {k: v.cpu() for k, v in ref.state_dict().items()}
        with torch.no_grad():
            for n, p in net.named_parameters():
                full = rsd[n]
                axis = getattr(p, "_smp_tp_axis", None)
                t = slice_for_param(full, p, smp.tp_rank(), smp.tp_size())
                assert t.shape == p.shape, (n, tuple(full.shape), tuple(t.shape), tuple(p.shape), axis)
                p.copy_(t)
    if not auto and pp > 1:
        # manual: first half of the layers on stage 0, rest on stage 1 (embeddings + head on 0)
        layers = list(net.transformer.seq_layers)
        for i, layer in enumerate(layers):
            smp.set_partition(layer, (i * pp) // len(layers))
    model = smp.DistributedModel(net, **extra.get("dm_kwargs", {}))
    if delayed:
        # meta parameters: the reference weights load once the partition has materialised them
        model.load_state_dict(ref.state_dict())
    if extra.get("jitter"):
        # perturb message timing differently on every rank: TP peers must still agree on order
        import random
        import time

        rnd = random.Random(smp.rank() * 7919 + 1)
        tr = smp.state.transport
        orig_send = tr.send

        def jittery_send(*a, **k):
            time.sleep(rnd.random() * 0.003)
            return orig_send(*a, **k)

        tr.send = jittery_send
    if extra.get("ckpt_layers"):
        for layer in model.get_module().transformer.seq_layers:
            smp.set_activation_checkpointing(layer)
    lr = 0.05
    if low == "fp16":
        # dynamic loss scaling (reference test_gpt_grad.py:121-154 fp16 variants)
        opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=lr), dynamic_loss_scale=True,
                                       dynamic_loss_args={"init_scale": 2.0 ** 12, "scale_window": 1000})
    else:
        opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=lr))
    ropt = torch.optim.SGD(ref.parameters(), lr=lr)
    from smdistributed_modelparallel_amd.ops.attention import FLASH_CALLS

    flash0 = dict(FLASH_CALLS)

    @smp.step
    def train(model, ids, labels):
        loss, _ = model((ids, None, None, None, labels))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(7)
    prescaled = bool(extra.get("cfg", {}).get("prescaled_batch"))
    # prescaled_batch: every TP rank of a group sees the SAME batch (distinct per RDP rank)
    dp = smp.rdp_size() if prescaled else smp.dp_size()
    my_dp = smp.rdp_rank() if prescaled else smp.dp_rank()
    local_bs = 2 * mbs
    seq = int(extra.get("seq", 16))
    grad_tol = extra.get("grad_tol")
    for it in range(steps):
        ids_all = torch.randint(0, kw["vocab_size"], (local_bs * dp, seq), generator=g).to(dev)
        ids = ids_all[my_dp * local_bs:(my_dp + 1) * local_bs]
        opt.zero_grad()
        out = train(model, ids, ids)
        snap = None
        if it == 0 and (grad_tol or fp32_tol):
            # reduced gradients of the first step, before the update (fp16: loss-scaled)
            inv = 1.0 / float(getattr(opt, "loss_scale", 1.0) or 1.0)
            snap = {n: p.grad.detach().float() * inv for n, p in model.local_named_parameters()
                    if p.grad is not None and p.numel() > 0}
        if extra.get("opt_clip"):
            opt.clip_master_grads(extra["opt_clip"])
        opt.step()
        # reference on the global batch, averaged the same way (per microbatch mean, then mean)
        ropt.zero_grad()
        losses = []
        for d in range(dp):
            chunk = ids_all[d * local_bs:(d + 1) * local_bs]
            for m in range(mbs):
                x = chunk[m * 2:(m + 1) * 2]
                if prescaled and not kw.get("distribute_embedding"):
                    # objective = mean over TP ranks of each rank's sequence-shard loss
                    # (a vocab-parallel head computes the whole batch's loss on every TP rank)
                    _, logits = ref((x, None, None, None, x))
                    lab = torch.nn.functional.pad(x[:, 1:], (0, 1), value=-100)
                    half = x.shape[1] // 2
                    sl = [torch.nn.functional.cross_entropy(logits[:, a:b].reshape(-1, logits.shape[-1]),
                                                            lab[:, a:b].reshape(-1), ignore_index=-100)
                          for a, b in ((0, half), (half, x.shape[1]))]
                    losses.append(torch.stack(sl).mean())
                    continue
                l, _ = ref((x, None, None, None, x))
                losses.append(l)
        ref_loss = torch.stack(losses).mean()
        ref_loss.backward()
        if snap is not None:
            _check_grads(model, snap, ref, sd0, ids_all, kw, base, grad_tol, fp32_tol)
        if extra.get("ref_clip") or extra.get("opt_clip"):
            torch.nn.utils.clip_grad_norm_(ref.parameters(), extra.get("ref_clip") or extra["opt_clip"])
        ropt.step()
        if extra.get("expect_overlap"):
            # DP buckets must have been launched while the pipeline was still running its
            # backward passes (GradTracker finality), not all at the step-end synchronize
            early = sum(r.launched_before_sync for r in model.reducers.values())
            total = sum(len(r.flat.buckets) for r in model.reducers.values())
            assert total > 1 and early >= 1, (smp.rank(), early, total)
            print(f"rank {smp.rank()} overlap: {early}/{total} buckets launched during backward", flush=True)
        my_losses = torch.stack([o.detach().float() for o in out.outputs]).mean()
        mine = torch.tensor([my_losses.item()])
        all_l = smp.allgather(mine.item(), smp.DP_GROUP)
        # prescaled: each TP rank reports its sequence shard's loss; averaging all DP-group
        # entries equally gives the mean over shards and RDP replicas (the objective above)
        if smp.pp_rank() == 0 or True:
            avg = sum(all_l) / len(all_l)
            assert abs(avg - ref_loss.item()) < float(extra.get("loss_tol", 1e-4)), (it, avg, ref_loss.item())
    # parameter check (local, TP-sliced)
    from smdistributed_modelparallel_amd.torch.checkpoint_utils import slice_for_param

    rp = dict(ref.named_parameters())
    worst, worst_name = 0.0, None
    if smp.state.cfg.zero2d_enabled():
        # parameters are sharded: compare the gathered full state dict
        sd = model.state_dict(gather_to_rank0=False)
        for n, full in rp.items():
            worst = max(worst, (sd[n].float().cpu() - full.detach().float().cpu()).abs().max().item())
    for n, p in model.local_named_parameters():
        if p.numel() == 0:
            continue
        full = rp[n].detach().to(p.device)
        t = slice_for_param(full, p, smp.tp_rank(), smp.tp_size())
        d = (p.detach().float() - t.float()).abs().max().item()
        if d > worst:
            worst, worst_name = d, n
    ptol = float(extra.get("param_tol", 2e-4))
    assert worst < ptol, (worst, worst_name if worst > 0 else None)
    if extra.get("expect_hier") is not None:
        sdp = smp.state.sdp
        assert sdp.hier == extra["expect_hier"], (sdp.hier, extra["expect_hier"])
        print(f"rank {smp.rank()} sharded-DP slot {sdp.slot} hierarchical {sdp.hier}", flush=True)
    if extra.get("expect_replay"):
        eng = smp.state.engine
        assert eng._replay, "schedule was never frozen"
        print(f"rank {smp.rank()} replaying {sum(len(v) for v in eng._replay.values())} recorded events", flush=True)
    if extra.get("cfg", {}).get("offload_activations") and smp.state.current_offloader is not None:
        st = smp.state.current_offloader.stats
        # every rank that runs checkpointed layers must have offloaded and reloaded them
        assert st["offloaded_bytes"] > 0 and st["loaded_bytes"] == st["offloaded_bytes"], st
        if extra.get("expect_task_prefetch"):
            assert st["task_prefetches"] > 0, st
    if extra.get("display_partition") and smp.rank() == 0:
        lines = model.display_partition()
        assert lines[0] == "Partition assignments:" and any("seq_layers" in x for x in lines), lines
        # a subtree held by one partition is not expanded: no layer internals are listed
        assert not any(".attention" in x or "/attention" in x for x in lines), lines
        print("\n".join("DISPLAY " + x for x in lines[1:]), flush=True)
    if extra.get("check_tp_overlap"):
        from smdistributed_modelparallel_amd.ops import linear as lin

        tr = lin.TP_OVERLAP_TRACE
        # last start of each run of consecutive starts (token-chunked dX: one start per chunk)
        starts = [i for i, e in enumerate(tr) if e == "dx_allreduce_start" and (i + 1 == len(tr) or
                                                                               tr[i + 1] != "dx_allreduce_start")]
        assert starts, tr[:20]
        for i in starts:
            # the weight gradient runs while the dX all-reduce(s) are in flight, then the wait
            assert tr[i + 1:i + 3] == ["wgrad", "dx_allreduce_wait"], (i, tr[i:i + 3])
        chunks = int(extra.get("expect_tp_chunks", 0))
        if chunks:
            runs = [i for i, e in enumerate(tr) if e == "dx_allreduce_start" and (i == 0 or tr[i - 1] != e)]
            longest = 0
            for i in runs:
                j = i
                while j < len(tr) and tr[j] == "dx_allreduce_start":
                    j += 1
                longest = max(longest, j - i)
            assert longest >= chunks and tr.count("fwd_chunk") >= chunks, (longest, tr.count("fwd_chunk"))
        print(f"rank {smp.rank()} tp overlap: {len(starts)} dX all-reduces overlapped with wgrad", flush=True)
    if extra.get("expect_flash"):
        ran = FLASH_CALLS["plain"] + FLASH_CALLS["key_bias"] - flash0["plain"] - flash0["key_bias"]
        assert ran > 0, ("the flash kernels did not run", FLASH_CALLS)
        print(f"rank {smp.rank()} flash launches {ran}", flush=True)
    print(f"rank {smp.rank()} OK loss={ref_loss.item():.5f} worst_param_diff={worst:.2e}", flush=True)
    smp.barrier()


def _check_grads(model, snap, ref, sd0, ids_all, kw, base, grad_tol, fp32_tol):
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS
    from smdistributed_modelparallel_amd.torch.checkpoint_utils import slice_for_param

    params = dict(model.local_named_parameters())
    refs = []
    if grad_tol:
        refs.append(("same-dtype model", {n: p.grad for n, p in ref.named_parameters()}, float(grad_tol)))
    if fp32_tol:
        from tests.torch_ref import gpt_loss

        leaves = {k: v.clone().requires_grad_(True) for k, v in sd0.items()}
        gpt_loss(leaves, ids_all, ids_all, dict(GPT_CONFIGS[base], **kw)).backward()
        refs.append(("plain-torch fp32", {n: t.grad for n, t in leaves.items()}, float(fp32_tol)))
    for label, grads, tol in refs:
        # 1-D parameters (biases, LayerNorm affine) and embedding tables are sums over the tokens
        # of the batch with heavy cancellation (an untied LM-head bias: sum_t (p - onehot)), so
        # their relative error at reduced precision is larger than the weights': bound them 4x
        # looser
        worst = {2: (0.0, None), 1: (0.0, None)}
        for n, g in snap.items():
            r = grads.get(n)
            assert r is not None, (label, n, "no reference gradient")
            r = slice_for_param(r.detach().float(), params[n], smp.tp_rank(), smp.tp_size())
            err = float((g - r).norm() / (r.norm() + 1e-12))
            k = 1 if (g.dim() == 1 or "embedding" in n) else 2
            worst[k] = max(worst[k], (err, n))
        for k, lim in ((2, tol), (1, 4 * tol)):
            assert worst[k][0] < lim, f"rank {smp.rank()}: grad rel err vs {label} {worst[k][0]:.4f} > {lim} ({worst[k][1]})"
        print(f"rank {smp.rank()} grads vs {label}: worst rel err {worst[2][0]:.4f} ({worst[2][1]}) weights, "
              f"{worst[1][0]:.4f} ({worst[1][1]}) 1-D / embeddings, over {len(snap)} params", flush=True)


if __name__ == "__main__":
    main()
