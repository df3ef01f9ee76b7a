"""Worker: one-shot IPC all-reduce on ranks sharing one GPU (SMP_ONESHOT_ALLREDUCE=1).

argv: kernel            -- sizes x dtypes x ops x repeated epochs against a gloo fp32 reference,
                           results bitwise identical on every rank, aligned and odd-offset views
      tp <steps>        -- GPT with tensor_parallel_degree = world through smp; prints the losses
"""
import os
import sys

import torch
import torch.distributed as dist


def kernel():
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from smdistributed_modelparallel_amd.parallel import oneshot

    r, ws = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    checked = 0
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        for n in (1, 7, 8, 1000, 4099, 65536, 262147, oneshot._MAX_BYTES // (4 if dt == torch.float32 else 2)):
            for op in (dist.ReduceOp.SUM, dist.ReduceOp.MAX):
                for it in range(3):
                    g = torch.Generator().manual_seed(1000 * r + 17 * it + n)
                    host = torch.randn(n + 1, generator=g).to(dt)
                    buf = host.to(dev)
                    x = buf[1:] if it == 1 else buf[:n].clone()  # it 1: a view at an odd offset
                    ref = host[1:].float().clone() if it == 1 else host[:n].float().clone()
                    dist.all_reduce(ref, op=op)
                    oneshot.all_reduce(x, op=op)
                    got = x.float().cpu()
                    tol = 1e-5 if dt == torch.float32 else (2e-2 if dt == torch.bfloat16 else 4e-3)
                    assert torch.allclose(got, ref.to(dt).float(), rtol=tol, atol=tol * ws), (dt, n, op, it)
                    # every rank holds the same bits
                    allv = [torch.empty_like(got) for _ in range(ws)]
                    dist.all_gather(allv, got)
                    assert all(torch.equal(a, allv[0]) for a in allv), (dt, n, op, it, "ranks differ")
                    checked += int(n * host.element_size() <= oneshot._MAX_BYTES)
    inst = oneshot._instances.get("world")
    assert inst is not None, "one-shot path was not enabled"
    st = inst.stats()
    assert st["calls"] >= checked, st
    oneshot.check_errors()
    print(f"rank {r} OK checked={checked} stats={st}", flush=True)
    dist.barrier()


def skip():
    """Rank 1 skips one one-shot call: rank 0's kernel must time out and poison its output,
    the abort must reach rank 1, and check_errors() must raise on BOTH ranks."""
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from smdistributed_modelparallel_amd.parallel import oneshot

    r = dist.get_rank()
    dev = torch.device("cuda", 0)
    x = torch.ones(4096, device=dev)
    oneshot.all_reduce(x)  # set-up + one good call on both ranks
    torch.cuda.synchronize()
    assert torch.all(x == dist.get_world_size()), x[:4]
    oneshot.check_errors()
    if r == 0:
        y = torch.ones(4096, device=dev)
        oneshot.all_reduce(y)  # rank 1 never joins this one: times out
        torch.cuda.synchronize()
        assert torch.isnan(y).all(), "timed-out call must not return stale sums"
    dist.barrier()
    z = torch.ones(4096, device=dev)
    oneshot.all_reduce(z)
    torch.cuda.synchronize()
    assert torch.isnan(z).all(), f"rank {r}: call after a peer's abort must fail"
    try:
        oneshot.check_errors()
    except oneshot.OneShotAllReduceError as e:
        raised = str(e)
    else:
        raise AssertionError(f"rank {r}: check_errors did not raise")
    try:
        oneshot.all_reduce(torch.ones(8, device=dev))
    except oneshot.OneShotAllReduceError:
        pass
    else:
        raise AssertionError("a failed instance must refuse later calls")
    print(f"rank {r} OK raised: {raised[:60]}", flush=True)
    dist.barrier()


def agree():
    """Rank 0's instance fails (injected) while rank 1's kernels all succeeded: the end-of-step
    check must raise on BOTH ranks in the same call (rank 1 used to pass and apply
    its update, raising only a step later)."""
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from smdistributed_modelparallel_amd.parallel import oneshot

    r = dist.get_rank()
    x = torch.ones(4096, device="cuda")
    oneshot.all_reduce(x)
    oneshot.check_errors(dist.group.WORLD)  # healthy: no raise on either rank
    if r == 0:
        oneshot.inject_failure()
    try:
        oneshot.check_errors(dist.group.WORLD)
    except oneshot.OneShotAllReduceError as e:
        print(f"rank {r} OK raised in the same step: {str(e)[:40]}", flush=True)
    else:
        raise AssertionError(f"rank {r}: check_errors did not raise")
    dist.barrier()


def tp(steps):
    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.models import build_gpt
    from smdistributed_modelparallel_amd.parallel import oneshot

    ws = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    smp.init({"tensor_parallel_degree": ws, "ddp": True, "bf16": False, "microbatches": 1})
    torch.manual_seed(5)
    kw = dict(num_layers=2, hidden_size=256, num_attention_heads=4, attention_head_size=64, intermediate_size=1024,
              vocab_size=512, num_positions=128)
    with smp.model_creation(tensor_parallelism=True, dtype=torch.float32):
        net = build_gpt("gpt2-small", dropout=0.0, **kw)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05))

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(11 + smp.rank())
    losses = []
    for _ in range(steps):
        ids = torch.randint(0, kw["vocab_size"], (2, 64), generator=g).to(dev)
        opt.zero_grad()
        out = train(model, ids)
        opt.step()
        losses.append(float(out.reduce_mean()))
    calls = sum(i.stats()["calls"] for i in oneshot._instances.values() if i is not None)
    print(f"rank {smp.rank()} OK losses={','.join(f'{v:.6f}' for v in losses)} oneshot_calls={calls}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    if sys.argv[1] == "kernel":
        kernel()
    elif sys.argv[1] == "skip":
        skip()
    elif sys.argv[1] == "agree":
        agree()
    else:
        tp(int(sys.argv[2]))
