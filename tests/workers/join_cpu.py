"""Worker: DistributedModel.join() with uneven inputs (pure DP over gloo) and
DistributedModel.cpu() gathering a PP2 model onto every rank.

argv: mode = join | join_active | cpu
"""
import copy
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp


def _net():
    torch.manual_seed(5)
    return nn.Sequential(nn.Linear(8, 16), nn.Tanh(), nn.Linear(16, 4))


def join(divide_initial):
    smp.init({"ddp": True, "microbatches": 1})
    rank, world = smp.dp_rank(), smp.dp_size()
    net = _net()
    ref = copy.deepcopy(net)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(9)
    nsteps = [3 + 2 * r for r in range(world)]  # rank r has 3 + 2r batches
    data = [[torch.randn(4, 8, generator=g) for _ in range(max(nsteps))] for _ in range(world)]

    @smp.step
    def train(model, x):
        loss = model(x).pow(2).mean()
        model.backward(loss)
        return loss

    with model.join(divide_by_initial_world_size=divide_initial):
        for i in range(nsteps[rank]):
            opt.zero_grad()
            train(model, data[rank][i])
            opt.step()
    # reference: step i averages the ranks that still have data (over the initial world
    # size or over the active ranks)
    for i in range(max(nsteps)):
        active = [r for r in range(world) if i < nsteps[r]]
        ropt.zero_grad()
        loss = sum(ref(data[r][i]).pow(2).mean() for r in active) / (world if divide_initial else len(active))
        loss.backward()
        ropt.step()
    for (n, p), (_, q) in zip(model.module.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.detach(), q.detach(), atol=1e-6), (n, (p - q).abs().max())
    print(f"rank {smp.rank()} OK join divide_initial={divide_initial}", flush=True)


def cpu():
    smp.init({"pipeline_parallel_degree": 2, "microbatches": 2, "ddp": True, "auto_partition": False,
              "default_partition": 0})
    net = _net()
    ref = copy.deepcopy(net)
    smp.set_partition(net[2], 1)
    model = smp.DistributedModel(net)

    @smp.step
    def fwd(model, x):
        return model(x)

    x = torch.randn(4, 8)
    out = fwd(model, x)
    model.cpu()
    for (n, p), (_, q) in zip(model.module.named_parameters(), ref.named_parameters()):
        assert p.device.type == "cpu" and p.shape == q.shape and torch.equal(p.detach(), q), n
    if smp.pp_rank() == 0:
        assert torch.allclose(torch.cat(out.outputs), ref(x), atol=1e-6)
    print(f"rank {smp.rank()} OK cpu", flush=True)


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "cpu":
        cpu()
    else:
        join(mode == "join")
    smp.barrier()
