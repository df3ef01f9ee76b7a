"""Worker (dp=2): DDP features of DistributedModel -- no_sync gradient accumulation,
user comm hooks (torch-DDP style, returning a Future) and the builtin bf16 compression
hook, checked against a plain PyTorch model on the global batch."""
import sys

import torch
import torch.distributed as dist

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    mode = sys.argv[1]
    torch.manual_seed(0)
    kw = dict(num_layers=2, hidden_size=64, num_attention_heads=4, attention_head_size=16, intermediate_size=128,
              vocab_size=96, num_positions=32)
    ref = build_gpt("gpt2-tiny", dropout=0.0, **kw)
    smp.init({"ddp": True})
    net = build_gpt("gpt2-tiny", dropout=0.0, **kw)
    net.load_state_dict(ref.state_dict())
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    calls = []
    if mode == "hook":
        def allreduce_hook(state, bucket):
            calls.append(bucket.index())
            buf = bucket.buffer()
            return dist.all_reduce(buf, group=bucket.process_group(), async_op=True).get_future()

        model.register_comm_hook(None, allreduce_hook)
    elif mode == "bf16":
        model._register_builtin_comm_hook("BF16_COMPRESS")

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(1)
    r = smp.dp_rank()
    batches = [torch.randint(0, 96, (4, 16), generator=g) for _ in range(2)]
    opt.zero_grad()
    if mode == "nosync":
        with model.no_sync():
            train(model, batches[0][2 * r:2 * r + 2])
        train(model, batches[1][2 * r:2 * r + 2])
    else:
        train(model, batches[0][2 * r:2 * r + 2])
    opt.step()
    ropt.zero_grad()
    used = batches if mode == "nosync" else batches[:1]
    loss = 0
    for b in used:
        for q in range(2):
            l, _ = ref((b[2 * q:2 * q + 2], None, None, None, b[2 * q:2 * q + 2]))
            loss = loss + l / 2
    loss.backward()
    ropt.step()
    tol = 3e-3 if mode == "bf16" else 2e-5
    rp = dict(ref.named_parameters())
    worst = max((p.detach() - rp[n].detach()).abs().max().item() for n, p in model.local_named_parameters())
    assert worst < tol, (mode, worst)
    if mode == "hook":
        assert calls, "comm hook never called"
    print(f"rank {smp.rank()} OK {mode} {worst:.2e}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
