"""Worker: GPT pipeline parallelism on GPU ranks sharing one device, against an
unpartitioned model trained in the same process.

argv: pp microbatches steps dtype(fp32|bf16) [extra_json]
The pipeline tensors travel through the native IpcP2P engine (hipIpc mapping + event
wait + D2D pull); control messages through the mailbox; object collectives over gloo.
Checks the loss of every step and every local parameter after training.
"""
import json
import os
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    pp, mbs, steps, dtype = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    extra = json.loads(sys.argv[5]) if len(sys.argv) > 5 else {}
    bf16 = dtype == "bf16"
    dev = torch.device("cuda", 0)
    kw = dict(num_layers=4, hidden_size=256, num_attention_heads=4, attention_head_size=64, intermediate_size=1024,
              vocab_size=512, num_positions=256)
    kw.update(extra.get("model", {}))
    torch.manual_seed(123)
    ref = build_gpt("gpt2-small", dropout=0.0, **kw).to(dev)
    if bf16:
        ref = ref.to(torch.bfloat16)
    cfg = {"pipeline_parallel_degree": pp, "microbatches": mbs, "pipeline": extra.get("pipeline", "interleaved"),
           "auto_partition": bool(extra.get("auto")), "bf16": bf16, "ddp": int(os.environ["WORLD_SIZE"]) > pp}
    if not extra.get("auto"):
        cfg["default_partition"] = 0
    smp.init(cfg)
    want_mode = extra.get("expect_mode", os.environ.get("SMP_P2P", "ipc"))
    assert smp.state.transport.mode == want_mode, (smp.state.transport.mode, want_mode)
    if extra.get("max_mappings"):  # bounded IPC import table: evictions under churn
        smp.state.transport._ipc.set_max_imports(int(extra["max_mappings"]))
    net = build_gpt("gpt2-small", dropout=0.0, **kw)
    net.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    if not extra.get("auto") and pp > 1:
        layers = list(net.transformer.seq_layers)
        for i, layer in enumerate(layers):
            smp.set_partition(layer, (i * pp) // len(layers))
    model = smp.DistributedModel(net)
    lr = 0.05
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=lr))
    ropt = torch.optim.SGD(ref.parameters(), lr=lr)

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(7)
    seq = extra.get("seq", 128)
    local_bs = extra.get("mb_size", 2) * mbs
    tol = 2e-2 if bf16 else 2e-4
    for it in range(steps):
        ids = torch.randint(0, kw["vocab_size"], (local_bs, seq), generator=g).to(dev)
        opt.zero_grad()
        out = train(model, ids)
        opt.step()
        ropt.zero_grad()
        losses = []
        for m in range(mbs):
            x = ids[m * (local_bs // mbs):(m + 1) * (local_bs // mbs)]
            l, _ = ref((x, None, None, None, x))
            losses.append(l.float())
        ref_loss = torch.stack(losses).mean()
        ref_loss.backward()
        ropt.step()
        mine = float(torch.stack([o.detach().float() for o in out.outputs]).mean())
        assert abs(mine - ref_loss.item()) < tol * max(1.0, abs(ref_loss.item())), (it, mine, ref_loss.item())
    rp = dict(ref.named_parameters())
    worst, worst_name = 0.0, None
    for n, p in model.local_named_parameters():
        if p.numel() == 0:
            continue
        d = (p.detach().float() - rp[n].detach().float()).abs().max().item()
        if d > worst:
            worst, worst_name = d, n
    ptol = 5e-2 if bf16 else 1e-4
    assert worst < ptol, (worst, worst_name)
    st = smp.state.transport.stats()
    if pp > 1 and st["mode"] == "ipc":
        assert st["imports"] > 0 and st["exports"] > 0, st
        # every exported activation / gradient was released by its receiver at step end
        assert st["held"] == 0 and st["event_slots_busy"] == 0 and st["release_wait_timeouts"] == 0, st
        assert st["comm_stream"] == (os.environ.get("SMP_P2P_COMM_STREAM", "1") != "0"), st
    if extra.get("max_mappings"):
        ist = smp.state.transport._ipc.stats()
        assert ist["mappings_open"] <= int(extra["max_mappings"]), ist
        assert ist["mappings_evicted"] > 0, ist  # the churn really went through the eviction path
    print(f"rank {smp.rank()} OK pp={pp} loss={ref_loss.item():.5f} worst_param_diff={worst:.2e} p2p={st}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
