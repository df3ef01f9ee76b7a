"""Worker (world 2, sharded data parallel degree 2, fp16 + dynamic loss scale): an inf
injected into ONE rank's gradient shard must make BOTH ranks skip the step and back off
the loss scale identically (the overflow flag is reduced over the world)."""
import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    smp.init({"sharded_data_parallel_degree": 2, "fp16": True, "ddp": True, "sdp_param_persistence_threshold": 100,
              "sdp_reduce_bucket_size": 20000, "sdp_gradient_clipping": 0.0})
    torch.manual_seed(3)
    net = build_gpt("gpt2-tiny", dropout=0.0, num_layers=2, hidden_size=64, num_attention_heads=4,
                    attention_head_size=16, intermediate_size=128, vocab_size=96, num_positions=32)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-2), dynamic_loss_scale=True,
                                   dynamic_loss_args={"init_scale": 2.0 ** 10})

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    ids = torch.randint(0, 96, (4, 16), generator=torch.Generator().manual_seed(1 + smp.rank()))
    opt.zero_grad()
    train(model, ids)
    before = [opt._param_range(d).detach().clone() for d in opt.domains]
    if smp.rank() == 1:
        g = opt._grad_range(opt.domains[0])
        g[0] = float("inf")
    scale0 = opt.loss_scale
    opt.step()
    after = [opt._param_range(d) for d in opt.domains]
    assert all(torch.equal(a, b) for a, b in zip(before, after)), "a rank applied an overflowing step"
    scales = smp.allgather(opt.loss_scale, smp.WORLD)
    assert scales[0] == scales[1] and scales[0] < scale0, (scales, scale0)
    print(f"rank {smp.rank()} OK scale {scale0} -> {opt.loss_scale}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
