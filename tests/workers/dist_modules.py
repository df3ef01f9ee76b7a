"""Worker (TP=2, gloo): smp.nn distributed modules vs plain torch references (reference
`smp/test/torch/mpi_4ps/test_dist_modules.py`) and the tensor collectives of the comm API
(`mpi_4ps/test_collectives.py`: allgatherv, scatter_and_merge incl. uneven shapes)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import (DistributedCrossEntropy, DistributedEmbedding, DistributedLayerNorm,
                                                DistributedLinear)
from smdistributed_modelparallel_amd.torch.checkpoint_utils import slice_for_param


def close(a, b, tol=1e-5, what=""):
    err = (a - b).abs().max().item()
    assert err < tol, (what, err)


def scaled_batch_check(dist_mod, ref_mod, make_input, tp, r):
    """Each rank feeds its own batch; compare outputs, input grads and sliced weight grads."""
    torch.manual_seed(100)
    xs = [make_input() for _ in range(tp)]
    gs = None
    # reference on the concatenated TP-group batch
    ref_in = [x.clone().requires_grad_(x.is_floating_point()) for x in xs]
    ref_out = [ref_mod(x) for x in ref_in]
    torch.manual_seed(200)
    gs = [torch.randn_like(o) for o in ref_out]
    sum((o * g).sum() for o, g in zip(ref_out, gs)).backward()
    x = xs[r].clone().requires_grad_(xs[r].is_floating_point())
    out = dist_mod(x)
    close(out, ref_out[r], what="out")
    (out * gs[r]).sum().backward()
    if x.is_floating_point():
        close(x.grad, ref_in[r].grad, what="dx")
    rp = dict(ref_mod.named_parameters())
    for n, p in dist_mod.named_parameters():
        want = slice_for_param(rp[n].grad, p, r, tp)
        close(p.grad, want, 1e-4, what="grad " + n)


def main():
    smp.init({"tensor_parallel_degree": 2, "ddp": True})
    tp, r = smp.tp_size(), smp.tp_rank()
    torch.manual_seed(0)
    # ---- DistributedLinear (input-partitioned, bias on rank 0, uneven in_features)
    ref = nn.Linear(9, 6)
    dl = DistributedLinear(9, 6)
    with torch.no_grad():
        dl.weight.copy_(slice_for_param(ref.weight, dl.weight, r, tp))
        if dl.bias is not None:
            dl.bias.copy_(ref.bias)
    scaled_batch_check(dl, ref, lambda: torch.randn(3, 5, 9), tp, r)
    # ---- DistributedEmbedding: embedding-dim parallel and vocab parallel (uneven)
    for vp in (False, True):
        ref = nn.Embedding(11, 7)
        de = DistributedEmbedding(11, 7, vocab_parallel=vp)
        with torch.no_grad():
            de.weight.copy_(slice_for_param(ref.weight, de.weight, r, tp))
        scaled_batch_check(de, ref, lambda: torch.randint(0, 11, (2, 5)), tp, r)
    # ---- DistributedLayerNorm: the SAME batch, hidden dim sharded (uneven 13 = 7 + 6)
    torch.manual_seed(1)
    full = torch.randn(4, 13)
    ln = nn.LayerNorm(13)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    dln = DistributedLayerNorm(13)
    start, n = dln.start, dln.local_dim
    with torch.no_grad():
        dln.weight.copy_(ln.weight[start:start + n])
        dln.bias.copy_(ln.bias[start:start + n])
    xr = full.clone().requires_grad_()
    yr = ln(xr)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    x = full[:, start:start + n].clone().requires_grad_()
    y = dln(x)
    close(y, yr[:, start:start + n], what="dln out")
    (y * g[:, start:start + n]).sum().backward()
    close(x.grad, xr.grad[:, start:start + n], 1e-5, "dln dx")
    close(dln.weight.grad, ln.weight.grad[start:start + n], 1e-5, "dln dw")
    # ---- DistributedCrossEntropy: vocab-sharded logits of the same batch
    torch.manual_seed(2)
    logits = torch.randn(6, 11)
    target = torch.randint(0, 11, (6,))
    target[1] = -100
    ref_loss = F.cross_entropy(logits, target, reduction="none")
    V = [6, 5]
    lo = sum(V[:r])
    ce = DistributedCrossEntropy(vocab_range=(lo, lo + V[r]))
    shard = logits[:, lo:lo + V[r]].contiguous().requires_grad_(True)
    mine = ce(shard, target)
    close(mine, ref_loss, 1e-5, "dist CE")
    # backward: the shard of the full softmax gradient, multiplied by tp (every TP rank holds
    # the same loss; reference nn/cross_entropy.py:95-96)
    full = logits.clone().requires_grad_(True)
    F.cross_entropy(full, target, reduction="none").sum().backward()
    mine.sum().backward()
    close(shard.grad, full.grad[:, lo:lo + V[r]] * tp, 1e-5, "dist CE grad")
    # ---- tensor collectives
    counts = [3, 5]
    t = torch.arange(10, dtype=torch.float32) + 100 * r
    got = smp.allgatherv_tensor(t, counts, smp.TP_GROUP)
    want = torch.cat([torch.arange(counts[q], dtype=torch.float32) + 100 * q for q in range(tp)])
    assert torch.equal(got, want), got
    # scatter_and_merge: [4, 6] split on axis 0 (batch), merge on axis 1 with uneven widths
    widths = [2, 3]
    x = torch.full((4, widths[r]), float(r)) + torch.arange(4).view(4, 1) * 10
    y = smp.scatter_and_merge_tensor(x, 0, 1, smp.TP_GROUP, merge_shapes=widths)
    assert y.shape == (2, 5), y.shape
    expect = torch.cat([torch.full((2, widths[q]), float(q)) + torch.arange(2 * r, 2 * r + 2).view(2, 1) * 10
                        for q in range(tp)], dim=1)
    assert torch.equal(y, expect), (y, expect)
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
