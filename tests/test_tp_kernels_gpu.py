"""Tensor-parallel native kernels vs fp32 PyTorch references:
* the strided pack / unpack copy (K21) used by the uneven all-gather / reduce-scatter /
  all-to-all packing;
* the distributed-LayerNorm trio (K6 apply-with-global-stats, K7 backward local sums,
  K8 backward finish with the TP-summed sums) -- the TP all-reduces are emulated by summing
  the per-shard statistics of a hidden dim split into uneven shards."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.int64])
def test_strided_copy_views(dt):
    from smdistributed_modelparallel_amd.ops.pack import strided_copy_

    torch.manual_seed(0)
    src = (torch.randn(6, 5, 7, 16, device="cuda") * 10).to(dt)
    cases = [
        (lambda t: t.permute(2, 0, 1, 3), (7, 6, 5, 16)),  # movedim-like, vectorisable inner run
        (lambda t: t.permute(3, 2, 1, 0), (16, 7, 5, 6)),  # fully transposed
        (lambda t: t[:, 1:4, ::2], (6, 3, 4, 16)),  # narrow + step
        (lambda t: t.reshape(30, 112)[:, 5:77], (30, 72)),  # unaligned inner run
    ]
    for view, shape in cases:
        s = view(src)
        assert tuple(s.shape) == shape
        d = torch.empty(shape, device="cuda", dtype=dt)
        strided_copy_(d, s)
        assert torch.equal(d, s.contiguous())
        # copy into a strided destination (the unpack direction)
        big = torch.zeros((shape[0] + 2,) + tuple(shape[1:]), device="cuda", dtype=dt)
        dst = big[1:1 + shape[0]]
        strided_copy_(dst.transpose(0, -1), s.transpose(0, -1))
        assert torch.equal(dst, s) and torch.equal(big[0], torch.zeros_like(big[0]))


def test_pack_rank_blocks_uneven():
    """The all-gather packing: shard [A, n_r, B] -> block [n_r, A, B] and back."""
    from smdistributed_modelparallel_amd.ops.pack import strided_copy_

    A, B, sizes = 6, 40, [7, 6, 6]
    shards = [torch.randn(A, n, B, device="cuda", dtype=torch.bfloat16) for n in sizes]
    mx = max(sizes)
    recv = torch.empty(len(sizes), mx, A, B, device="cuda", dtype=torch.bfloat16)
    for r, x in enumerate(shards):
        strided_copy_(recv[r, : sizes[r]], x.permute(1, 0, 2))
    out = torch.empty(A, sum(sizes), B, device="cuda", dtype=torch.bfloat16)
    off = 0
    for r, n in enumerate(sizes):
        strided_copy_(out[:, off:off + n].permute(1, 0, 2), recv[r, :n])
        off += n
    assert torch.equal(out, torch.cat(shards, dim=1))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_distributed_layernorm_kernels_emulated_tp(dt):
    from smdistributed_modelparallel_amd.ops._ext import ext

    C = ext()
    torch.manual_seed(1)
    rows, H, eps = 300, 1600, 1e-5
    splits = [534, 533, 533]  # uneven TP=3 shards of the hidden dim
    x = (torch.randn(rows, H, device="cuda") * 3 + 1.5).to(dt)
    w = torch.randn(H, device="cuda").to(dt)
    b = torch.randn(H, device="cuda").to(dt)
    dy = torch.randn(rows, H, device="cuda").to(dt)
    xs, ws_, bs, dys = (list(t.split(splits, dim=-1)) for t in (x, w, b, dy))
    xs, dys = [t.contiguous() for t in xs], [t.contiguous() for t in dys]
    # forward: local stats -> "all-reduce" -> global mean / var -> apply on every shard
    st = sum(C.layernorm_local_stats(t) for t in xs)
    mean = st[:, 0] / H
    var = ((st[:, 1] + st[:, 2]) / H - mean * mean).clamp_min(0)
    ys, rstd = [], torch.empty_like(mean)
    for t, wi, bi in zip(xs, ws_, bs):
        ys.append(C.layernorm_apply_stats(t, wi.contiguous(), bi.contiguous(), mean, var, rstd, eps))
    y = torch.cat(ys, dim=-1)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, eps)
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    assert (y.float() - yr).abs().max().item() / yr.abs().max().item() < tol
    # backward: local sums -> "all-reduce" -> finish on every shard
    sums = sum(C.layernorm_bwd_local_sums(d, t, wi.contiguous(), mean, rstd) for d, t, wi in zip(dys, xs, ws_))
    dxs, dws, dbs = [], [], []
    for d, t, wi in zip(dys, xs, ws_):
        dx, dw, db = C.layernorm_bwd(d, t, wi.contiguous(), mean, rstd, True, True, None, ext_sums=sums, ext_n=float(H))
        dxs.append(dx), dws.append(dw), dbs.append(db)
    yr.backward(dy.float())
    for name, got, ref in (("dx", torch.cat(dxs, -1), xr.grad), ("dw", torch.cat(dws), wr.grad),
                           ("db", torch.cat(dbs), br.grad)):
        err = (got.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert err < (3e-2 if dt == torch.bfloat16 else 1e-4), (name, err)


def test_distributed_layernorm_module_single_rank_matches_layernorm():
    """DistributedLayerNorm's GPU autograd path (K6-K8 with the external-sum finish) on an
    unsharded row equals a plain LayerNorm, fwd and bwd."""
    from smdistributed_modelparallel_amd.nn.layer_norm import _DistLayerNormHIP

    torch.manual_seed(2)
    x = torch.randn(4, 64, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = _DistLayerNormHIP.apply(x, w, b, 1e-5, 1024, None)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (1024,), wr, br, 1e-5)
    assert (y.float() - yr).abs().max().item() < 6e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (a.float() - r).abs().max().item() / (r.abs().max().item() + 1e-6) < 3e-2
