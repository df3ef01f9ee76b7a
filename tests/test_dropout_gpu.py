"""Mask-free fused dropout kernels (ops/dropout.py, csrc/kernels/dropout.hip, the dropout
option of the LayerNorm kernel) vs fp32 PyTorch references that apply the keep factors
rebuilt on the host from the same (seed, offset)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _seed_off():
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    return gen.initial_seed() & ((1 << 63) - 1), gen.get_offset()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("with_res", [True, False])
def test_dropout_add_fwd_bwd(dt, with_res):
    from smdistributed_modelparallel_amd.ops.dropout import dropout_add, dropout_keep_reference

    torch.manual_seed(0)
    p = 0.1
    x = torch.randn(64, 1603, device="cuda", dtype=dt, requires_grad=True)  # odd size: tail path
    r = torch.randn(64, 1603, device="cuda", dtype=dt, requires_grad=True) if with_res else None
    seed, off = _seed_off()
    y = dropout_add(x, r, p, True)
    f = dropout_keep_reference(x.numel(), p, seed, off, device="cuda").view(x.shape)
    ref = x.detach().float() * f + (r.detach().float() if with_res else 0.0)
    tol = 1e-6 if dt == torch.float32 else 2e-2
    assert (y.float() - ref).abs().max().item() < tol * 4
    kept = (f > 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01, kept
    g = torch.randn_like(y)
    y.backward(g)
    assert torch.allclose(x.grad.float(), g.float() * f, atol=tol * 4, rtol=1e-2)
    if with_res:
        assert torch.equal(r.grad, g)


def test_add_layer_norm_with_dropout():
    from smdistributed_modelparallel_amd.ops.dropout import dropout_keep_reference
    from smdistributed_modelparallel_amd.ops.layernorm import add_layer_norm

    torch.manual_seed(1)
    p, h = 0.1, 1600
    x = torch.randn(512, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(512, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    seed, off = _seed_off()
    y, s = add_layer_norm(x, r, w, b, 1e-5, p)
    f = dropout_keep_reference(x.numel(), p, seed, off, device="cuda").view(x.shape)
    xr, rr, wr, br = (t.detach().float().requires_grad_() for t in (x, r, w, b))
    sr = xr * f + rr
    yr = torch.nn.functional.layer_norm(sr, (h,), wr, br, 1e-5)
    assert (s.float() - sr).abs().max().item() < 3e-2
    # the kernel normalises the bf16-rounded sum: compare against LN of the rounded reference
    y_of_rounded = torch.nn.functional.layer_norm(sr.detach().bfloat16().float(), (h,), wr.detach(), br.detach(), 1e-5)
    err = (y.float() - y_of_rounded).abs().max().item() / y_of_rounded.abs().max().item()
    assert err < 1e-2, err  # bf16 output rounding
    gy, gs = torch.randn_like(yr), torch.randn_like(sr)
    (y.float() * gy + s.float() * gs).sum().backward()
    (yr * gy + sr * gs).sum().backward()
    for name, a, ref in (("x", x.grad, xr.grad), ("r", r.grad, rr.grad), ("w", w.grad, wr.grad), ("b", b.grad, br.grad)):
        err = (a.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert err < 3e-2, (name, err)


def test_dropout_replays_under_activation_checkpointing():
    """Recompute inside torch.utils.checkpoint regenerates the same decisions (the device
    generator state, offset included, is restored)."""
    from torch.utils.checkpoint import checkpoint

    from smdistributed_modelparallel_amd.ops.dropout import dropout_add

    torch.manual_seed(2)
    x = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16)

    def f(a):
        return dropout_add(a * 2.0, r, 0.3, True)

    torch.manual_seed(5)
    y1 = f(x)
    g = torch.randn_like(y1)
    (gx1,) = torch.autograd.grad(y1, x, g)
    torch.manual_seed(5)
    y2 = checkpoint(f, x, use_reentrant=False)
    (gx2,) = torch.autograd.grad(y2, x, g)
    assert torch.equal(y1, y2) and torch.equal(gx1, gx2)


@pytest.mark.parametrize("h", [1024, 1600, 4096])
def test_ln_bwd_fused_dropout_output_bitwise(h):
    """The LN backward's fused dropout output (dx * keep / (1 - p), written beside dx by the
    block kernels) is bitwise what the separate dropout_bwd pass over dx gives."""
    from smdistributed_modelparallel_amd.ops._ext import ext

    torch.manual_seed(2)
    rows = 777
    x = torch.randn(rows, h, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(h, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(h, device="cuda", dtype=torch.bfloat16)
    _, mean, rstd = ext().layernorm_fwd(x, None, w, b, 1e-5)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    out = ext().layernorm_bwd(dy, x, w, mean, rstd, True, True, dres, None, None, None, 0.0,
                              dropout_p=0.1, seed=1234, offset=8)
    assert len(out) == 4, "block kernels must serve this width"
    ref = ext().dropout_bwd(out[0], 0.1, 1234, 8)
    assert torch.equal(out[3], ref)
    plain = ext().layernorm_bwd(dy, x, w, mean, rstd, True, True, dres)
    assert torch.equal(out[0], plain[0]) and torch.equal(out[1], plain[1]) and torch.equal(out[2], plain[2])


def test_cross_layer_residual_fusion_is_bitwise_neutral():
    """A layer's MLP dropout + residual add deferred into the next layer's LayerNorm kernel gives
    bitwise the same loss and gradients as the separate kernels (tests/workers/cross_layer.py)."""
    from tests.dist_utils import run_workers

    outs = run_workers("cross_layer", 1, [], timeout=300, env_extra={"SMP_FORCE_CPU": "0"})
    assert "OK bitwise" in outs[0], outs[0][-2000:]
