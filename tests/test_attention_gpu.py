"""Flash attention HIP kernel vs a plain fp32 PyTorch reference."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, scale, causal, window=None):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))  # [b, h, s, d]
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    sq, sk = s.shape[-2:]
    i = torch.arange(sq, device=q.device).view(-1, 1) + (sk - sq)
    j = torch.arange(sk, device=q.device).view(1, -1)
    masked = torch.zeros(sq, sk, dtype=torch.bool, device=q.device)
    if causal:
        masked |= j > i
    if window:
        masked |= j <= i - window
    s = s.masked_fill(masked, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("s", [128, 200, 1024])
def test_flash_fwd_bwd(dt, d, causal, s):
    from smdistributed_modelparallel_amd.ops.attention import _FlashAttention

    torch.manual_seed(0)
    b, h = 2, 3
    q = torch.randn(b, s, h, d, device="cuda", dtype=dt, requires_grad=True)
    k = torch.randn(b, s, h, d, device="cuda", dtype=dt, requires_grad=True)
    v = torch.randn(b, s, h, d, device="cuda", dtype=dt, requires_grad=True)
    scale = 1.0 / math.sqrt(d)
    o = _FlashAttention.apply(q, k, v, scale, causal, 0)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _ref(qr, kr, vr, scale, causal)
    tol = 2e-2 if dt == torch.bfloat16 else 4e-3
    assert (o.float() - orf).abs().max().item() < tol
    g = torch.randn_like(orf)
    o.backward(g.to(dt))
    orf.backward(g)
    for name, a, ref in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        err = (a.float() - ref).abs().max().item()
        scale_ref = ref.abs().max().item() + 1e-6
        assert err / scale_ref < (3e-2 if dt == torch.bfloat16 else 8e-3), (name, err, scale_ref)


def test_flash_packed_qkv_and_window():
    from smdistributed_modelparallel_amd.ops.attention import _FlashAttention, _FlashAttentionPacked

    torch.manual_seed(1)
    qkv = torch.randn(2, 256, 3, 4, 64, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = _FlashAttentionPacked.apply(qkv, 0.125, True, 0)
    qkv2 = qkv.detach().clone().requires_grad_()
    o2 = _FlashAttention.apply(qkv2[:, :, 0], qkv2[:, :, 1], qkv2[:, :, 2], 0.125, True, 0)
    assert torch.equal(o, o2)
    g = torch.randn_like(o)
    o.backward(g)
    o2.backward(g)
    assert torch.equal(qkv.grad, qkv2.grad)
    # local (GPT-Neo) window
    q = torch.randn(1, 300, 2, 64, device="cuda", dtype=torch.bfloat16)
    ow = _FlashAttention.apply(q, q, q, 0.125, True, 37)
    ref = _ref(q.float(), q.float(), q.float(), 0.125, True, 37)
    assert (ow.float() - ref).abs().max().item() < 2e-2


def test_flash_long_sequence():
    """No sequence cap (the reference's fused softmax stops at 2048)."""
    from smdistributed_modelparallel_amd.ops.attention import _FlashAttention

    torch.manual_seed(2)
    q = torch.randn(1, 8192, 1, 64, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, 8192, 1, 64, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, 8192, 1, 64, device="cuda", dtype=torch.bfloat16)
    o = _FlashAttention.apply(q, k, v, 0.125, True, 0)
    ref = _ref(q, k, v, 0.125, True)
    assert (o.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("causal", [True, False])
def test_materialised_chunked_d256(monkeypatch, causal):
    """Head dim 256 (GPT-J) runs the materialised path (HIP scaled softmax kernels); forced
    batch chunking (2 of 4 rows per chunk) still matches the fp32 reference, fwd and bwd."""
    from smdistributed_modelparallel_amd.ops import attention as A

    torch.manual_seed(0)
    b, s, h, d = 4, 512, 4, 256
    monkeypatch.setattr(A, "_MAX_SCORE_ELEMS", 2 * h * s * s)
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    o = A.attention(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _ref(qr, kr, vr, 1.0 / 16, causal)
    assert (o.float() - orf).abs().max().item() < 2e-2
    g = torch.randn_like(orf)
    o.backward(g.to(torch.bfloat16))
    orf.backward(g)
    for name, a, ref in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        err = (a.float() - ref).abs().max().item()
        assert err / (ref.abs().max().item() + 1e-6) < 3e-2, (name, err)
