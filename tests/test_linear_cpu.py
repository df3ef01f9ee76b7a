"""ops.linear autograd plumbing on CPU tensors (the GPU kernels are covered by
tests/test_wgrad_gpu.py): the layer's own bias gradient and ``dbias_of`` -- the gradient of a
bias a fused activation adds downstream, returned by the linear layer -- against plain autograd."""
import torch
import torch.nn.functional as F

from smdistributed_modelparallel_amd.ops.linear import linear


def _data(seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(3, 17, 24, generator=g)
    w = torch.randn(40, 24, generator=g)
    b = torch.randn(40, generator=g)
    up = torch.randn(3, 17, 40, generator=g)
    return x, w, b, up


def test_linear_own_bias_matches_autograd():
    x, w, b, up = _data()
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    (F.linear(xr, wr, br) * up).sum().backward()
    xa, wa, ba = (t.clone().requires_grad_(True) for t in (x, w, b))
    # the custom-function path (a no-op input-gradient all-reduce forces it)
    y = linear(xa, wa, ba, dx_allreduce=lambda dx: None)
    (y * up).sum().backward()
    for a, r in ((xa, xr), (wa, wr), (ba, br)):
        assert torch.allclose(a.grad, r.grad, atol=1e-5, rtol=1e-5)


def test_linear_dbias_of_returns_downstream_bias_gradient():
    """y = linear(x, W, dbias_of=b); z = gelu(y + b) with b's gradient left to the linear
    (the bias-GeLU's bias_grad=False contract): b.grad = sum over tokens of dz/d(y + b)."""
    x, w, b, up = _data(1)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    (F.gelu(F.linear(xr, wr) + br) * up).sum().backward()

    xa, wa, ba = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = linear(xa, wa, dbias_of=ba)
    z = F.gelu(y + ba.detach())  # the activation adds b but does not differentiate it
    (z * up).sum().backward()
    for a, r in ((xa, xr), (wa, wr), (ba, br)):
        assert torch.allclose(a.grad, r.grad, atol=1e-5, rtol=1e-5), (a.grad - r.grad).abs().max()


def test_linear_dbias_of_without_weight_grad():
    """A frozen weight: the downstream bias still gets its gradient through the linear."""
    x, w, b, up = _data(2)
    br = b.clone().requires_grad_(True)
    (F.gelu(F.linear(x, w) + br) * up).sum().backward()
    ba = b.clone().requires_grad_(True)
    y = linear(x, w, dbias_of=ba)
    (F.gelu(y + ba.detach()) * up).sum().backward()
    assert torch.allclose(ba.grad, br.grad, atol=1e-5, rtol=1e-5)
