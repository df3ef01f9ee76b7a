"""Standalone fused optimizers on the multi-tensor HIP kernels (optim.hip mt_*: one launch per
tensor list, <= 64K-element chunks) against the same optimizers' fp32 CPU reference math:
fp32 parameters and bf16 parameters with fp32 masters, tensors spanning several chunks and
with sizes that are not multiples of the 4-element vector width."""
import pytest
import torch

from smdistributed_modelparallel_amd.optimizers import FusedAdam, FusedLAMB, FusedNovoGrad

pytestmark = pytest.mark.gpu

SHAPES = [(300, 700), (1000,), (3, 5, 7), (100003,)]


def _run(make, dtype, steps=3):
    g = torch.Generator().manual_seed(0)
    base = [torch.randn(s, generator=g) for s in SHAPES]
    grads = [[torch.randn(s, generator=g) for s in SHAPES] for _ in range(steps)]
    out = {}
    for dev in ("cpu", "cuda"):
        ps = [b.clone().to(dev, dtype).requires_grad_() for b in base]
        opt = make(ps)
        for gs in grads:
            for p, gr in zip(ps, gs):
                p.grad = gr.to(dev, dtype)
            opt.step()
        out[dev] = [(opt.state[p].get("master", p)).detach().float().cpu() for p in ps]
    for a, b in zip(out["cpu"], out["cuda"]):
        err = (a - b).abs().max().item()
        assert err < 2e-5 * max(1.0, a.abs().max().item()), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [True, False])
def test_fused_adam_multi_tensor(dtype, adamw):
    # weight decay 0.0123, not a round number: with 0.05 some bf16 (g, p) pairs have g / p = -4/5
    # * 2^-4 exactly, so the L2 gradient g + 0.05f p is 0 on the CPU (product rounded first) and
    # ~1e-9 on the GPU (fused multiply-add) -- below eps = 1e-8 the Adam step then differs by
    # ~0.1 lr on those few elements (tools/opt_debug.py: 5 of 310K), a rounding artefact
    _run(lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.0123, adam_w_mode=adamw), dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [True, False])
def test_fused_lamb_multi_tensor(dtype, adamw):
    # max_grad_norm below the gradient norm: the global-norm clip is active
    _run(lambda ps: FusedLAMB(ps, lr=1e-2, weight_decay=0.01, max_grad_norm=5.0, adam_w_mode=adamw), dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kw", [dict(), dict(norm_type=0), dict(reg_inside_moment=True), dict(init_zero=True)])
def test_fused_novograd_multi_tensor(dtype, kw):
    _run(lambda ps: FusedNovoGrad(ps, lr=1e-2, weight_decay=0.01, **kw), dtype)


def test_multi_tensor_adam_is_one_launch_per_list():
    """The whole list is one kernel launch (no per-parameter loop)."""
    from torch.profiler import ProfilerActivity, profile

    ps = [torch.randn(s, device="cuda", requires_grad=True) for s in SHAPES]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = FusedAdam(ps, lr=1e-3)
    opt.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        opt.step()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if "adam" in e.name.lower() and e.device_type.name == "CUDA"]
    assert len(names) == 1, names
