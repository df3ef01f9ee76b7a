"""Numerics of the CDNA4 HIP kernels against plain PyTorch fp32 references
(reference test strategy: `smp/test/torch/test_kernels.py:14-86`)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DT = [torch.bfloat16, torch.float16, torch.float32]


def _tol(dt):
    return {torch.float32: 2e-5, torch.float16: 2e-3, torch.bfloat16: 2e-2}[dt]


# relative-norm bound for reductions over rows (parameter gradients): ||out - ref|| / ||ref||.
# An absolute element tolerance scaled for the largest sums let a reduction that drops a tile
# pass; a dropped 1/37 of the rows moves the norm by ~3 %.
_REL = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 1e-2}


def _rel(out, ref):
    out, ref = out.double(), ref.double()
    return ((out - ref).norm() / ref.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def C():
    from smdistributed_modelparallel_amd.ops._ext import ext

    return ext()


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("cols", [64, 1600, 4096, 1000, 5000, 6144, 8192, 12288])
def test_layernorm_fwd_bwd(C, dt, cols):
    from smdistributed_modelparallel_amd.ops.layernorm import layer_norm

    torch.manual_seed(0)
    x = torch.randn(37, cols, device="cuda", dtype=dt, requires_grad=True)
    w = (1 + 0.1 * torch.randn(cols, device="cuda", dtype=dt)).requires_grad_()
    b = (0.1 * torch.randn(cols, device="cuda", dtype=dt)).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (cols,), wr, br, 1e-5)
    tol = _tol(dt) * 4
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 4, rtol=tol * 4)
    assert _rel(w.grad, wr.grad) < _REL[dt], _rel(w.grad, wr.grad)
    assert _rel(b.grad, br.grad) < _REL[dt], _rel(b.grad, br.grad)


@pytest.mark.parametrize("cols", [6144, 8192])
@pytest.mark.parametrize("with_dres", [False, True])
def test_layernorm_wide_bwd_many_rows(C, cols, with_dres):
    """Wide-row LayerNorm backward over many rows per block (the two-row register ring carries
    the next row's x / dy / residual gradient across iterations): dx, dgamma, dbeta against
    fp32 at 4099 rows (odd, so the last block is short)."""
    torch.manual_seed(2)
    rows = 4099
    x = torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(cols, device="cuda")).to(torch.bfloat16)
    b = (0.1 * torch.randn(cols, device="cuda")).to(torch.bfloat16)
    y, mean, rstd = C.layernorm_fwd(x, None, w, b, 1e-5)
    dy = torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16)
    dr = torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16) if with_dres else None
    dx, dw, db = C.layernorm_bwd(dy, x, w, mean, rstd, True, True, dr, None, None, None, 0.0)[:3]
    xr = x.float().requires_grad_()
    wr, br = w.float().requires_grad_(), b.float().requires_grad_()
    torch.nn.functional.layer_norm(xr, (cols,), wr, br, 1e-5).backward(dy.float())
    want = xr.grad + (dr.float() if with_dres else 0.0)
    assert _rel(dx, want) < 1e-2, _rel(dx, want)
    assert _rel(dw, wr.grad) < 1e-2, _rel(dw, wr.grad)
    assert _rel(db, br.grad) < 1e-2, _rel(db, br.grad)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cols", [1600, 6144])
def test_add_layernorm(C, dt, cols):
    """Residual add + LayerNorm in one kernel (register rows; 6144: the wide block-per-row
    kernels of GPT-NeoX / the 175B shape's TP-sliced widths)."""
    from smdistributed_modelparallel_amd.ops.layernorm import add_layer_norm

    torch.manual_seed(1)
    x = torch.randn(64, cols, device="cuda", dtype=dt, requires_grad=True)
    r = torch.randn(64, cols, device="cuda", dtype=dt, requires_grad=True)
    w = torch.ones(cols, device="cuda", dtype=dt, requires_grad=True)
    b = torch.zeros(cols, device="cuda", dtype=dt, requires_grad=True)
    y, s = add_layer_norm(x, r, w, b)
    xr, rr = x.detach().float().requires_grad_(), r.detach().float().requires_grad_()
    sr = xr + rr
    yr = torch.nn.functional.layer_norm(sr, (cols,), w.detach().float(), b.detach().float())
    tol = _tol(dt) * 4
    assert torch.allclose(s.float(), sr, atol=tol, rtol=tol)
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    gy, gs = torch.randn_like(yr), torch.randn_like(sr)
    torch.autograd.backward([y, s], [gy.to(dt), gs.to(dt)])
    torch.autograd.backward([yr, sr], [gy, gs])
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 4, rtol=tol * 4)
    assert torch.allclose(r.grad.float(), rr.grad, atol=tol * 4, rtol=tol * 4)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("rows,cols", [(33, 6400), (5000, 6400), (777, 1600), (1031, 4800), (300, 40), (129, 1001),
                                       (3001, 2056), (4097, 4800)])
@pytest.mark.parametrize("exact", [False, True])
def test_bias_gelu(C, dt, rows, cols, exact):
    from smdistributed_modelparallel_amd.ops.gelu import _gelu_tanh_ref, bias_gelu

    torch.manual_seed(2)
    x = torch.randn(rows, cols, device="cuda", dtype=dt, requires_grad=True)
    b = torch.randn(cols, device="cuda", dtype=dt, requires_grad=True)
    y = bias_gelu(x, b, exact=exact)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(xr + br) if exact else _gelu_tanh_ref(xr + br)
    tol = _tol(dt) * 2
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    assert _rel(b.grad, br.grad) < _REL[dt], _rel(b.grad, br.grad)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("rows,cols", [(32768, 1600), (4097, 4800), (100, 6400), (7, 40), (515, 1001), (64, 8)])
def test_col_sum_and_accumulate(C, dt, rows, cols):
    torch.manual_seed(5)
    x = torch.randn(rows, cols, device="cuda", dtype=dt)
    ref = x.double().sum(0)
    out = C.col_sum(x)
    tol = {torch.float32: 1e-4, torch.float16: 2e-3, torch.bfloat16: 1e-2}[dt]
    scale = max(1.0, rows ** 0.5)
    assert torch.allclose(out.double(), ref, atol=tol * scale, rtol=tol)
    # in-place accumulation into an existing gradient view (flat-buffer bias grads)
    base = torch.randn(cols, device="cuda", dtype=dt)
    acc = base.clone()
    r = C.col_sum(x, acc)
    assert r.data_ptr() == acc.data_ptr()
    assert torch.allclose(acc.double(), base.double() + ref, atol=tol * scale, rtol=tol)
    # fused gelu backward accumulating its dbias
    if cols % 8 == 0 and dt != torch.float32:
        from smdistributed_modelparallel_amd.ops.gelu import _gelu_tanh_ref

        b = torch.randn(cols, device="cuda", dtype=dt)
        dy = torch.randn_like(x)
        db = base.clone()
        dx, db2 = C.bias_gelu_bwd_dbias(dy, x, b, db)
        assert db2.data_ptr() == db.data_ptr()
        xr = (x.float() + b.float()).requires_grad_()
        _gelu_tanh_ref(xr).backward(dy.float())
        assert torch.allclose(dx.float(), xr.grad, atol=tol * 4, rtol=tol * 4)
        assert torch.allclose(db.double(), base.double() + xr.grad.double().sum(0), atol=tol * 4 * scale, rtol=tol * 4)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("sk", [128, 1024, 2048, 4096, 20000])
def test_causal_softmax(C, dt, sk):
    from smdistributed_modelparallel_amd.ops.softmax import _ref_softmax, scaled_causal_softmax

    torch.manual_seed(3)
    b, h = (2, 4) if sk <= 4096 else (1, 1)
    sq = sk if sk <= 4096 else 64
    x = torch.randn(b, h, sq, sk, device="cuda", dtype=dt, requires_grad=True)
    y = scaled_causal_softmax(x, 0.125)
    xr = x.detach().float().requires_grad_()
    yr = _ref_softmax(xr, None, 0.125, True)
    assert torch.allclose(y.float(), yr, atol=1e-3 if dt == torch.float16 else 4e-3)
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    assert torch.allclose(x.grad.float(), xr.grad, atol=2e-3 if dt == torch.float16 else 1e-2)


def test_masked_softmax(C):
    from smdistributed_modelparallel_amd.ops.softmax import _ref_softmax, scaled_masked_softmax

    torch.manual_seed(4)
    x = torch.randn(4, 16, 1024, 1024, device="cuda", dtype=torch.float16)
    mask = (torch.rand(4, 1, 1024, 1024, device="cuda") < 0.2).to(torch.uint8)
    y = scaled_masked_softmax(x, mask, 1.0)
    yr = _ref_softmax(x.float(), mask, 1.0, False)
    assert torch.allclose(y.float(), yr, atol=1e-3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("vocab", [50257, 1024, 12563])
def test_cross_entropy(C, dt, vocab):
    from smdistributed_modelparallel_amd.ops.cross_entropy import cross_entropy

    torch.manual_seed(5)
    logits = torch.randn(61, vocab, device="cuda", dtype=dt, requires_grad=True)
    tgt = torch.randint(0, vocab, (61,), device="cuda")
    tgt[3] = -100
    loss = cross_entropy(logits, tgt)
    lr = logits.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr, tgt, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    loss.backward()
    ref.backward()
    assert torch.allclose(logits.grad.float(), lr.grad, atol=1e-4 if dt == torch.float32 else 2e-4)


@pytest.mark.parametrize("pdt", [torch.bfloat16, None])
def test_fused_adam(C, pdt):
    from smdistributed_modelparallel_amd.ops.multi_tensor import fused_adam_

    torch.manual_seed(6)
    n = 100003
    master = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    ref = master.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    low = master.to(pdt) if pdt is not None else None
    for step in range(1, 4):
        g = torch.randn(n, device="cuda")
        gl = g.to(pdt) if pdt is not None else g
        fused_adam_(low, gl, master, m, v, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, grad_scale=1.0, adamw=True)
        ref.grad = gl.float()
        opt.step()
    assert torch.allclose(master, ref.detach(), atol=1e-5, rtol=1e-5)
    if low is not None:
        assert torch.allclose(low.float(), master, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("n", [1, 4097, 16384 * 4096 // 64 + 3])
def test_add3(C, dt, n):
    from smdistributed_modelparallel_amd.ops.dropout import add3

    a, b, c = (torch.randn(n, device="cuda", dtype=dt, requires_grad=True) for _ in range(3))
    y = add3(a, b, c)
    ref = a.detach().float() + b.detach().float() + c.detach().float()
    torch.testing.assert_close(y.float(), ref, rtol=_tol(dt), atol=_tol(dt))
    g = torch.randn_like(y)
    y.backward(g)
    for t in (a, b, c):
        assert torch.equal(t.grad, g)
    # unaligned views take the two-add fallback
    z = add3(a.detach()[1:], b.detach()[1:], c.detach()[1:])
    torch.testing.assert_close(z.float(), ref[1:], rtol=_tol(dt), atol=_tol(dt))


def test_sumsq_nonfinite(C):
    from smdistributed_modelparallel_amd.ops.multi_tensor import nonfinite_flag, sumsq

    x = torch.randn(1 << 20, device="cuda", dtype=torch.bfloat16)
    assert math.isclose(sumsq(x).item(), x.float().pow(2).sum().item(), rel_tol=1e-3)
    assert nonfinite_flag(x).item() == 0.0
    x[12345] = float("inf")
    assert nonfinite_flag(x).item() == 1.0


def test_gpt_step_gpu(C):
    """End-to-end: tiny GPT forward/backward on GPU through the kernels matches fp32 CPU."""
    from smdistributed_modelparallel_amd.models import build_gpt

    torch.manual_seed(7)
    m = build_gpt("gpt2-tiny", dropout=0.0, hidden_size=128, num_attention_heads=2, attention_head_size=64,
                  intermediate_size=512)
    ids = torch.randint(0, 512, (2, 64))
    loss_cpu, _ = m((ids, None, None, None, ids))
    loss_cpu.backward()
    g_cpu = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    m = m.cuda()
    loss_gpu, _ = m((ids.cuda(), None, None, None, ids.cuda()))
    loss_gpu.backward()
    assert abs(loss_gpu.item() - loss_cpu.item()) < 1e-3
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad.cpu(), g_cpu[n], atol=2e-3, rtol=1e-2), n


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gpt_fused_grad_accumulation_gpu(C, dt):
    """Gradients bound to pre-allocated views (the flat-buffer layout: `_smp_fused_grad`)
    are accumulated in place by the kernels -- weight GEMMs with beta=1, bias column sums,
    GeLU dbias, LayerNorm dgamma/dbeta -- and the residual stream's two gradient paths meet
    inside the LN backward.  Two accumulated backwards must equal autograd's."""
    from smdistributed_modelparallel_amd.models import build_gpt

    torch.manual_seed(11)
    kw = dict(dropout=0.0, hidden_size=128, num_attention_heads=2, attention_head_size=64, intermediate_size=512)
    ref = build_gpt("gpt2-tiny", **kw).cuda().to(dt)
    fused = build_gpt("gpt2-tiny", **kw).cuda().to(dt)
    fused.load_state_dict(ref.state_dict())
    for p in fused.parameters():
        p.grad = torch.zeros_like(p)
        p._smp_fused_grad = True
    ids = torch.randint(0, 512, (2, 64), device="cuda")
    for _ in range(2):
        for m in (ref, fused):
            loss, _ = m((ids, None, None, None, ids))
            loss.float().backward()
    tol = 2e-4 if dt == torch.float32 else 3e-2
    for (n, p), (_, q) in zip(ref.named_parameters(), fused.named_parameters()):
        assert torch.allclose(q.grad.float(), p.grad.float(), atol=tol, rtol=tol * 5), n


@pytest.mark.parametrize("family", ["gptj-6b", "gptneox-20b", "gpt3-175b"])
def test_model_family_step_gpu(C, family):
    """The BASELINE model families at reduced width/depth (same architecture flags: GPT-J
    parallel attention + interleaved RoPE, NeoX half-rotation RoPE, GPT-3 pre-LN with
    tanh GeLU) through the HIP kernels (bf16 flash attention, RoPE, fused GeLU / LN) match
    an fp32 CPU forward/backward of the same weights."""
    from smdistributed_modelparallel_amd.models import build_gpt

    torch.manual_seed(21)
    kw = dict(dropout=0.0, num_layers=2, hidden_size=256, num_attention_heads=4, attention_head_size=64,
              intermediate_size=1024, vocab_size=512, num_positions=128)
    if family != "gpt3-175b":
        kw["rotary_dim"] = 32 if family == "gptj-6b" else 16
    cpu = build_gpt(family, **kw)
    gpu = build_gpt(family, **kw)
    gpu.load_state_dict(cpu.state_dict())
    gpu = gpu.cuda().to(torch.bfloat16)
    ids = torch.randint(0, 512, (2, 128))
    lc, _ = cpu((ids, None, None, None, ids))
    lc.backward()
    lg, _ = gpu((ids.cuda(), None, None, None, ids.cuda()))
    lg.float().backward()
    assert abs(lg.item() - lc.item()) < 2e-2, (lg.item(), lc.item())
    gc = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        ref = gc[n].grad
        err = (p.grad.float().cpu() - ref).norm() / (ref.norm() + 1e-12)
        assert err < 5e-2, (n, float(err))


def test_padded_lm_head_ce_gpu(C, monkeypatch):
    """LM head + CE through the 64-padded vocabulary (odd V): loss, logits, input and
    (in-place accumulated) weight gradients equal the plain unpadded computation."""
    import smdistributed_modelparallel_amd.ops.lm_head as LH
    from smdistributed_modelparallel_amd.ops.linear import bump_weight_epoch

    torch.manual_seed(4)
    V, H, T = 1001, 256, 300
    w = (torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    x = torch.randn(2, T // 2, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    lab = torch.randint(0, V, (2, T // 2), device="cuda")
    lab[0, :7] = -100
    bump_weight_epoch()
    rows, logits = LH.padded_lm_head_cross_entropy(x, w, lab)
    assert logits.shape == (2, T // 2, V)
    gl = torch.randn(logits.shape, device="cuda") * 1e-3
    (rows.sum() + (logits.float() * gl).sum()).backward()
    wr, xr = w.detach().float().requires_grad_(), x.detach().float().requires_grad_()
    lr_ = xr @ wr.t()
    rr = torch.nn.functional.cross_entropy(lr_.view(-1, V), lab.view(-1), ignore_index=-100, reduction="none")
    (rr.sum() + (lr_ * gl).sum()).backward()
    assert torch.allclose(rows.float().view(-1), rr, atol=3e-2, rtol=1e-2)
    assert torch.allclose(logits.float(), lr_, atol=3e-2, rtol=1e-2)
    for a, b in ((x.grad, xr.grad), (w.grad, wr.grad)):
        err = (a.float() - b).norm() / b.norm()
        assert err < 2e-2, float(err)
    # in-place accumulation into a bound (flat-buffer style) gradient view
    base = torch.randn(V, H, device="cuda").to(torch.bfloat16)
    w2 = w.detach().clone().requires_grad_()
    w2.grad = base.clone()
    w2._smp_fused_grad = True
    rows2, _ = LH.padded_lm_head_cross_entropy(x.detach(), w2, lab)
    rows2.sum().backward()
    w3 = w.detach().clone().requires_grad_()
    rows3, _ = LH.padded_lm_head_cross_entropy(x.detach(), w3, lab)
    rows3.sum().backward()
    assert torch.allclose(w2.grad.float(), base.float() + w3.grad.float(), atol=2e-2)


def test_transposed_dgrad_gpu(C, monkeypatch):
    """Input gradients computed against the cached W^T (forward GEMM layout) equal
    autograd's; the cache refreshes when the weight epoch advances."""
    import smdistributed_modelparallel_amd.ops.linear as L
    from smdistributed_modelparallel_amd.models import build_gpt

    monkeypatch.setattr(L, "_use_transposed", lambda w: w.is_cuda and w.dim() == 2)
    torch.manual_seed(13)
    kw = dict(dropout=0.0, hidden_size=128, num_attention_heads=2, attention_head_size=64, intermediate_size=512)
    ref = build_gpt("gpt2-tiny", **kw).cuda()
    fused = build_gpt("gpt2-tiny", **kw).cuda()
    fused.load_state_dict(ref.state_dict())
    for p in fused.parameters():
        p.grad = torch.zeros_like(p)
        p._smp_fused_grad = True
    ids = torch.randint(0, 512, (2, 64), device="cuda")
    for step in range(2):
        L.bump_weight_epoch()
        for m in (ref, fused):
            m.zero_grad(set_to_none=(m is ref))
            loss, _ = m((ids, None, None, None, ids))
            loss.backward()
        for (n, p), (_, q) in zip(ref.named_parameters(), fused.named_parameters()):
            assert torch.allclose(q.grad, p.grad, atol=2e-4, rtol=1e-3), (step, n)
        with torch.no_grad():  # an "optimizer step" on both: W^T must follow
            for p, q in zip(ref.parameters(), fused.parameters()):
                p.add_(p.grad, alpha=-0.5)
                q.add_(q.grad, alpha=-0.5)
    w = fused.transformer.seq_layers[0].output.dense1_weight
    assert not torch.equal(w.__dict__["_smp_wt"][1], w.detach().t())  # lazily refreshed on next use
    L.bump_weight_epoch()
    fused((ids, None, None, None, ids))
    assert torch.equal(w.__dict__["_smp_wt"][1], w.detach().t())


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("shape", [(6400, 1600), (1600, 4800), (64, 64), (100, 37), (3, 1000), (1000, 72)])
def test_transpose_kernel(C, dt, shape):
    x = torch.randn(*shape, device="cuda").to(dt)
    out = torch.empty(shape[1], shape[0], device="cuda", dtype=dt)
    C.transpose_into(x, out)
    assert torch.equal(out, x.t())


def test_layer_norm_passthrough_gpu(C):
    from smdistributed_modelparallel_amd.ops.layernorm import layer_norm_passthrough

    torch.manual_seed(3)
    x = torch.randn(4, 33, 1600, device="cuda", requires_grad=True)
    w = torch.randn(1600, device="cuda", requires_grad=True)
    b = torch.randn(1600, device="cuda", requires_grad=True)
    y, r = layer_norm_passthrough(x, w, b)
    gy, gr = torch.randn_like(y), torch.randn_like(r)
    (y * gy).sum().add_((r * gr).sum()).backward()
    xr, wr, br = (t.detach().clone().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (1600,), wr, br)
    ((yr * gy).sum() + (xr * gr).sum()).backward()
    assert torch.allclose(y, yr, atol=1e-4)
    for a, c in ((x, xr), (w, wr), (b, br)):
        assert torch.allclose(a.grad, c.grad, atol=1e-3, rtol=1e-3)


def test_offloaded_checkpoint_gpu():
    """Checkpointed inputs parked in pinned host memory (D2H/H2D side streams) give the
    same gradients as plain autograd."""
    import torch.nn as nn

    from smdistributed_modelparallel_amd.runtime.checkpointing import offloaded_checkpoint
    from smdistributed_modelparallel_amd.runtime.offload import ActivationOffloader

    torch.manual_seed(9)
    layers = [nn.Sequential(nn.Linear(256, 512), nn.GELU(), nn.Dropout(0.1), nn.Linear(512, 256)).cuda()
              for _ in range(4)]
    x = torch.randn(128, 256, device="cuda", requires_grad=True)
    off = ActivationOffloader(torch.device("cuda"), horizon=2)
    torch.manual_seed(3)
    h = x
    for m in layers:
        h = offloaded_checkpoint(m, off, h)
    h.square().sum().backward()
    g_off = [p.grad.clone() for m in layers for p in m.parameters()] + [x.grad.clone()]
    assert off.stats["offloaded_bytes"] > 0 and off.stats["loaded_bytes"] == off.stats["offloaded_bytes"]
    for m in layers:
        m.zero_grad()
    x.grad = None
    torch.manual_seed(3)
    h = x
    for m in layers:
        h = m(h)
    h.square().sum().backward()
    g_ref = [p.grad for m in layers for p in m.parameters()] + [x.grad]
    for a, b in zip(g_off, g_ref):
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("neox", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("d,rd", [(64, 32), (96, 24), (64, 10), (256, 64)])
def test_rope_kernel(neox, dt, d, rd):
    """HIP RoPE vs the torch formula, fwd (strided packed-QKV view, position offset) and bwd.
    (d, rd) covers the 16-bit vector kernel with 16-byte chunks (64/32, GPT-J's 256/64), with
    8-byte chunks (NeoX-20B's 96/24) and the scalar fallback (rd 10)."""
    from smdistributed_modelparallel_amd.ops.rope import apply_rotary, apply_rotary_torch

    torch.manual_seed(4)
    qkv = torch.randn(2, 37, 3, 5, d, device="cuda", dtype=dt)
    q = qkv[:, :, 0]  # strided view into the packed QKV projection
    x = q.detach().clone().requires_grad_()
    y = apply_rotary(q, rd, 10000, neox)
    yr = apply_rotary_torch(q.float(), rd, 10000, neox)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    y2 = apply_rotary(x, rd, 10000, neox, offset=3)
    xr = x.detach().float().requires_grad_()
    yr2 = apply_rotary_torch(xr, rd, 10000, neox, offset=3)
    assert torch.allclose(y2.float(), yr2, atol=tol, rtol=tol)
    g = torch.randn_like(yr2)
    y2.backward(g.to(dt))
    yr2.backward(g)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)


@pytest.mark.parametrize("neox", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d,rd", [(64, 32), (96, 24), (64, 10), (256, 64)])
def test_rope_packed_qkv(neox, dt, d, rd):
    """Rotary on a packed QKV projection output (ops.rope.apply_rotary_qkv: q / k rotated in
    place on their rotary channels only, v and the pass-through channels untouched; the
    backward rotates the one dqkv buffer back in place) against the fp32 torch formula."""
    from smdistributed_modelparallel_amd.ops import rope

    torch.manual_seed(5)
    leaf = torch.randn(2, 37, 3 * 5 * d, device="cuda", dtype=dt, requires_grad=True)
    y = leaf * 1  # a non-leaf, non-view tensor, like a linear layer's output
    before = y.detach().clone().view(2, 37, 3, 5, d)
    n0 = rope.PACKED_CALLS[0]
    out = rope.apply_rotary_qkv(y, 2, 37, 5, d, rd, 10000, neox)
    assert rope.PACKED_CALLS[0] == n0 + 1
    assert out.shape == (2, 37, 3, 5, d) and out.data_ptr() == y.data_ptr()  # in place
    ref_in = before.float().requires_grad_()
    ref = torch.stack((rope.apply_rotary_torch(ref_in[:, :, 0], rd, 10000, neox),
                       rope.apply_rotary_torch(ref_in[:, :, 1], rd, 10000, neox), ref_in[:, :, 2]), dim=2)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert torch.allclose(out.float(), ref, atol=tol, rtol=tol)
    assert torch.equal(out[:, :, 2], before[:, :, 2])
    assert torch.equal(out[..., rd:], before[..., rd:])  # pass-through channels untouched
    g = torch.randn_like(ref)
    gd = g.to(dt).clone()
    keep = gd.clone()
    out.backward(gd)
    ref.backward(g)
    assert torch.allclose(leaf.grad.float().view_as(ref_in.grad), ref_in.grad, atol=tol * 2, rtol=tol * 2)
    assert torch.equal(gd, keep)  # a caller's gradient is not modified (only marked fresh buffers are)


@pytest.mark.parametrize("neox", [False, True])
def test_rotary_layer_packed_matches_per_view(neox):
    """A rotary DistributedTransformer (GPT-J / NeoX style) on GPU: the packed in-place rotary
    path gives the same outputs and gradients as the per-view path (SMP_ROPE_PACKED=0)."""
    import smdistributed_modelparallel_amd.nn.transformer as T
    from smdistributed_modelparallel_amd.nn import DistributedTransformer
    from smdistributed_modelparallel_amd.ops import rope

    torch.manual_seed(0)
    kw = dict(num_layers=2, num_attention_heads=4, attention_head_size=64, hidden_size=256, intermediate_size=512,
              rotary_dim=16 if neox else 32, gpt_neox_type_rotary=neox, causal_mask_size=128,
              attention_dropout_prob=0.0, hidden_dropout_prob=0.0, pre_layernorm=True, post_layernorm=False,
              parallel_attn_output=True)
    ref = DistributedTransformer(**kw).cuda().to(torch.bfloat16)
    x = torch.randn(2, 128, 256, device="cuda", dtype=torch.bfloat16)
    res = {}
    for packed in (True, False):
        T._ROPE_PACKED = packed
        try:
            m = DistributedTransformer(**kw).cuda().to(torch.bfloat16)
            m.load_state_dict(ref.state_dict())
            xi = x.clone().requires_grad_()
            n0 = rope.PACKED_CALLS[0]
            out = m((xi, None))[0]
            out.float().pow(2).sum().backward()
            assert (rope.PACKED_CALLS[0] > n0) == packed
            res[packed] = (out.float(), xi.grad.float(), [p.grad.float() for p in m.parameters()])
        finally:
            T._ROPE_PACKED = True
    a, b = res[True], res[False]
    assert torch.allclose(a[0], b[0], atol=2e-2, rtol=2e-2)
    for u, v in [(a[1], b[1])] + list(zip(a[2], b[2])):
        assert ((u - v).norm() / v.norm().clamp_min(1e-6)).item() < 2e-2


def test_lamb_segmented_kernel_matches_cpu():
    """Whole-domain LAMB stage 2 (lamb_norms_chunked + lamb_stage2_chunked): per-segment trust
    ratios equal the per-parameter CPU computation; the bf16 param copy is written too."""
    from smdistributed_modelparallel_amd.ops import multi_tensor as mt

    torch.manual_seed(0)
    pieces = [(0, 70000), (70000, 70013), (70100, 200000)]
    n = 200000
    master = torch.randn(n)
    upd = torch.randn(n) * 0.1
    table = mt.lamb_chunk_table(pieces, "cpu")
    ref_m = master.clone()
    mt.lamb_segmented_(None, ref_m, upd, table, len(pieces), 0.01, True)
    gm = master.cuda()
    gp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    mt.lamb_segmented_(gp, gm, upd.cuda(), table.cuda(), len(pieces), 0.01, True)
    torch.testing.assert_close(gm.cpu(), ref_m, rtol=1e-5, atol=1e-6)
    covered = torch.zeros(n, dtype=torch.bool)
    for s, e in pieces:
        covered[s:e] = True
    torch.testing.assert_close(gp.float().cpu()[covered], ref_m[covered], rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("rows,cols", [(4097, 6400), (3001, 2056), (65, 40)])
def test_gelu_one_pass_matches_unfused_dbias(C, rows, cols):
    """The one-pass bias-GeLU kernels (forward, and the pure elementwise backward used when the
    weight-gradient kernel supplies the bias gradient) against the column-walker backward that
    also sums dbias: same per-element math, so y and dx are bitwise equal."""
    torch.manual_seed(11)
    x = torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(cols, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    for exact in (False, True):
        dx1 = C.bias_gelu_bwd(dy, x, b, exact)
        dx2, db = C.bias_gelu_bwd_dbias(dy, x, b, None, exact)
        assert torch.equal(dx1, dx2)
        ref = (x.float() + b.float())
        y = C.bias_gelu_fwd(x, b, exact)
        yr = torch.nn.functional.gelu(ref, approximate="none" if exact else "tanh")
        assert (y.float() - yr).abs().max().item() < 2e-2


@pytest.mark.parametrize("xdt,wdt", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                     (torch.float16, torch.float32)])
@pytest.mark.parametrize("cols", [1600, 1001])
def test_mixed_fused_layer_norm(xdt, wdt, cols):
    """MixedFusedLayerNorm (K10): output in the parameters' dtype straight from the kernel;
    forward and backward against fp32 torch."""
    from smdistributed_modelparallel_amd.nn.layer_norm import MixedFusedLayerNorm

    torch.manual_seed(4)
    ln = MixedFusedLayerNorm(cols).cuda().to(wdt)
    with torch.no_grad():
        ln.weight.normal_(1.0, 0.1)
        ln.bias.normal_(0.0, 0.1)
    x = torch.randn(257, cols, device="cuda", dtype=xdt, requires_grad=True)
    y = ln(x)
    assert y.dtype == wdt
    xr = x.detach().float().requires_grad_()
    wr, br = ln.weight.detach().float().requires_grad_(), ln.bias.detach().float().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (cols,), wr, br, ln.eps)
    tol = 2e-2 if torch.bfloat16 in (xdt, wdt) else 5e-3
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(wdt))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 4, rtol=tol * 4)
    torch.testing.assert_close(ln.weight.grad.float(), wr.grad, atol=tol * 20, rtol=tol * 4)
