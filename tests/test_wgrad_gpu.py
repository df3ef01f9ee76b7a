"""Weight-gradient GEMM of ops/linear.py (library GEMM or the split-K MFMA kernel of
csrc/kernels/wgrad.hip, picked from the fixed per-shape table or -- opt-in -- timed) against
an fp32 PyTorch reference."""
import pytest
import torch

from smdistributed_modelparallel_amd.ops import linear as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(4096, 1600, 1600), (65536, 256, 256), (8200, 4800, 1600), (5000, 392, 1048),
                                   (16384, 1600, 6400)])
@pytest.mark.parametrize("gdtype", [torch.bfloat16, torch.float32])
def test_wgrad_kernel_matches_fp32(shape, gdtype):
    """csrc/kernels/wgrad.hip (split-K MFMA, LDS transpose reads): c += dy^T x against the
    fp32 reference, ragged token counts and edge tiles included; bf16 grads and fp32 main
    grads."""
    from smdistributed_modelparallel_amd.ops._ext import ext

    T, N, K = shape
    g0 = torch.Generator(device="cuda").manual_seed(2)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    g = torch.randn(N, K, device="cuda", dtype=gdtype, generator=g0)
    ref = g.float() + dy.float().t() @ x.float()
    ext().wgrad_(g, dy, x, True)
    err = (g.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (1e-2 if gdtype == torch.bfloat16 else 1e-5), err
    # explicit split counts give the same sums; accumulate=False overwrites
    for splits in (1, 3, 5, 6, 8):
        h = torch.empty(N, K, device="cuda", dtype=torch.float32)
        ext().wgrad_(h, dy, x, False, splits)
        torch.testing.assert_close(h, dy.float().t() @ x.float(), rtol=1e-4, atol=1e-3 * ref.abs().max().item())


def test_wgrad_kernel_strided_rows_and_f16():
    from smdistributed_modelparallel_amd.ops._ext import ext

    g0 = torch.Generator(device="cuda").manual_seed(3)
    big = torch.randn(6000, 3 * 512, device="cuda", dtype=torch.float16, generator=g0)
    dy = big[:, 512:1024]  # row stride 1536
    x = torch.randn(6000, 264, device="cuda", dtype=torch.float16, generator=g0)
    g = torch.zeros(512, 264, device="cuda", dtype=torch.float32)
    ext().wgrad_(g, dy, x, True)
    torch.testing.assert_close(g, dy.float().t() @ x.float(), rtol=1e-4, atol=1e-2)


def test_linear_uses_wgrad_kernel_for_bound_grads(monkeypatch):
    """ops.linear: a weight whose .grad is bound (flat buffer) accumulates through the kernel
    (forced) and through the timed per-shape choice (auto): one accumulation either way."""
    monkeypatch.setattr(L, "_WGRAD_KERNEL", "1")
    T, N, K = 8192, 512, 384
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w.grad = torch.zeros_like(w)
    w._smp_fused_grad = True
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = L.linear(x, w)
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = dy.float().t() @ x.detach().float()
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_wgrad_timed_choice_accumulates_once(monkeypatch):
    """SMP_WGRAD_PICK=timed: the trials restore the gradient; exactly one accumulation lands."""
    monkeypatch.setattr(L, "_WGRAD_KERNEL", "auto")
    monkeypatch.setattr(L, "_WGRAD_PICK", "timed")
    T, N, K = 8192, 1024, 512
    g0 = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    g = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    ref = g.float() + dy.float().t() @ x.float()
    L._WGRAD_KERNEL_CHOICE.clear()
    L._wgrad_accumulate(g, dy, x)
    assert len(L._WGRAD_KERNEL_CHOICE) == 1
    err = (g.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_wgrad_static_pick_is_deterministic(monkeypatch):
    """Default table pick: the measured per-shape winner without timing trials; two runs give
    bitwise identical gradients (same split-K accumulation order).  Off-table shapes take the
    library GEMM (no trial, no host sync)."""
    monkeypatch.setattr(L, "_WGRAD_PICK", "table")
    T, N, K = 16384, 1600, 1600  # table entry: kernel, 5 splits
    g0 = torch.Generator(device="cuda").manual_seed(3)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    base = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    key = (T, N, K, torch.bfloat16, torch.bfloat16)
    L._WGRAD_KERNEL_CHOICE.pop(key, None)
    outs = []
    for _ in range(2):
        g = base.clone()
        L._wgrad_accumulate(g, dy, x)
        outs.append(g)
    assert L._WGRAD_KERNEL_CHOICE[key] == 5
    assert torch.equal(outs[0], outs[1])
    ref = base.float() + dy.float().t() @ x.float()
    err = (outs[0].float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    L._WGRAD_KERNEL_CHOICE.pop(key, None)
    off = (T, 1024, 512, torch.bfloat16, torch.bfloat16)
    L._WGRAD_KERNEL_CHOICE.pop(off, None)
    g = torch.zeros(1024, 512, device="cuda", dtype=torch.bfloat16)
    L._wgrad_accumulate(g, dy[:, :1024].contiguous(), x[:, :512].contiguous())
    assert L._WGRAD_KERNEL_CHOICE[off] == 0


# K 1600 / 1048: idle-wave MFMA column sums; K 6400 / 1000: LDS column sums
@pytest.mark.parametrize("shape", [(4096, 1600, 1600), (8200, 4800, 1600), (5000, 392, 1048), (16384, 1600, 6400),
                                   (4160, 1040, 1000)])
@pytest.mark.parametrize("bdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("accumulate", [True, False])
def test_wgrad_kernel_fused_bias_colsum(shape, bdtype, accumulate):
    """The weight-gradient kernel's fused bias pass: dbias (+)= sum over tokens of dy from the
    staged dy tiles (edge column tile, ragged token tail, several split counts) against fp32;
    the weight gradient of the same call is unchanged."""
    from smdistributed_modelparallel_amd.ops._ext import ext

    T, N, K = shape
    g0 = torch.Generator(device="cuda").manual_seed(3)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    for splits in (0, 1, 3):
        g = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g0)
        b = torch.randn(N, device="cuda", dtype=bdtype, generator=g0)
        ref_g = g.float() + dy.float().t() @ x.float()
        ref_b = (b.float() if accumulate else 0.0) + dy.float().sum(0)
        ext().wgrad_(g, dy, x, True, splits, b, accumulate)
        eg = (g.float() - ref_g).abs().max().item() / ref_g.abs().max().item()
        eb = (b.float() - ref_b).abs().max().item() / ref_b.abs().max().item()
        assert eg < 1e-2, (splits, eg)
        assert eb < (1e-2 if bdtype == torch.bfloat16 else 1e-4), (splits, eb)


def test_mlp_dense1_bias_grad_through_wgrad_kernel(monkeypatch):
    """GPT MLP on GPU: dense1_bias's gradient comes from dense1's weight-gradient kernel
    (bias-GeLU backward without its own column sums); it must match the unfused path
    (SMP_WGRAD_DBIAS off) and an fp32 CPU reference of the same layer."""
    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.nn.transformer import DistributedTransformerOutputLayer
    from smdistributed_modelparallel_amd.ops import linear as lin

    smp.init({"bf16": True})
    torch.manual_seed(0)
    ref = DistributedTransformerOutputLayer(hidden_size=256, intermediate_size=1024, activation="gelu",
                                            pre_layernorm=True, post_layernorm=False, hidden_dropout_prob=0.0)
    with torch.no_grad():
        for p in ref.parameters():
            p.normal_(0.0, 0.05)
    x = torch.randn(4, 2048, 256)
    ref.float()
    xr = x.clone().requires_grad_(True)
    ref(xr).float().pow(2).sum().backward()
    want = ref.dense1_bias.grad.clone()

    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(lin, "_WGRAD_DBIAS", fused)
        m = DistributedTransformerOutputLayer(hidden_size=256, intermediate_size=1024, activation="gelu",
                                              pre_layernorm=True, post_layernorm=False, hidden_dropout_prob=0.0)
        m.load_state_dict(ref.state_dict())
        m = m.cuda().to(torch.bfloat16)
        # bind flat-buffer-style grads so the weight-gradient kernel path is taken
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
            p._smp_fused_grad = True
        xc = x.cuda().to(torch.bfloat16).requires_grad_(True)
        m(xc).float().pow(2).sum().backward()
        torch.cuda.synchronize()
        grads[fused] = m.dense1_bias.grad.float().cpu()
    scale = want.abs().max().item()
    for fused, g in grads.items():
        err = (g - want).abs().max().item() / scale
        assert err < 3e-2, (fused, err)
    assert (grads[True] - grads[False]).abs().max().item() / scale < 3e-2


@pytest.mark.parametrize("shape", [(64, 256, 256), (192, 520, 264), (4160, 1040, 1000), (8192, 4800, 1600),
                                   (12288, 1600, 6400), (2048, 264, 1032)])
@pytest.mark.parametrize("impl", [0, 1])
def test_wgrad_impls_match_fp32(shape, impl):
    """Both kernels of csrc/kernels/wgrad.hip (1 = ping-pong, 0 = one barrier per tile) against
    fp32 torch by relative norm: 1-3 token tiles (prologue / tail paths), odd tile counts,
    split counts that leave a split with no tokens, edge row / column tiles."""
    from smdistributed_modelparallel_amd.ops._ext import ext

    T, N, K = shape
    g0 = torch.Generator(device="cuda").manual_seed(11)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    ref = dy.float().t() @ x.float()
    for splits in (1, 2, 3, 7):
        h = torch.full((N, K), float("nan"), device="cuda", dtype=torch.float32)
        ext().wgrad_(h, dy, x, False, splits, impl=impl)
        rel = ((h - ref).norm() / ref.norm()).item()
        assert rel < 1e-5, (splits, rel)


@pytest.mark.parametrize("shape", [(4096, 1600, 1600), (8256, 4800, 1600), (5000, 392, 1048), (4160, 1040, 1000),
                                   (4096, 1600, 6400), (4096, 1536, 6144), (2048, 520, 512), (4096, 800, 1200)])
def test_wgrad_pp_bias_quadrant(shape):
    """The ping-pong kernel's bias-gradient sums against fp32 column sums: the idle-quadrant mode
    (K % 256 in [1, 128]: B fragment = ones in the idle qb = 1 quadrant of the last K tile) and
    the row-sum MFMA mode for every other K (K % 256 == 0 as in the GPT-J / NeoX shards, and
    K % 256 > 128), beside the round-4 kernel's modes on the same call API."""
    from smdistributed_modelparallel_amd.ops._ext import ext

    T, N, K = shape
    g0 = torch.Generator(device="cuda").manual_seed(12)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g0)
    ref_g = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    # impl 2: the ping-pong kernel with the row-sum mode allowed (K % 256 == 0 or > 128)
    for impl in (2, 1, 0):
        for splits in (1, 4):
            g = torch.zeros(N, K, device="cuda", dtype=torch.float32)
            b = torch.zeros(N, device="cuda", dtype=torch.float32)
            ext().wgrad_(g, dy, x, True, splits, b, True, impl=impl)
            assert ((g - ref_g).norm() / ref_g.norm()).item() < 1e-5
            assert ((b - ref_b).norm() / ref_b.norm()).item() < 1e-5, (impl, splits)
