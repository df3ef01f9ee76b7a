"""Batch-chunked materialised attention (ops/attention.py _MAX_SCORE_ELEMS) equals the
single-shot computation, forward and backward, with and without a per-batch mask."""
import torch

from smdistributed_modelparallel_amd.ops import attention as A


def _run(q, k, v, mask, causal):
    q, k, v = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = A.attention(q, k, v, causal=causal, mask=mask)
    o.backward(torch.ones_like(o))
    return o.detach(), q.grad, k.grad, v.grad


def test_chunked_matches_single_shot(monkeypatch):
    torch.manual_seed(0)
    b, s, h, d = 5, 16, 2, 8
    q, k, v = (torch.randn(b, s, h, d) for _ in range(3))
    mask = torch.rand(b, 1, s, s) > 0.7
    for m, causal in ((None, True), (mask, False), (mask[:1], True)):
        ref = _run(q, k, v, m, causal)
        monkeypatch.setattr(A, "_MAX_SCORE_ELEMS", 2 * h * s * s)  # chunks of 2 batch rows (2, 2, 1)
        got = _run(q, k, v, m, causal)
        monkeypatch.setattr(A, "_MAX_SCORE_ELEMS", 1 << 26)
        for r, g in zip(ref, got):
            torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)


def test_checkpoint_attentions_saves_no_scores_and_matches(monkeypatch):
    """checkpoint_attentions (reference nn/transformer.py:1487-1496): same outputs and
    gradients -- dropout included, the RNG state is replayed -- and no [b, h, s, s] tensor
    is kept for backward."""
    import types

    from smdistributed_modelparallel_amd.torch.state_mod import state

    torch.manual_seed(0)
    b, s, h, d = 2, 32, 2, 8
    q, k, v = (torch.randn(b, s, h, d) for _ in range(3))

    def run(ckpt):
        monkeypatch.setattr(state, "cfg", types.SimpleNamespace(checkpoint_attentions=ckpt))
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
        saved = []

        def pack(t):
            saved.append(tuple(t.shape))
            return t

        torch.manual_seed(3)
        with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
            o = A.attention(qq, kk, vv, causal=True, dropout_p=0.2)
        o.backward(torch.ones_like(o))
        return (o.detach(), qq.grad, kk.grad, vv.grad), saved

    ref, saved_ref = run(False)
    got, saved_ck = run(True)
    for r, g in zip(ref, got):
        torch.testing.assert_close(g, r, rtol=1e-5, atol=1e-6)
    assert any(sh[-2:] == (s, s) for sh in saved_ref)
    assert not any(len(sh) == 4 and sh[-2:] == (s, s) for sh in saved_ck)


def test_materialised_gemm_layouts_avoid_faulting_nt_product():
    """Regression for the GPT-J illegal address (profiles/r2/gptj_fault_root_cause.md): no
    batched GEMM of the materialised path (fwd + bwd) multiplies a score-sized [bh, sq, sk]
    operand by a TRANSPOSED view of a contiguous [bh, d, sk] tensor -- the layout whose
    hipBLASLt stream-K solution faults on MI355X."""
    from torch.utils._python_dispatch import TorchDispatchMode

    b, s, h, d = 2, 32, 4, 16
    bad = []

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if func in (torch.ops.aten.bmm.default, torch.ops.aten.baddbmm.default):
                a, bm = (args[0], args[1]) if func == torch.ops.aten.bmm.default else (args[1], args[2])
                if a.shape[-1] == s and a.shape[-2] == s and bm.shape[-1] == d and bm.stride(-1) != 1:
                    bad.append((tuple(a.shape), tuple(bm.shape), tuple(bm.stride())))
            return func(*args, **(kwargs or {}))

    for causal in (True, False):
        q, k, v = (torch.randn(b, s, h, d, requires_grad=True) for _ in range(3))
        with Spy():
            o = A.attention(q, k, v, causal=causal, use_flash=False)
            o.backward(torch.ones_like(o))
    assert not bad, bad


def test_flash_dropout_byte_keep_test_swar():
    """The flash kernels' per-byte keep test (attention_impl.h keep_flags, constants from
    bindings.cpp attn_params): bit 8i+7 set iff byte i >= thr, for every threshold, in both
    the thr <= 128 and the complemented thr > 128 form; realised keep probability 1 - thr/256."""
    import random

    M = 0xFFFFFFFF
    rnd = random.Random(0)
    words = [rnd.getrandbits(32) for _ in range(64)] + [0, M, 0x7F7F7F7F, 0x80808080, 0x807F0180]
    for thr in range(0, 257):
        t7 = thr if thr <= 128 else 256 - thr
        xr = 0 if thr <= 128 else M
        c = (128 - t7) * 0x01010101
        for h in words:
            hx = h ^ xr
            f = ((((hx & 0x7F7F7F7F) + c) & M) | hx) ^ xr
            for i in range(4):
                assert bool((f >> (8 * i + 7)) & 1) == (((h >> (8 * i)) & 0xFF) >= thr), (thr, hex(h), i)
    # exact rate (the plain 8-bit threshold turned p = 0.001 into 0.0039): the
    # per-block {lo, lo + 1} threshold mixture keeps every element at dropout_p to 2^-24
    for p in (0.001, 0.01, 0.1, 0.37, 0.999):
        lo, frac = A.flash_dropout_threshold(p)
        assert abs((lo + frac / 65536.0) / 256.0 - p) < 2 ** -24
        assert abs(A.flash_dropout_keep_prob(p) - (1 - p)) < 2 ** -24
    keep = A.flash_dropout_keep_mask(2, 3, 256, 256, 0.1, 1234, 7)
    assert abs(keep.float().mean().item() - 0.9) < 0.005
    keep = A.flash_dropout_keep_mask(4, 4, 256, 256, 0.01, 99, 3)
    assert abs((1 - keep.float().mean().item()) - 0.01) < 0.002
