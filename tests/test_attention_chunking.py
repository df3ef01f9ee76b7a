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
