"""Linear layer whose weight gradient is accumulated by the GEMM itself.

With the flat gradient buffer (`parallel/flat.py`) every ``param.grad`` is a view into one
HBM buffer.  Stock autograd computes ``dW = dY^T X`` into a fresh tensor and then runs a
separate elementwise ``grad += dW`` (one full read-modify-write of every weight per
backward).  Here the weight-gradient GEMM runs with beta = 1 directly on the bound view
(``grad.addmm_(dY^T, X)``: hipBLASLt reads C in its epilogue), so the extra pass and the
temporary disappear, and the reducers' post-accumulate-grad hooks still fire once per
backward (bucketed all-reduce overlap is unchanged).

Falls back to ``F.linear``'s autograd whenever the weight has no bound flat-buffer grad
(plain modules, sharded data parallelism, dtype mismatch).
"""
import torch
import torch.nn.functional as F


def _col_sum(x2, out=None):
    """Bias gradient: HIP two-stage column sum on GPU (HBM-rate), torch elsewhere.
    With ``out`` the sums are accumulated into it in place (and ``out`` is returned)."""
    if x2.is_cuda and x2.dtype in (torch.float16, torch.bfloat16, torch.float32) and x2.is_contiguous():
        from ._ext import ext

        return ext().col_sum(x2, out)
    if out is not None:
        return out.add_(x2.sum(0).to(out.dtype))
    return x2.sum(0)


def _fusable(w):
    g = w.grad
    return (getattr(w, "_smp_fused_grad", False) and g is not None and g.dtype == w.dtype and g.shape == w.shape
            and g.is_contiguous())


class _LinearWGradAccum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias = bias
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = db = None
        dy2 = dy.reshape(-1, dy.shape[-1])
        if ctx.needs_input_grad[0]:
            dx = torch.matmul(dy, w)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if _fusable(ctx.bias) and dy2.is_cuda:
                _col_sum(dy2, ctx.bias.grad)  # into the bound flat-buffer view (no temp + add)
            else:
                db = _col_sum(dy2)
        if ctx.needs_input_grad[1]:
            if _fusable(w):
                # beta = 1 GEMM into the bound flat-buffer view; returning None still runs the
                # weight's AccumulateGrad node (a no-op), so post-accumulate-grad hooks -- the
                # reducers' bucket-ready signals -- fire exactly once, after this write
                w.grad.addmm_(dy2.t(), x.reshape(-1, x.shape[-1]))
            else:
                # grad slot re-bound/removed since forward: hand the gradient to autograd
                return dx, dy2.t().mm(x.reshape(-1, x.shape[-1])), db
        return dx, None, db


def linear(x, weight, bias=None):
    """F.linear with GEMM-fused weight-gradient accumulation into the flat grad buffer."""
    if torch.is_grad_enabled() and weight.requires_grad and _fusable(weight):
        return _LinearWGradAccum.apply(x, weight, bias)
    return F.linear(x, weight, bias)
