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

Input gradients run in the forward GEMM's layout.  hipBLASLt on gfx950 is markedly
faster when both operands are contiguous along the reduction dimension (the forward's
``x @ W^T``: e.g. 1.79 PFLOP/s for 32768x1600 @ 1600x6400) than for the input-gradient
product ``dY @ W`` whose W operand is strided along the reduction (1.18 PFLOP/s for the
same m/n/k, TunableOp-selected, `configs/tunableop`).  Inside an ``@smp.step`` each
weight therefore keeps a transposed copy ``W^T`` (refreshed once per step on first use,
~1 ms per step for GPT-2 XL's 1.5 B weights, +2 B/param of HBM, capped at 8 % of the device
by default: ``SMP_TRANSPOSED_DGRAD_BUDGET_GB``) and the input gradient is
``F.linear(dY, W^T)`` -- the fast layout.  ``SMP_TRANSPOSED_DGRAD=0`` disables it.
"""
import os

import torch
import torch.nn.functional as F

_WT_EPOCH = [0]
_WT_MIN_NUMEL = 1 << 20
_WT_ENABLED = os.environ.get("SMP_TRANSPOSED_DGRAD", "1") != "0"
# HBM spent on W^T copies is capped: by default at min(8 % of the device, 10 % of the memory
# still free when the first copy is requested -- model, gradients and optimizer state are
# allocated by then), so models near the memory limit keep their capacity; the first
# weights up to the cap get a copy, the rest use the strided-layout GEMM
_WT_BUDGET = [None, 0]  # [cap bytes, bytes in use]


def bump_weight_epoch():
    """Weights may have changed (new step, optimizer update, load): transposed copies are
    refreshed on their next use."""
    _WT_EPOCH[0] += 1


def _transposed(w):
    """Contiguous W^T of a 2-D weight, cached per (epoch, storage, version); the cached
    buffer is reused across refreshes (no allocator churn)."""
    key = (_WT_EPOCH[0], w.data_ptr(), w._version)
    ent = w.__dict__.get("_smp_wt")
    if ent is not None and ent[0] == key:
        return ent[1]
    buf = ent[1] if ent is not None and ent[1].dtype == w.dtype and ent[1].shape == (w.shape[1], w.shape[0]) else None
    with torch.no_grad():
        if buf is None:
            try:
                buf = torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
            except torch.OutOfMemoryError:
                w.__dict__["_smp_wt_ok"] = False  # no room: this weight keeps the strided GEMM
                return None
        if w.is_cuda and w.is_contiguous():
            from ._ext import ext

            ext().transpose_into(w.detach(), buf)  # LDS-tiled HIP transpose (HBM rate)
        else:
            buf.copy_(w.detach().t())
    w.__dict__["_smp_wt"] = (key, buf)
    return buf


def _wt_admit(w):
    """Reserve W^T bytes for w under the HBM cap (decided once per weight)."""
    ok = w.__dict__.get("_smp_wt_ok")
    if ok is not None:
        return ok
    if _WT_BUDGET[0] is None:
        gb = os.environ.get("SMP_TRANSPOSED_DGRAD_BUDGET_GB")
        if gb:
            _WT_BUDGET[0] = int(float(gb) * 2**30)
        else:
            total = torch.cuda.get_device_properties(w.device).total_memory
            free = torch.cuda.mem_get_info(w.device)[0]
            free += torch.cuda.memory_reserved(w.device) - torch.cuda.memory_allocated(w.device)
            _WT_BUDGET[0] = int(min(0.08 * total, 0.10 * free))
    need = w.numel() * w.element_size()
    ok = _WT_BUDGET[1] + need <= _WT_BUDGET[0]
    if ok:
        _WT_BUDGET[1] += need
    w.__dict__["_smp_wt_ok"] = ok
    return ok


def _use_transposed(w):
    if not (_WT_ENABLED and w.is_cuda and w.dim() == 2 and w.numel() >= _WT_MIN_NUMEL):
        return False
    if w.shape[0] % 64 != 0:
        # W^T rows of an odd length (e.g. a 50257-token LM head) are misaligned for the GEMM:
        # measured slower than the strided form (5.54 vs 4.74 ms for GPT-2 XL's LM head)
        return False
    from ..torch.state_mod import state

    return bool(getattr(state, "in_step_func", False)) and _wt_admit(w)


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
        ctx.wt = _transposed(weight) if _use_transposed(weight) else None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = db = None
        dy2 = dy.reshape(-1, dy.shape[-1])
        if ctx.needs_input_grad[0]:
            dx = F.linear(dy, ctx.wt) if ctx.wt is not None else torch.matmul(dy, w)
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
