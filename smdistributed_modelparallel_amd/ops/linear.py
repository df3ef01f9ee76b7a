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

from ..backend.logger import get_logger

logger = get_logger()

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


# ----------------------------------------------------------------- weight-gradient algorithm
# dW[N, K] += dY[T, N]^T X[T, K] reduces over all T = batch x sequence tokens: few output tiles
# and both operands strided along the reduction, the layout hipBLASLt runs slowest.  The
# hand-written split-K MFMA kernel (csrc/kernels/wgrad.hip) reads both token-major operands as
# they are and accumulates into the gradient with beta = 1.  Which one runs, and at how many
# splits, comes from a FIXED per-shape table measured on MI355X -- no timing trials in the
# backward, no host synchronisation, and the same split-K accumulation order on every run and
# every rank.  Shapes off the table use the library GEMM.  (Measured and removed: transposing
# the operands for a TN GEMM and a batched split-K through the library -- isolated wins that
# did not survive the step, profiles/r2/gemm_epilogue_and_wgrad_stream.md; weight gradients on
# a side HIP stream -- 773.6 vs 776.0 ms/step, 256 x 256-tile GEMM workgroups fill a CU.)
#
# SMP_WGRAD_KERNEL=0 never uses the kernel, =1 always does (occupancy-model split count);
# SMP_WGRAD_PICK=timed times library vs kernel split counts per shape on first use (the
# measurement mode that produced the table; per-process, so ranks may pick differently).
_WGRAD_KERNEL = os.environ.get("SMP_WGRAD_KERNEL", "auto")
_WGRAD_KERNEL_MIN_T = 4096
_WGRAD_KERNEL_CHOICE = {}
_WGRAD_KERNEL_SPLIT_BEST = {}  # (T, N, K) -> fastest kernel split count seen by the timing pick
_WGRAD_PICK_ROUNDS = 2


def _wgrad_native_ok(g, dy2, x2):
    return (_WGRAD_KERNEL != "0" and g.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16)
            and x2.dtype == dy2.dtype and g.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and g.is_contiguous() and dy2.shape[0] >= _WGRAD_KERNEL_MIN_T and dy2.stride(1) == 1
            and x2.stride(1) == 1 and dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0 and dy2.stride(0) % 8 == 0
            and x2.stride(0) % 8 == 0 and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0)


# The table: (N, K) -> kernel split count (0 = library GEMM), for T >= _WGRAD_STATIC_MIN_T tokens.
# GPT-2 XL (T = 65536, profiles/r2/session4_wgrad_pick_ab.md, profiles/r3/wgrad_variants.md);
# (4800, 1600): s7 in the b32 step with the fused bias sums (1092-1099 us vs s5 1131, s8 1167).
# BASELINE config 3-5 rank shapes (scaled-batch TP): tools/wgrad_table.py, profiles/r4/.
# Round 5 (ping-pong kernel, tools/wgrad_pp_ab.py, profiles/r5/wgrad_pp.md): the kernel now wins
# every GPT-2 XL shape, fc2's (1600, 6400) included (s4 1325 us vs library 1891 us isolated).
_WGRAD_STATIC = {(1600, 6400): 4, (6400, 1600): 4, (1600, 1600): 5, (4800, 1600): 7,
                 # GPT-J TP4 attention output (T = 16384): s4 137 us vs library 168 us; GPT-NeoX
                 # TP4 QKV: s1 959 vs 1034 us; the other config 3-5 shapes measured library-best
                 (4096, 1024): 4, (4608, 6144): 1}
# kernel split count for a library-table shape when the fused bias pass makes the kernel the choice
_WGRAD_STATIC_KERNEL = {(1600, 6400): 4}
_WGRAD_PICK = os.environ.get("SMP_WGRAD_PICK", "table")
_WGRAD_STATIC_MIN_T = 16384


def _wgrad_static_pick(dy2, x2):
    return _WGRAD_STATIC.get((dy2.shape[1], x2.shape[1]), 0) if dy2.shape[0] >= _WGRAD_STATIC_MIN_T else 0


def _wgrad_kernel_splits(g, dy2, x2):
    """Split count for the MFMA kernel at this (T, N, K, dtypes), or 0 for the library GEMM:
    the fixed table (default), or -- SMP_WGRAD_PICK=timed -- timed once per shape: the kernel
    at its occupancy-model split count and a ladder of smaller counts, and the library."""
    if _WGRAD_KERNEL == "1" or g.dtype != dy2.dtype:  # (fp32 accumulators: no library equivalent)
        return -1  # kernel, default split count
    key = (dy2.shape[0], dy2.shape[1], x2.shape[1], dy2.dtype, g.dtype)
    hit = _WGRAD_KERNEL_CHOICE.get(key)
    if hit is not None:
        return hit
    if _WGRAD_PICK != "timed" or torch.are_deterministic_algorithms_enabled():
        _WGRAD_KERNEL_CHOICE[key] = _wgrad_static_pick(dy2, x2)
        return _WGRAD_KERNEL_CHOICE[key]
    from ._ext import ext

    C = ext()
    T = dy2.shape[0]
    model = C.wgrad_splits(T, dy2.shape[1], x2.shape[1], torch.cuda.get_device_properties(g.device).multi_processor_count)
    # the occupancy model over-splits the long GPT-2 XL shapes (measured: s4 beats s10 on
    # 6400x1600, s7 beats s15 on 4800x1600), so a ladder of small counts is timed as well
    splits = sorted({s for s in (model, max(1, model // 2), 8, 6, 5, 4, 3, 2) if s <= max(1, T // 512)},
                    reverse=True)
    cands = [(s, (lambda s=s: C.wgrad_(g, dy2, x2, True, s))) for s in splits]
    cands.append((0, lambda: g.addmm_(dy2.t(), x2)))
    saved = g.clone()
    times = {}
    for name, fn in cands:
        fn()  # warm-up (library solution selection, allocator)
    g.copy_(saved)
    # interleaved rounds, best of each: the first use of a shape falls in a warm-up step where
    # clocks still move, and a single back-to-back round favoured whichever ran last
    for _ in range(_WGRAD_PICK_ROUNDS):
        for name, fn in cands:
            start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            start.record()
            for _ in range(3):
                fn()
            end.record()
            end.synchronize()
            times[name] = min(times.get(name, float("inf")), start.elapsed_time(end))
            g.copy_(saved)
    del saved
    best = min(times, key=times.get)
    _WGRAD_KERNEL_CHOICE[key] = best
    ks = {sp: t for sp, t in times.items() if sp != 0}
    if ks:
        _WGRAD_KERNEL_SPLIT_BEST[(key[0], key[1], key[2])] = min(ks, key=ks.get)
    logger.debug(f"wgrad T={key[0]} N={key[1]} K={key[2]}: "
                 + ", ".join(f"{'library' if s == 0 else f'kernel s{s}'} {t / 3:.3f} ms" for s, t in times.items())
                 + f" -> {'library' if best == 0 else f'kernel s{best}'}")
    return best


def _wgrad_kernel_wins(g, dy2, x2):
    return _wgrad_kernel_splits(g, dy2, x2) != 0


# Bias gradients from the weight-gradient kernel (SMP_WGRAD_DBIAS, default on): when a layer's
# weight gradient runs on the MFMA kernel with bf16 operands, the kernel also sums dY over the
# tokens (the bias gradient) from the dY tiles it stages anyway, so no separate column-sum
# pass reads dY again -- and for the MLP's first projection, whose bias is added by the fused
# bias-GeLU, that GeLU's backward becomes a pure elementwise pass (ops/gelu.py bias_grad).
# Two kernel modes (csrc/kernels/wgrad.hip): when the input width K leaves a wave column of the
# last 256-wide output tile idle (K % 256 in [1, 192] -- every GPT-2 XL layer but fc2, K = 1600)
# that wave sums dY on the matrix core (B fragment = ones): no cost on the busy SIMDs, so it is
# always fused.  Otherwise the sums would go through LDS inside the round-4 kernel's MFMA loop
# (the ping-pong kernel has no such mode), and forcing that kernel for the fused sums loses to
# the table's pick plus a separate column-sum pass on the wide config 3 / 4 shapes (round 5,
# tools/gpu_r5wb.sh: GPT-NeoX PP2xTP4 shard 263.0 / 265.7 vs 274.2 / 274.1 ms per step, GPT-J
# TP4 shard 160.9 / 160.3 vs 162.2 / 163.1), so only the idle-wave mode is fused.
# SMP_WGRAD_DBIAS=0 turns the fused bias sums off (separate column-sum pass); =wide restores the
# round-4 LDS mode for dY of >= 4096 columns.
_WGRAD_DBIAS = os.environ.get("SMP_WGRAD_DBIAS", "1") != "0"
_WGRAD_DBIAS_MIN_N = 4096 if os.environ.get("SMP_WGRAD_DBIAS", "1") == "wide" else 1 << 62


def _wgrad_dbias_free(k):
    """A wave column of the weight-gradient kernel idles in the last K tile for input width ``k``
    and sums the bias gradient there at no cost: worth forcing the kernel over a faster library
    pick (it saves the separate full read of dY)."""
    return 0 < k % 256 <= 192


def _wgrad_dbias_rowsum(k):
    """Any other ``k``: the ping-pong kernel can sum the bias gradient with two extra MFMAs per
    wave in two of each tile's four phases of the last K tile's workgroups (CS mode 2).  Opt-in
    (SMP_WGRAD_PP_CS=rowsum): in the GPT-2 XL step its fc2 weight gradient (K = 6400) ran 1369.9 us
    against 1275 us + a 40 us column-sum pass without it (`profiles/r6/wgrad_rowsum_bias.md`)."""
    return os.environ.get("SMP_WGRAD_PP_CS") == "rowsum" and os.environ.get("SMP_WGRAD_IMPL") != "glds"


def _wgrad_accumulate(g, dy2, x2, dbias=None):
    """g += dy2^T x2 with the weight-gradient algorithm chosen for this shape.  ``dbias``: a
    tensor to accumulate the column sums of dy2 into from the same kernel pass; returns True
    when that happened (False: the caller computes them)."""
    if _wgrad_native_ok(g, dy2, x2):
        s = _wgrad_kernel_splits(g, dy2, x2)
        cheap = _wgrad_dbias_free(x2.shape[1]) or dy2.shape[1] >= _WGRAD_DBIAS_MIN_N
        fuse = (dbias is not None and _WGRAD_DBIAS and dy2.dtype == torch.bfloat16
                and (cheap or (s != 0 and _wgrad_dbias_rowsum(x2.shape[1]))))
        if fuse and s == 0:
            # the fused bias pass makes the kernel the cheaper choice (it saves a full read of dY)
            s = _wgrad_dbias_splits(dy2, x2)
        if s != 0:
            from ._ext import ext

            ext().wgrad_(g, dy2, x2, True, max(s, 0), dbias if fuse else None, True)
            return fuse
    g.addmm_(dy2.t(), x2)
    return False


def _wgrad_dbias_splits(dy2, x2):
    """Kernel split count for a shape whose timed pick was the library GEMM (the fused bias
    pass is not part of that timing): the fastest kernel count measured, or the static table."""
    key = (dy2.shape[0], dy2.shape[1], x2.shape[1])
    hit = _WGRAD_KERNEL_SPLIT_BEST.get(key)
    if hit:
        return hit
    k = (dy2.shape[1], x2.shape[1])
    return _WGRAD_STATIC.get(k, 0) or _WGRAD_STATIC_KERNEL.get(k, -1)


def _fusable(w):
    g = w.grad
    return (getattr(w, "_smp_fused_grad", False) and g is not None and g.dtype == w.dtype and g.shape == w.shape
            and g.is_contiguous())


# SMP_TRACE_TP_OVERLAP=1 records the backward's order of (dX all-reduce start, weight
# gradient, dX all-reduce wait) -- tests check that the weight gradient runs while the
# tensor-parallel all-reduce of the input gradient is in flight
TRACE_TP_OVERLAP = os.environ.get("SMP_TRACE_TP_OVERLAP", "0") == "1"
TP_OVERLAP_TRACE = []


# Token-chunked TP all-reduce overlap (reference row-parallel forward
# all-reduce `torch/nn/transformer.py:1515-1522`, column-parallel backward `:1134-1141`): under
# scaled-batch TP a row-parallel output is [B s, h] with a large B, so its GEMM is split into
# token chunks and chunk i's all-reduce runs on RCCL's stream while chunk i + 1's GEMM runs; the
# column-parallel input gradient likewise (each chunk's all-reduce starts right after its dX
# GEMM, the weight gradient follows, then the waits).  SMP_TP_AR_CHUNKS: chunk count (default:
# 4 from 16384 tokens, 2 from 4096, else 1 = one all-reduce).
_TP_AR_CHUNKS = os.environ.get("SMP_TP_AR_CHUNKS", "auto")


def tp_ar_chunks(tokens):
    if _TP_AR_CHUNKS != "auto":
        return max(1, int(_TP_AR_CHUNKS))
    return 4 if tokens >= 16384 else (2 if tokens >= 4096 else 1)


def _chunk_bounds(T, n):
    step = -(-T // n)
    step = -(-step // 16) * 16  # 16-row aligned chunks
    return [(a, min(T, a + step)) for a in range(0, T, step)]


def _chunked_fwd_allreduce(x, weight, bias, chunks, fwd_ar):
    """out = all-reduce(x W^T + b) with the GEMM and the all-reduce overlapped per token chunk."""
    x2 = x.reshape(-1, x.shape[-1])
    T = x2.shape[0]
    out = torch.empty(T, weight.shape[0], dtype=x.dtype, device=x.device)
    works = []
    wt = weight.t()
    for a, b in _chunk_bounds(T, chunks):
        if bias is not None:
            torch.addmm(bias, x2[a:b], wt, out=out[a:b])
        else:
            torch.mm(x2[a:b], wt, out=out[a:b])
        works.append(fwd_ar(out[a:b]))
        if TRACE_TP_OVERLAP:
            TP_OVERLAP_TRACE.append("fwd_chunk")
    from ..parallel.comm_timer import timer as _comm_timer

    with _comm_timer.region("tp", x.device):
        for w in works:
            if w is not None:
                w.wait()
    return out.view(*x.shape[:-1], weight.shape[0])


class _LinearWGradAccum(torch.autograd.Function):
    """y = x W^T + b with (a) the weight gradient accumulated by a GEMM straight into the
    flat gradient buffer, (b) the bias gradient -- of ``b`` or of ``dbias_of``, a bias that a
    fused activation adds downstream -- summed by the weight-gradient kernel in the same pass
    over dY when that kernel runs, and (c) optionally the tensor-parallel all-reduce of the input
    gradient (column-parallel layer of the speed mode; reference `nn/utils.py:548-570`
    BackwardAllreduceForTP) issued asynchronously right after dX and waited for only after
    the weight-gradient GEMM, so the two overlap."""

    @staticmethod
    def forward(ctx, x, weight, bias, dx_allreduce=None, dbias_of=None, fwd_ar=None):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias = bias
        ctx.dbias_of = dbias_of
        ctx.dx_allreduce = dx_allreduce
        ctx.wt = _transposed(weight) if _use_transposed(weight) else None
        if fwd_ar is not None:
            # row-parallel layer: the output leaves already all-reduced over TP (the all-reduce
            # has an identity backward, so the backward below is unchanged)
            n = tp_ar_chunks(x.numel() // x.shape[-1])
            if n > 1:
                return _chunked_fwd_allreduce(x, weight, bias, n, fwd_ar)
            out = F.linear(x, weight, bias)
            w = fwd_ar(out)
            if w is not None:
                w.wait()
            return out
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        if dy.dtype != w.dtype or x.dtype != w.dtype:
            # forward under torch.autocast (the GEMM ran in the autocast dtype, the inputs were
            # saved as given): the backward runs in the parameters' dtype, and autograd casts dX
            # back to the input's dtype
            dy, x = dy.to(w.dtype), x.to(w.dtype)
        dx = dw = None
        grads = {2: None, 4: None}  # input index -> gradient returned to autograd
        dy2 = dy.reshape(-1, dy.shape[-1])
        works = []
        if ctx.needs_input_grad[0]:
            n = tp_ar_chunks(dy2.shape[0]) if ctx.dx_allreduce is not None else 1
            if n > 1:
                # column-parallel dX in token chunks: each chunk's all-reduce starts right after
                # its GEMM (a fresh tensor, reduced in place), overlapping the next chunk's GEMM
                # and then the weight gradient
                wm = ctx.wt.t() if ctx.wt is not None else w
                dx2 = torch.empty(dy2.shape[0], wm.shape[1], dtype=dy.dtype, device=dy.device)
                for a, b in _chunk_bounds(dy2.shape[0], n):
                    if ctx.wt is not None:
                        torch.mm(dy2[a:b], ctx.wt.t(), out=dx2[a:b])
                    else:
                        torch.mm(dy2[a:b], w, out=dx2[a:b])
                    works.append(ctx.dx_allreduce(dx2[a:b]))
                    if TRACE_TP_OVERLAP:
                        TP_OVERLAP_TRACE.append("dx_allreduce_start")
                dx = dx2.view(*dy.shape[:-1], wm.shape[1])
            else:
                dx = F.linear(dy, ctx.wt) if ctx.wt is not None else torch.matmul(dy, w)
                if ctx.dx_allreduce is not None:
                    works.append(ctx.dx_allreduce(dx))  # fresh tensor: reduced in place, async when large
                    if TRACE_TP_OVERLAP:
                        TP_OVERLAP_TRACE.append("dx_allreduce_start")
        # the bias whose gradient is colsum(dY): this layer's own, or the downstream one
        bidx = 2 if (ctx.has_bias and ctx.needs_input_grad[2]) else (
            4 if (ctx.dbias_of is not None and ctx.needs_input_grad[4]) else None)
        bparam = None if bidx is None else (ctx.bias if bidx == 2 else ctx.dbias_of)
        # fused target: the bound flat-buffer view (accumulated in place), else a fresh fp32 sum
        btarget = None
        if bparam is not None and dy2.is_cuda:
            btarget = bparam.grad if _fusable(bparam) else torch.zeros(bparam.shape, dtype=torch.float32,
                                                                        device=dy2.device)
        bdone = False
        if ctx.needs_input_grad[1]:
            if _fusable(w):
                # beta = 1 GEMM into the bound flat-buffer view; returning None still runs the
                # weight's AccumulateGrad node (a no-op), so post-accumulate-grad hooks -- the
                # reducers' bucket-ready signals -- fire exactly once, after this write
                bdone = _wgrad_accumulate(w.grad, dy2, x.reshape(-1, x.shape[-1]), dbias=btarget)
            else:
                # grad slot re-bound/removed since forward: hand the gradient to autograd
                dw = dy2.t().mm(x.reshape(-1, x.shape[-1]))
            if TRACE_TP_OVERLAP:
                TP_OVERLAP_TRACE.append("wgrad")
        if bparam is not None:
            if not bdone:
                if btarget is not None and btarget is bparam.grad:
                    _col_sum(dy2, btarget)  # into the bound flat-buffer view (no temp + add)
                else:
                    btarget = _col_sum(dy2)
            if btarget is not bparam.grad:
                grads[bidx] = btarget.to(bparam.dtype)
        if any(wk is not None for wk in works):
            from ..parallel.comm_timer import timer as _comm_timer

            with _comm_timer.region("tp", dy.device):
                for wk in works:
                    if wk is not None:
                        wk.wait()
        if works and TRACE_TP_OVERLAP:
            TP_OVERLAP_TRACE.append("dx_allreduce_wait")
        return dx, dw, grads[2], None, grads[4], None


def linear(x, weight, bias=None, dx_allreduce=None, dbias_of=None, fwd_ar=None):
    """F.linear with GEMM-fused weight-gradient accumulation into the flat grad buffer.
    ``dx_allreduce(dx) -> work | None``: the column-parallel layer's input-gradient
    all-reduce, overlapped with the weight-gradient GEMM (the caller then applies no
    separate backward all-reduce to x).  ``dbias_of``: a bias added to this layer's output
    by a fused activation that leaves its gradient to this layer (``bias_gelu(...,
    bias_grad=False)``): its gradient, the token sum of dY, is returned here -- from the
    weight-gradient kernel's own pass over dY when that kernel runs.  ``fwd_ar(out) -> work |
    None``: the row-parallel layer's forward all-reduce, applied here in token chunks
    overlapped with the GEMM (the output is returned reduced)."""
    if torch.is_grad_enabled() and (dbias_of is not None or dx_allreduce is not None or fwd_ar is not None) and (
            weight.requires_grad or x.requires_grad or (dbias_of is not None and dbias_of.requires_grad)):
        return _LinearWGradAccum.apply(x, weight, bias, dx_allreduce, dbias_of, fwd_ar)
    if torch.is_grad_enabled() and weight.requires_grad and _fusable(weight):
        return _LinearWGradAccum.apply(x, weight, bias, None, None, None)
    if fwd_ar is not None:  # no gradient needed: the chunked, reduced output alone
        n = tp_ar_chunks(x.numel() // x.shape[-1])
        if n > 1:
            return _chunked_fwd_allreduce(x, weight, bias, n, fwd_ar)
        out = F.linear(x, weight, bias)
        w = fwd_ar(out)
        if w is not None:
            w.wait()
        return out
    return F.linear(x, weight, bias)
