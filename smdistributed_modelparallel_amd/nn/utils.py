"""Tensor-parallel building blocks: channel splits, parameter scopes and the autograd
collectives used by the distributed modules.

Reference parity (`smp/torch/nn/utils.py:45-844`):
* ``get_local_channels(n)``: the first ``n % tp`` ranks get one extra channel;
  ``get_start_pos_for_slicing`` gives each rank's offset (uneven splits supported);
* collectives with forward/backward pairs: all-reduce (f/g), all-gather <-> narrow,
  reduce-scatter <-> all-gather, all-to-all (scatter-and-merge), sequence shard/unshard;
  uneven splits are padded to the largest shard for RCCL and un-padded after;
* ``mark_scaled_batch`` / ``mark_tp`` tag parameters of distributed modules (scaled-batch
  and their TP split layout) and ``init_weight_`` initialises a shard *as if unsharded*
  (fan-in of the full layer, or N(0, initializer_range)).

With tp_size == 1 every collective is an identity (no RCCL calls).
"""
import math

import torch
import torch.distributed as dist

from ..torch.state_mod import state
from ..ops.pack import strided_copy_
from ..parallel.throttle import throttler
from ..parallel import oneshot
from ..parallel.comm_timer import timer as _comm_timer


# --------------------------------------------------------------------- topology
def tp_size():
    return state.core.tp_size() if state.initialized else 1


def tp_rank():
    return state.core.tp_rank() if state.initialized else 0


def tp_group():
    return state.pgs.tp if state.initialized else None


def get_local_channels(num_channels, rank=None):
    size = tp_size()
    rank = tp_rank() if rank is None else rank
    base, rem = divmod(num_channels, size)
    return base + (1 if rank < rem else 0)


def get_start_pos_for_slicing(num_channels, rank=None):
    rank = tp_rank() if rank is None else rank
    return sum(get_local_channels(num_channels, r) for r in range(rank))


def get_merge_shapes(num_channels):
    return [get_local_channels(num_channels, r) for r in range(tp_size())]


# -------------------------------------------------------------- raw collectives
# RCCL's all-gather / reduce-scatter / all-to-all move whole [rank, rows, ...] blocks; a
# shard of dim `dim` is moved between its tensor layout and that block layout by ONE
# strided HIP copy (ops/pack.py, K21) -- uneven shards are padded to the largest one, the
# padding rows are never initialised (the receiver drops them).
def _split3(x, dim):
    """View x as [A, x.size(dim), B] (A = prod of leading dims, B = of trailing)."""
    A = 1
    for n in x.shape[:dim]:
        A *= n
    return x.reshape(A, x.size(dim), -1)


def _allgather(x, dim, sizes=None):
    """Concatenate every TP rank's x along dim (uneven sizes allowed)."""
    ws = tp_size()
    if ws == 1:
        return x
    group = tp_group()
    x = x.contiguous()
    if sizes is None:
        sizes = [x.size(dim)] * ws
    mx = max(sizes)
    even = all(n == mx for n in sizes)
    out_shape = list(x.shape)
    out_shape[dim] = sum(sizes)
    if dim == 0 and even:  # rank blocks are already the final layout
        out = x.new_empty(out_shape)
        with throttler().throttle(x), _comm_timer.region("tp", x.device):
            dist.all_gather_into_tensor(out, x, group=group)
        return out
    x3 = _split3(x, dim)  # [A, n, B]
    A, B = x3.shape[0], x3.shape[2]
    send = x.new_empty((mx, A, B))
    strided_copy_(send[: x3.shape[1]], x3.permute(1, 0, 2))
    recv = x.new_empty((ws, mx, A, B))
    with throttler().throttle(send), _comm_timer.region("tp", send.device):
        dist.all_gather_into_tensor(recv.view(ws * mx, A, B), send, group=group)
    out = x.new_empty(out_shape)
    o3 = out.view(A, sum(sizes), B)
    if even:
        strided_copy_(o3.view(A, ws, mx, B).permute(1, 2, 0, 3), recv)
    else:
        off = 0
        for r, n in enumerate(sizes):
            strided_copy_(o3[:, off:off + n].permute(1, 0, 2), recv[r, :n])
            off += n
    return out


def _reduce_scatter(x, dim, sizes=None):
    """Sum over TP ranks, keep this rank's slice along dim."""
    ws = tp_size()
    if ws == 1:
        return x
    group = tp_group()
    if sizes is None:
        assert x.size(dim) % ws == 0, "reduce_scatter requires divisible size or explicit sizes"
        sizes = [x.size(dim) // ws] * ws
    mx = max(sizes)
    even = all(n == mx for n in sizes)
    me = tp_rank()
    out_shape = list(x.shape)
    out_shape[dim] = sizes[me]
    if dim == 0 and even:
        x = x.contiguous()
        out = x.new_empty(out_shape)
        with throttler().throttle(x), _comm_timer.region("tp", x.device):
            dist.reduce_scatter_tensor(out, x, group=group)
        return out
    x3 = _split3(x, dim)
    A, B = x3.shape[0], x3.shape[2]
    inp = x.new_empty((ws, mx, A, B))
    if even:
        strided_copy_(inp, x3.view(A, ws, mx, B).permute(1, 2, 0, 3))
    else:
        off = 0
        for r, n in enumerate(sizes):
            strided_copy_(inp[r, :n], x3[:, off:off + n].permute(1, 0, 2))
            off += n
    red = x.new_empty((mx, A, B))
    with throttler().throttle(inp), _comm_timer.region("tp", inp.device):
        dist.reduce_scatter_tensor(red, inp.view(ws * mx, A, B), group=group)
    out = x.new_empty(out_shape)
    strided_copy_(out.view(A, sizes[me], B).permute(1, 0, 2), red[: sizes[me]])
    return out


def _allreduce(x, inplace=False):
    """Sum over the TP group.  inplace=False leaves x untouched (a copy is reduced); the
    autograd wrappers pass inplace=True where x is a dead temporary (a GEMM output or a
    gradient nobody else reads), saving a full-size copy per call."""
    if tp_size() == 1:
        return x
    if not inplace or not x.is_contiguous():
        x = x.clone(memory_format=torch.contiguous_format)
    with throttler().throttle(x), _comm_timer.region("tp", x.device):
        oneshot.all_reduce(x, group=tp_group())
    return x


def _narrow(x, dim, sizes=None):
    ws = tp_size()
    if ws == 1:
        return x
    if sizes is None:
        n = x.size(dim) // ws
        return x.narrow(dim, tp_rank() * n, n).contiguous()
    start = sum(sizes[: tp_rank()])
    return x.narrow(dim, start, sizes[tp_rank()]).contiguous()


def _all_to_all(x, split_dim, merge_dim, split_sizes=None, merge_sizes=None):
    """Split x along split_dim into tp pieces (piece r -> rank r); concatenate received
    pieces along merge_dim (uneven merge sizes allowed) -- `scatter_and_merge`."""
    ws = tp_size()
    if ws == 1:
        return x
    if split_sizes is None:
        split_sizes = [x.size(split_dim) // ws] * ws
    me = tp_rank()
    pieces = list(x.split(split_sizes, dim=split_dim))
    out_shapes = []
    for r in range(ws):
        s = list(pieces[me].shape)
        s[merge_dim] = merge_sizes[r] if merge_sizes is not None else x.size(merge_dim)
        out_shapes.append(s)
    group = tp_group()
    out_shape = list(out_shapes[0])
    out_shape[merge_dim] = sum(s[merge_dim] for s in out_shapes)
    if x.is_cuda:
        # one flat send buffer (pieces packed back to back) and one flat receive buffer:
        # a single RCCL all-to-all over xGMI with per-rank element counts
        numels = [p.numel() for p in pieces]
        send = x.new_empty(sum(numels))
        off = 0
        for p, n in zip(pieces, numels):
            strided_copy_(send[off:off + n].view(p.shape), p)
            off += n
        rn = [int(torch.Size(s).numel()) for s in out_shapes]
        recv = x.new_empty(sum(rn))
        with throttler().throttle(x), _comm_timer.region("tp", x.device):
            dist.all_to_all_single(recv, send, output_split_sizes=rn, input_split_sizes=numels, group=group)
        out = x.new_empty(out_shape)
        off, moff = 0, 0
        for s, n in zip(out_shapes, rn):
            strided_copy_(out.narrow(merge_dim, moff, s[merge_dim]), recv[off:off + n].view(s))
            off += n
            moff += s[merge_dim]
        return out
    # gloo has no all-to-all: pairwise exchange
    pieces = [p.contiguous() for p in pieces]
    outs = [x.new_empty(s) for s in out_shapes]
    ops = []
    for r in range(ws):
        if r == me:
            outs[r].copy_(pieces[r])
            continue
        peer = dist.get_global_rank(group, r)
        ops.append(dist.P2POp(dist.isend, pieces[r], peer, group))
        ops.append(dist.P2POp(dist.irecv, outs[r], peer, group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return torch.cat(outs, dim=merge_dim)


# ------------------------------------------------------------ autograd wrappers
class _FwdAllreduce(torch.autograd.Function):
    """fwd all-reduce (in place on x when the caller marks it a dead temporary, e.g. the
    row-parallel GEMM output -- no autograd node saves it); bwd identity."""

    @staticmethod
    def forward(ctx, x, inplace):
        if inplace and tp_size() > 1 and x.is_contiguous():
            # x is often a view returned by the GEMM Function (mark_dirty is forbidden there);
            # its data is reduced in place behind autograd's back -- safe because no node
            # saved x -- and a view of it is the output
            _allreduce(x.detach(), inplace=True)
            return x.view_as(x)
        return _allreduce(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _BwdAllreduce(torch.autograd.Function):
    """fwd identity; bwd all-reduce, in place when the caller guarantees the incoming
    gradient is a fresh tensor (the dgrad of the column-parallel GEMM that consumes x)."""

    @staticmethod
    def forward(ctx, x, inplace):
        ctx.inplace = inplace
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _allreduce(g, inplace=ctx.inplace), None


def dx_allreduce_async(dx):
    """Input-gradient all-reduce of a column-parallel layer, started without waiting (the
    layer's backward runs its weight-gradient GEMM, then waits).  dx is a fresh gradient:
    reduced in place."""
    if tp_size() == 1:
        return None
    if not dx.is_contiguous():
        raise RuntimeError("dx_allreduce_async: the input gradient must be contiguous")
    return oneshot.all_reduce(dx, group=tp_group(), async_op=True)


def fwd_allreduce_async(out):
    """Forward all-reduce of a row-parallel output chunk (ops.linear's token-chunked path):
    started without waiting -- the caller waits after issuing the next chunk's GEMM.  ``out``
    is a fresh GEMM output chunk: reduced in place.  Returns the work handle (None when the
    one-shot kernel ran: it is already ordered on the current stream)."""
    if tp_size() == 1:
        return None
    with throttler().throttle(out):
        return oneshot.all_reduce(out, group=tp_group(), async_op=True)


class _Allgather(torch.autograd.Function):
    """fwd all-gather along dim; bwd narrow (each rank keeps its own slice)."""

    @staticmethod
    def forward(ctx, x, dim, sizes):
        ctx.dim, ctx.sizes = dim, sizes
        return _allgather(x, dim, sizes)

    @staticmethod
    def backward(ctx, g):
        return _narrow(g, ctx.dim, ctx.sizes), None, None


class _FusedAllgather(torch.autograd.Function):
    """fwd all-gather; bwd reduce-scatter (the gathered tensor feeds rank-local math)."""

    @staticmethod
    def forward(ctx, x, dim, sizes):
        ctx.dim, ctx.sizes = dim, sizes
        return _allgather(x, dim, sizes)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter(g, ctx.dim, ctx.sizes), None, None


class _Narrow(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, sizes):
        ctx.dim, ctx.sizes = dim, sizes
        return _narrow(x, dim, sizes)

    @staticmethod
    def backward(ctx, g):
        return _allgather(g, ctx.dim, ctx.sizes), None, None


class _ReduceScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dim, sizes):
        ctx.dim, ctx.sizes = dim, sizes
        return _reduce_scatter(x, dim, sizes)

    @staticmethod
    def backward(ctx, g):
        return _allgather(g, ctx.dim, ctx.sizes), None, None


class _ScatterAndMerge(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, split_dim, merge_dim, split_sizes, merge_sizes):
        ctx.args = (split_dim, merge_dim, split_sizes, merge_sizes)
        ctx.in_merge = x.size(merge_dim)
        return _all_to_all(x, split_dim, merge_dim, split_sizes, merge_sizes)

    @staticmethod
    def backward(ctx, g):
        split_dim, merge_dim, split_sizes, merge_sizes = ctx.args
        # reverse: split along merge_dim by merge_sizes, merge along split_dim by split_sizes
        back = _all_to_all(g, merge_dim, split_dim, merge_sizes, split_sizes)
        return back, None, None, None, None


def fwd_allreduce_for_tp(x, inplace=False):
    """All-reduce in the forward (identity backward).  inplace=True: x is a dead temporary
    (a row-parallel GEMM output) and is reduced in place -- no copy."""
    return _FwdAllreduce.apply(x, inplace) if tp_size() > 1 else x


def bwd_allreduce_for_tp(x, inplace_grad=False):
    """Identity forward, all-reduce of the gradient.  inplace_grad=True: the consumer of the
    output is a column-parallel GEMM whose dgrad is a fresh tensor -- reduced in place."""
    return _BwdAllreduce.apply(x, inplace_grad) if tp_size() > 1 else x


def allgather_for_tp(x, dim, sizes=None):
    return _Allgather.apply(x, dim, sizes) if tp_size() > 1 else x


def fused_allgather_for_tp(x, dim, merge_shapes=None):
    return _FusedAllgather.apply(x, dim, merge_shapes) if tp_size() > 1 else x


def narrow_for_tp(x, dim, sizes=None):
    return _Narrow.apply(x, dim, sizes) if tp_size() > 1 else x


def reduce_scatter_for_tp(x, dim, split_shapes=None):
    return _ReduceScatter.apply(x, dim, split_shapes) if tp_size() > 1 else x


def scatter_and_merge_for_tp(x, split_dim, merge_dim, split_shapes=None, merge_shapes=None):
    return _ScatterAndMerge.apply(x, split_dim, merge_dim, split_shapes, merge_shapes) if tp_size() > 1 else x


def shard_sequence(*tensors, dim=1, shift=0, bwd_allgather=True):
    """prescaled_batch: keep this rank's contiguous chunk of the sequence dimension."""
    if tp_size() == 1:
        return tensors
    out = []
    for t in tensors:
        if t is None:
            out.append(None)
            continue
        sizes = get_merge_shapes(t.size(dim))
        if bwd_allgather and t.requires_grad:
            out.append(narrow_for_tp(t, dim, sizes))
        else:
            out.append(_narrow(t, dim, sizes))
    return tuple(out)


def unshard_sequence(seq_length, *tensors, dim=1):
    if tp_size() == 1:
        return tensors
    sizes = get_merge_shapes(seq_length)
    return tuple(allgather_for_tp(t, dim, sizes) if t is not None else None for t in tensors)


# ---------------------------------------------------------- parameter creation
def mark_scaled_batch(param, scaled=True):
    param._smp_scaled_batch = scaled
    param._smp_distributed = True
    return param


def is_scaled_batch(param):
    return getattr(param, "_smp_scaled_batch", False)


def mark_tp(param, axis, groups=1, rank0_only=False, unit=1):
    """Record how a parameter is split across the TP group, for checkpoint merge/slice:
    `axis` the sharded dim (None = replicated), `groups` > 1 when the full tensor is
    `groups` concatenated blocks each sharded separately (fused QKV), `rank0_only` for
    row-parallel biases that exist only on tp_rank 0, `unit` the split granularity
    (head_dim for attention projections: heads are split, not rows)."""
    param._smp_tp_axis = axis
    param._smp_tp_groups = groups
    param._smp_tp_rank0_only = rank0_only
    param._smp_tp_unit = unit
    return param


def init_weight_(w, full_in, full_out, initializer_range=0.02, use_normal=False):
    """Initialise a (possibly sharded) [out, in] weight as nn.Linear of the full shape."""
    with torch.no_grad():
        if use_normal:
            w.normal_(0.0, initializer_range)
        else:
            bound = 1.0 / math.sqrt(full_in) if full_in > 0 else 0.0
            # kaiming_uniform(a=sqrt(5)) on the full layer == U(-1/sqrt(fan_in), 1/sqrt(fan_in))
            w.uniform_(-bound, bound)
    return w
