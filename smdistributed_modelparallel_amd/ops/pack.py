"""Strided pack / unpack for the TP collectives (K21, `csrc/kernels/pack.hip`).

``strided_copy_(dst, src)`` copies between two same-shape views with arbitrary strides in
one HIP kernel.  Dims are collapsed first (adjacent dims that are contiguous with each
other in BOTH views merge), so e.g. a movedim + narrow + pad becomes one <= 4-D copy.
CPU tensors use ``Tensor.copy_`` (the gloo test target)."""
import torch

from ._ext import ext


def _collapse(shape, s_strides, d_strides):
    dims = [(n, a, b) for n, a, b in zip(shape, s_strides, d_strides) if n != 1]
    if not dims:
        return [1], [0], [0]
    out = [list(dims[0])]
    for n, a, b in dims[1:]:
        pn, pa, pb = out[-1]
        if pa == n * a and pb == n * b:  # previous dim steps over exactly this one in both
            out[-1] = [pn * n, a, b]
        else:
            out.append([n, a, b])
    return [d[0] for d in out], [d[1] for d in out], [d[2] for d in out]


def strided_copy_(dst, src):
    """dst[...] = src[...] (same shape, any strides). Returns dst."""
    if dst.shape != src.shape:
        raise ValueError(f"strided_copy_: shape mismatch {tuple(dst.shape)} vs {tuple(src.shape)}")
    if dst.numel() == 0:
        return dst
    if not dst.is_cuda:
        return dst.copy_(src)
    shape, ss, ds = _collapse(list(dst.shape), list(src.stride()), list(dst.stride()))
    if len(shape) > 4:
        # rare (> 4 non-mergeable dims): split the outermost dim
        for i in range(dst.shape[0]):
            strided_copy_(dst[i], src[i])
        return dst
    d = torch.as_strided(dst, shape, ds)
    s = torch.as_strided(src, shape, ss)
    ext().strided_copy_(d, s)
    return dst
