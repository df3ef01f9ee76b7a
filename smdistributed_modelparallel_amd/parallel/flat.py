"""Flat parameter / gradient storage.

MI355X-first memory layout: all trainable local parameters of one (dtype, reduction
group) live in ONE contiguous HBM buffer and every ``param.data`` / ``param.grad`` is a
view into it.  This gives:

* gradient buckets that are plain contiguous slices (no flatten/unflatten copies before
  each RCCL all-reduce -- the reference's ``gradient_as_bucket_view``, N1f);
* an optimizer step that is one fused HIP kernel per contiguous range instead of
  thousands of per-tensor launches (K14);
* optimizer-state sharding (ZeRO-1) where each rank owns chunk ``r`` of every bucket, so
  reduce-scatter / all-gather run directly on the bucket slices (`model.py:1237-1340`
  semantics without the reference's virtual-parameter copies).

Layout: parameters are grouped into *segments* (one per optimizer param group when the
optimizer is known); inside a segment they are stored in reverse registration order so
the first bucket covers the last layers, whose gradients are produced first in backward.
Every parameter starts at a multiple of 64 elements; each bucket is padded to a multiple of ``align`` elements (the data-parallel degree x 64)
so reduce-scatter chunks are equal and 128-byte aligned.
"""
import torch

# every parameter starts on a 128-byte boundary (bf16): kernels may use 16-byte vector
# loads on any parameter view
_PARAM_ALIGN = 64


class Bucket:
    __slots__ = ("index", "start", "end", "params", "ready", "work", "launched")

    def __init__(self, index, start, end, params):
        self.index = index
        self.start = start
        self.end = end
        self.params = params
        self.ready = 0
        self.work = None
        self.launched = False

    @property
    def numel(self):
        return self.end - self.start


class FlatParamGroup:
    def __init__(self, named_params, device, dtype, bucket_cap_bytes, first_bucket_bytes=None, align=64,
                 segments=None, grad_dtype=None):
        """named_params: list of (name, Parameter) in registration order.
        segments: optional list of lists of Parameters (optimizer groups) defining order."""
        self.device = device
        self.dtype = dtype
        self.grad_dtype = grad_dtype or dtype
        self.align = max(1, int(align))
        self.named = list(named_params)
        self.name_of = {p: n for n, p in self.named}
        params = [p for _, p in self.named]
        if segments is None:
            segments = [params]
        else:
            seen = set()
            segs = []
            for seg in segments:
                s = [p for p in seg if p in self.name_of and p not in seen]
                seen.update(s)
                if s:
                    segs.append(s)
            rest = [p for p in params if p not in seen]
            if rest:
                segs.append(rest)
            segments = segs
        reg_index = {p: i for i, p in enumerate(params)}
        self.segments = [sorted(seg, key=lambda p: -reg_index[p]) for seg in segments]

        esize = torch.empty((), dtype=dtype).element_size()
        cap = max(1, bucket_cap_bytes // esize)
        first_cap = max(1, (first_bucket_bytes or bucket_cap_bytes) // esize)

        self.offsets = {}
        self.buckets = []
        self.segment_ranges = []
        off = 0
        for seg in self.segments:
            seg_start = off
            cur, cur_start, cur_n = [], off, 0
            for p in seg:
                n = p.numel()
                limit = first_cap if not self.buckets else cap
                if cur and cur_n + n > limit:
                    off = self._close_bucket(cur, cur_start, off)
                    cur, cur_start, cur_n = [], off, 0
                off = (off + _PARAM_ALIGN - 1) // _PARAM_ALIGN * _PARAM_ALIGN
                self.offsets[p] = off
                off += n
                cur_n += n
                cur.append(p)
            if cur:
                off = self._close_bucket(cur, cur_start, off)
            self.segment_ranges.append((seg_start, off, seg))
        self.numel = off
        self.bucket_of = {p: b for b in self.buckets for p in b.params}

        self.data = torch.zeros(self.numel, dtype=dtype, device=device)
        self.grad = torch.zeros(self.numel, dtype=self.grad_dtype, device=device)
        with torch.no_grad():
            for p, o in self.offsets.items():
                n = p.numel()
                self.data[o : o + n].copy_(p.data.reshape(-1).to(device=device, dtype=dtype))
        self.bind()

    def _close_bucket(self, params, start, end):
        padded = start + ((end - start + self.align - 1) // self.align) * self.align
        self.buckets.append(Bucket(len(self.buckets), start, padded, list(params)))
        return padded

    def view(self, p, buf):
        o = self.offsets[p]
        return buf[o : o + p.numel()].view(p.shape)

    @property
    def fp32_accumulation(self):
        """Gradient buffer wider than the parameters (``_fp32_grad_accumulation``): each
        microbatch's low-precision gradient lands in ``param.grad`` and is folded into the
        fp32 ``param.main_grad`` view by the reducer's hook."""
        return self.grad_dtype != self.dtype

    def bind(self):
        """Point every param's .data and .grad (or .main_grad) at the flat buffers."""
        for p in self.offsets:
            p.data = self.view(p, self.data)
            if self.fp32_accumulation:
                p.grad = None
                p.main_grad = self.view(p, self.grad)
                p._smp_fused_grad = False
            else:
                p.grad = self.view(p, self.grad)
                p._smp_fused_grad = True  # ops.linear may accumulate dW straight into the view

    def fold_grad(self, p):
        """main_grad += grad (fp32 accumulation); frees the low-precision grad."""
        g = p.grad
        if g is not None:
            p.main_grad.add_(g)
            p.grad = None

    def rebind_grads(self):
        if self.fp32_accumulation:
            for p in self.offsets:
                self.fold_grad(p)
            return
        base, es = self.grad.data_ptr(), self.grad.element_size()
        for p, o in self.offsets.items():
            g = p.grad
            if g is None or g.data_ptr() != base + o * es:
                if g is not None:
                    # someone replaced the grad tensor: fold its value back into the buffer
                    self.view(p, self.grad).copy_(g)
                p.grad = self.view(p, self.grad)

    def zero_grad(self):
        self.grad.zero_()

    def params(self):
        return list(self.offsets.keys())
