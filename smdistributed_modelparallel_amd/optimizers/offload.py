"""Optimizer-state offload: fp32 master weights and moments in pinned host memory.

Sizing for 288 GB of HBM3E: with bf16 params + grads in HBM (4
B/param) and the 12 B/param of fp32 master/exp_avg/exp_avg_sq on the host, a GPU holds
~4x the parameters it could with all 16 B/param resident.  The fused optimizer kernel
still runs on the GPU: every domain (a gradient-bucket range of the flat buffers) is
streamed through one of two HBM staging slots --

    H2D stream : copy master/m/v of domain i+1 into slot (i+1)%2   (after slot's D2H done)
    compute    : fused update of domain i from slot i%2 (+ bf16 param write-back)
    D2H stream : copy slot i%2 back to the pinned host arrays

-- so PCIe transfers in both directions overlap the update of the neighbouring domain.
Completion is HIP-event ordered; host readers (checkpointing) call ``wait()``.  Same
kernels, same math: results are bitwise identical to the resident optimizer.
"""
import torch


class OptimizerStateOffload:
    def __init__(self, domains, device):
        self.device = device
        n = max((d.numel for d in domains), default=0)
        # the host-resident fields (SMP_OFFLOAD_OPTIMIZER_FIELDS); the rest stay in HBM
        fields = [k for k in ("master", "m", "v")
                  if domains and getattr(domains[0], k) is not None and not getattr(domains[0], k).is_cuda]
        self.fields = fields
        self.slots = [{k: torch.empty(n, dtype=torch.float32, device=device) for k in fields} for _ in range(2)]
        self.h2d = torch.cuda.Stream(device=device)
        self.d2h = torch.cuda.Stream(device=device)
        self._free = [None, None]  # event: slot's D2H finished
        self._last = []

    def _upload(self, d, slot):
        st = self.slots[slot]
        ev = torch.cuda.Event()
        with torch.cuda.stream(self.h2d):
            if self._free[slot] is not None:
                self.h2d.wait_event(self._free[slot])
            for k in self.fields:
                st[k][: d.numel].copy_(getattr(d, k), non_blocking=True)
            ev.record(self.h2d)
        return ev

    def run(self, domains, update):
        """update(domain, (master, m, v) staging views) runs the fused kernel on the
        current stream."""
        comp = torch.cuda.current_stream(self.device)
        if not domains:
            return
        up = {0: self._upload(domains[0], 0)}
        for i, d in enumerate(domains):
            slot = i % 2
            if i + 1 < len(domains):
                up[i + 1] = self._upload(domains[i + 1], 1 - slot)
            comp.wait_event(up.pop(i))
            st = self.slots[slot]
            views = tuple(st[k][: d.numel] if k in st else getattr(d, k) for k in ("master", "m", "v"))
            update(d, views)
            done = torch.cuda.Event()
            done.record(comp)
            free = torch.cuda.Event()
            with torch.cuda.stream(self.d2h):
                self.d2h.wait_event(done)
                for k in self.fields:
                    getattr(d, k).copy_(st[k][: d.numel], non_blocking=True)
                free.record(self.d2h)
            self._free[slot] = free
        # the next step's first upload waits on these; the compute stream need not
        self._last = [e for e in self._free if e is not None]

    def wait(self):
        for e in self._last:
            e.synchronize()
