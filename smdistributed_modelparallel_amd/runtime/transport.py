"""Pipeline data plane.

Replaces the reference's D2D engine + listener (N1c/N1d, `smp/torch/server_comm.py`,
`smp/torch/ops.py:42-123`) with:

* control messages (pickled, tensors stubbed) on the native mailbox SERVER channel;
* CPU tensors embedded in the control message (gloo/CPU runs);
* GPU tensors over RCCL point-to-point.  Each *directed* stage pair owns its own RCCL
  communicator, so a communicator only ever carries traffic in one direction:
  sends and receives on it are matched FIFO, and a send in one direction can never be
  stuck behind a receive in the other (the classic rendezvous deadlock of a shared
  bidirectional P2P stream).  The receiver posts its irecvs in control-message order,
  which is the sender's isend order (mailbox links are FIFO per pair).
* completion is stream-ordered: the receiver's compute stream waits on the RCCL
  event (``work.wait()``), the host never blocks.
"""
import torch
import torch.distributed as dist

from ..backend.collectives import SERVER_CHANNEL, dumps, loads


class PipelineTransport:
    def __init__(self, core, pgs, device):
        self.mailbox = core.mailbox
        self.rank = core.rank()
        self.pgs = pgs
        self.device = device
        self._inflight = []
        self.bytes_sent = 0
        self.bytes_recv = 0

    def warmup(self, pp_group_ranks):
        """Initialise every directed RCCL communicator in one global order (no deadlock on
        lazy communicator creation)."""
        if self.device.type != "cuda":
            return
        for a in pp_group_ranks:
            for b in pp_group_ranks:
                if a == b or self.rank not in (a, b):
                    continue
                g = self.pgs.p2p[(a, b)]
                t = torch.zeros(1, device=self.device)
                if self.rank == a:
                    dist.send(t, b, group=g)
                else:
                    dist.recv(t, a, group=g)
        torch.cuda.synchronize(self.device)

    def _prune(self):
        if self._inflight:
            self._inflight = [(w, t) for (w, t) in self._inflight if not w.is_completed()]

    def send(self, dst, stubbed, tensors):
        meta, cpu = [], []
        gpu = []
        for t in tensors:
            if t.is_cuda:
                meta.append((tuple(t.shape), t.dtype, True))
                cpu.append(None)
                gpu.append(t)
            else:
                meta.append((tuple(t.shape), t.dtype, False))
                cpu.append(t.detach())
        self.mailbox.send(dst, 0, SERVER_CHANNEL, dumps((stubbed, meta, cpu)))
        if gpu:
            g = self.pgs.p2p[(self.rank, dst)]
            for t in gpu:
                t = t.detach().contiguous()
                self.bytes_sent += t.numel() * t.element_size()
                self._inflight.append((dist.isend(t, dst, group=g), t))
        self._prune()

    def poll(self, timeout):
        """Returns (src, stubbed, tensors) or None."""
        r = self.mailbox.next_server_message(timeout)
        if r is None:
            return None
        src, _tid, payload = r
        stubbed, meta, cpu = loads(payload)
        tensors = []
        for (shape, dtype, is_gpu), c in zip(meta, cpu):
            if not is_gpu:
                tensors.append(c)
                continue
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            w = dist.irecv(buf, src, group=self.pgs.p2p[(src, self.rank)])
            w.wait()  # stream-ordered: compute stream waits for the RCCL event
            self.bytes_recv += buf.numel() * buf.element_size()
            tensors.append(buf)
        return src, stubbed, tensors

    def has_message(self):
        return self.mailbox.has_server_message()

    def drain(self):
        for w, _ in self._inflight:
            w.wait()
        self._inflight.clear()
