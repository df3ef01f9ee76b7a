"""Pipeline data plane.

Replaces the reference's D2D engine + listener (N1c/N1d, `smp/torch/server_comm.py:30-353`,
`smp/torch/ops.py:42-123`): control messages are pickled (tensors stubbed) on the native
mailbox SERVER channel; tensor payloads travel by one of four paths:

* ``cpu``  -- CPU tensors embedded in the control message (gloo/CPU runs);
* ``ipc``  -- the default between GPU ranks of one node: the native ``IpcP2P`` engine
  (`csrc/torchrt/ipc_p2p.cpp`).  The sender publishes the caching-allocator segment that
  holds the tensor plus an inter-process HIP event recorded after the producer kernels;
  the receiver maps the segment once and, as soon as the control message arrives, enqueues
  event-wait + one D2D pull copy (xGMI between GPUs) on its compute stream.  Neither host
  blocks.  The receiver returns a release note (batched, out of band) once its copy has
  completed, and only then does the sender drop the source tensor and recycle the event
  slot.  Because the pull is posted on arrival of the metadata, every receive is
  effectively pre-posted; there is no receive pool to size or overflow.
* ``rccl`` -- RCCL point-to-point (multi-node, or ``SMP_P2P=rccl``).  Each *directed* stage
  pair owns its own communicator, so sends and receives on it are matched FIFO and a send
  in one direction can never sit behind a receive in the other; the receiver posts its
  irecvs in control-message order (mailbox links are FIFO per pair).
* ``host`` -- host-staged copies inside the control message (GPU ranks on a gloo-only
  process group, e.g. single-GPU multi-rank rehearsals with ``SMP_P2P=host``).
"""
import itertools
import os

import torch
import torch.distributed as dist

from ..backend.collectives import SERVER_CHANNEL, dumps, loads
from ..backend.logger import get_logger

logger = get_logger()

_REL = "__p2p_release__"


def choose_mode(core, device, backend):
    if device.type != "cuda":
        return "cpu"
    mode = os.environ.get("SMP_P2P", "").lower()
    if mode in ("ipc", "rccl", "host"):
        return mode
    if os.environ.get("SMP_DISABLE_D2D", "0") not in ("0", "", "false", "False"):
        # reference: SMP_DISABLE_D2D routes pipeline tensors through the host path
        return "host"
    same_node = all(core.is_in_same_instance(r) for r in core.get_pp_group())
    if same_node:
        return "ipc"
    return "rccl" if backend == "nccl" else "host"


class PipelineTransport:
    def __init__(self, core, pgs, device, mode=None, backend="nccl"):
        self.mailbox = core.mailbox
        self.rank = core.rank()
        self.pgs = pgs
        self.device = device
        self.mode = mode or ("cpu" if device.type != "cuda" else "rccl")
        self._inflight = []
        self._ids = itertools.count()
        self._held = {}  # (dst, xfer_id) -> (source tensor, event slot)   [ipc sender]
        self._pending_rel = {}  # src -> [(xfer_id, slot, event)]         [ipc receiver]
        self._ipc = None
        if self.mode == "ipc":
            from ..ops._ext import ext

            self._ipc = ext().IpcP2P(device.index if device.index is not None else torch.cuda.current_device())
        self.bytes_sent = 0
        self.bytes_recv = 0

    # ------------------------------------------------------------ set-up
    def warmup(self, pp_group_ranks):
        """RCCL: initialise every directed communicator in one global order (no deadlock on
        lazy communicator creation)."""
        if self.mode != "rccl":
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

    # ------------------------------------------------------------ sending
    def _prune(self):
        if self._inflight:
            self._inflight = [(w, t) for (w, t) in self._inflight if not w.is_completed()]

    def send(self, dst, stubbed, tensors):
        meta, rccl = [], []
        for t in tensors:
            if not t.is_cuda:
                meta.append(("cpu", t.detach()))
                continue
            t = t.detach()
            nbytes = t.numel() * t.element_size()
            self.bytes_sent += nbytes
            if self.mode == "ipc":
                t = t.contiguous()
                rec = self._ipc.export_tensor(t)
                xid = next(self._ids)
                self._held[(dst, xid)] = (t, rec[5])
                meta.append(("ipc", tuple(t.shape), t.dtype, xid, rec))
            elif self.mode == "rccl":
                meta.append(("rccl", tuple(t.shape), t.dtype))
                rccl.append(t.contiguous())
            else:  # host staging
                meta.append(("host", t.to("cpu")))
        self.mailbox.send(dst, 0, SERVER_CHANNEL, dumps((stubbed, meta)))
        if rccl:
            g = self.pgs.p2p[(self.rank, dst)]
            for t in rccl:
                self._inflight.append((dist.isend(t, dst, group=g), t))
        self._prune()
        self._pump_releases()

    # ------------------------------------------------------------ receiving
    def poll(self, timeout):
        """Returns (src, stubbed, tensors) or None.  Release notes are consumed here."""
        self._pump_releases()
        while True:
            r = self.mailbox.next_server_message(timeout)
            if r is None:
                return None
            src, _tid, payload = r
            stubbed, meta = loads(payload)
            if isinstance(stubbed, tuple) and stubbed and stubbed[0] == _REL:
                self._on_release(src, stubbed[1])
                continue
            return src, stubbed, [self._materialize(src, m) for m in meta]

    def _materialize(self, src, m):
        kind = m[0]
        if kind == "cpu":
            return m[1]
        if kind == "host":
            return m[1].to(self.device, non_blocking=False)
        if kind == "ipc":
            _, shape, dtype, xid, rec = m
            base, gen, mh, off, nbytes, slot, eh = rec
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            self._ipc.import_copy(buf, src, base, gen, mh, off, nbytes, slot, eh)
            ev = torch.cuda.Event()
            ev.record()
            self._pending_rel.setdefault(src, []).append((xid, slot, ev))
            self.bytes_recv += nbytes
            return buf
        _, shape, dtype = m
        buf = torch.empty(shape, dtype=dtype, device=self.device)
        w = dist.irecv(buf, src, group=self.pgs.p2p[(src, self.rank)])
        w.wait()  # stream-ordered: compute stream waits for the RCCL event
        self.bytes_recv += buf.numel() * buf.element_size()
        return buf

    # ------------------------------------------------------------ ipc lifetime
    def _pump_releases(self, block=False):
        if not self._pending_rel:
            return
        for src in list(self._pending_rel):
            pend = self._pending_rel[src]
            done, keep = [], []
            for item in pend:
                ev = item[2]
                if block:
                    ev.synchronize()
                if block or ev.query():
                    done.append((item[0], item[1]))
                else:
                    keep.append(item)
            if done:
                self.mailbox.send(src, 0, SERVER_CHANNEL, dumps(((_REL, done), [])))
            if keep:
                self._pending_rel[src] = keep
            else:
                del self._pending_rel[src]

    def _on_release(self, src, items):
        for xid, slot in items:
            held = self._held.pop((src, xid), None)
            if held is not None:
                self._ipc.release_event(slot)

    def has_message(self):
        return self.mailbox.has_server_message()

    def drain(self):
        for w, _ in self._inflight:
            w.wait()
        self._inflight.clear()
        self._pump_releases(block=True)

    def stats(self):
        d = {"mode": self.mode, "bytes_sent": self.bytes_sent, "bytes_recv": self.bytes_recv,
             "held": len(self._held)}
        if self._ipc is not None:
            d.update(self._ipc.stats())
        return d
