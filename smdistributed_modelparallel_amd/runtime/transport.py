"""Pipeline data plane.

Replaces the reference's D2D engine + listener (N1c/N1d, `smp/torch/server_comm.py:30-353`,
`smp/torch/ops.py:42-123`): control messages are pickled (tensors stubbed) on the native
mailbox SERVER channel; tensor payloads travel by one of four paths:

* ``cpu``  -- CPU tensors embedded in the control message (gloo/CPU runs);
* ``ipc``  -- the default between GPU ranks of one node: the native ``IpcP2P`` engine
  (`csrc/torchrt/ipc_p2p.cpp`).  The sender publishes the caching-allocator segment that
  holds the tensor plus an inter-process HIP event recorded after the producer kernels;
  the control message is a GATED send of the native mailbox: the destination's sender
  thread lets it out once a plain HIP event recorded after the producer kernels has
  completed (no inter-process events, no device-side cross-process waits), keeping FIFO
  order per peer.  The receiver maps the segment once and, as soon as the control message
  arrives, enqueues one D2D pull copy (xGMI between GPUs) on a dedicated high-priority
  *communication* stream.  The compute stream only waits on that copy's event, at the
  point where the consuming task is enqueued, so pulls overlap the kernels already queued
  on the compute stream (reference: asynchronous D2D handles polled by the server,
  `smp/torch/ops.py:42-123`, `server_comm.py:260-302`).  Neither host blocks.  The
  receiver returns a release note (batched, out of band) once its copy has completed, and
  only then does the sender drop the source tensor and recycle the event slot; at the end
  of every step each rank waits for the release notes of everything it exported, so no
  activation stays pinned into the next step.  Because the pull is posted on arrival of
  the metadata, every receive is effectively pre-posted; there is no receive pool to size
  or overflow.  An init-time self-check (``ipc_self_check``) exports a pattern from every
  stage to every PP peer and compares the pulled bytes; if any pair fails anywhere, every
  rank falls back to ``rccl`` (or ``host`` on gloo) with a warning.
* ``rccl`` -- RCCL point-to-point (multi-node, or ``SMP_P2P=rccl``).  Each *directed* stage
  pair owns its own communicator, so sends and receives on it are matched FIFO and a send
  in one direction can never sit behind a receive in the other; the receiver posts its
  irecvs in control-message order (mailbox links are FIFO per pair).
* ``host`` -- host-staged copies inside the control message (GPU ranks on a gloo-only
  process group, e.g. single-GPU multi-rank rehearsals with ``SMP_P2P=host``).
"""
import itertools
import os
from collections import deque

import torch
import torch.distributed as dist

from ..backend.collectives import SERVER_CHANNEL, dumps, loads
from ..backend.logger import get_logger
from ..parallel.comm_timer import timer as comm_timer

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


def _selfcheck_forced_fail(rank):
    """SMP_P2P_SELFCHECK_FAIL=1 (every rank) or a comma list of global ranks: make the IPC
    self-check fail there, so the fallback path is testable on a one-GPU box."""
    v = os.environ.get("SMP_P2P_SELFCHECK_FAIL", "").strip()
    if not v or v in ("0", "false", "False"):
        return False
    if v in ("1", "true", "True", "all"):
        return True
    return str(rank) in [x.strip() for x in v.split(",")]


def ipc_self_check(core, device, numel=1 << 18):
    """Export a rank-specific pattern, let every PP peer pull it over IpcP2P and compare the
    bytes.  Collective over WORLD (every rank calls it, in every PP group at once) and the
    verdict is agreed over WORLD, because the transport choice decides which process groups
    every rank creates next.  Returns (ok, [failure descriptions])."""
    from ..backend.collectives import CommGroup

    comm = core.comm
    me = core.rank()
    err = None
    ipc = src = rec = None
    try:
        from ..ops._ext import ext

        ipc = ext().IpcP2P(device.index if device.index is not None else torch.cuda.current_device())
        src = (torch.arange(numel, dtype=torch.int32, device=device) * 7 + me * 1000003)
        rec = tuple(ipc.export_tensor(src))
        torch.cuda.synchronize(device)
    except Exception as e:  # noqa: B902 - reported and agreed below
        err = f"rank {me}: export failed: {e!r}"
        rec = None
    recs = comm.allgather((me, rec), CommGroup.PP_GROUP)
    fails = [err] if err else []
    if ipc is not None:
        for peer, prec in recs:
            if peer == me:
                continue
            if prec is None:
                fails.append(f"rank {me}: peer {peer} exported nothing")
                continue
            try:
                base, gen, mh, off, nbytes = prec
                buf = torch.empty(numel, dtype=torch.int32, device=device)
                ipc.import_copy(buf, peer, base, gen, mh, off, nbytes)
                torch.cuda.synchronize(device)
                want = torch.arange(numel, dtype=torch.int32, device=device) * 7 + peer * 1000003
                if _selfcheck_forced_fail(me) or not torch.equal(buf, want):
                    fails.append(f"rank {me}: bytes pulled from rank {peer} differ")
            except Exception as e:  # noqa: B902
                fails.append(f"rank {me}: pull from rank {peer} failed: {e!r}")
    all_fails = comm.allgather(fails, CommGroup.WORLD)  # also keeps `src` alive until every pull is done
    if ipc is not None:
        try:
            ipc.close()
        except Exception:  # noqa: B902
            pass
    flat = [f for fl in all_fails for f in fl]
    return not flat, flat


# verdict of the init-time IPC self-check: "passed", "failed -> <fallback>", or "not run"
SELFCHECK = {"verdict": "not run", "failures": []}


def resolve_mode(core, device, backend):
    """choose_mode + (for ``ipc`` with PP > 1) the init-time self-check and fallback."""
    mode = choose_mode(core, device, backend)
    SELFCHECK.update(verdict="not run", failures=[])
    if mode != "ipc" or core.pp_size() == 1 or os.environ.get("SMP_P2P_SELFCHECK", "1") == "0":
        return mode
    ok, fails = ipc_self_check(core, device)
    if ok:
        SELFCHECK["verdict"] = "passed"
        return mode
    fallback = "rccl" if backend == "nccl" else "host"
    SELFCHECK.update(verdict=f"failed -> {fallback}", failures=fails[:8])
    if os.environ.get("SMP_P2P", "").lower() == "ipc" and not os.environ.get("SMP_P2P_SELFCHECK_FAIL"):
        from ..backend.exceptions import SMPRuntimeError

        raise SMPRuntimeError("SMP_P2P=ipc requested but the IPC self-check failed: " + "; ".join(fails[:8]))
    if core.rank() == 0:
        logger.warning(f"IPC pipeline transport self-check failed ({'; '.join(fails[:4])}); "
                       f"falling back to '{fallback}' pipeline transport on every rank")
    return fallback


class PipelineTransport:
    def __init__(self, core, pgs, device, mode=None, backend="nccl"):
        self.mailbox = core.mailbox
        self.rank = core.rank()
        self.pgs = pgs
        self.device = device
        self.mode = mode or ("cpu" if device.type != "cuda" else "rccl")
        self._inflight = []
        self._ids = itertools.count()
        self._held = {}  # (dst, xfer_id) -> (source tensors, event slot)   [ipc sender]
        self._pending_rel = {}  # src -> [(xfer_id, slot, event)]          [ipc receiver]
        self._ipc = None
        self._comm = None  # receive-side communication stream (ipc pulls)
        self._deferred = deque()  # messages read while draining, delivered by the next poll()
        if self.mode == "ipc":
            from ..ops._ext import ext

            self._ipc = ext().IpcP2P(device.index if device.index is not None else torch.cuda.current_device())
            self._gate_fn = ext().IpcP2P.gate_fn()
            if os.environ.get("SMP_P2P_COMM_STREAM", "1") != "0":
                lo, hi = torch.cuda.Stream.priority_range()
                self._comm = torch.cuda.Stream(device=device, priority=min(lo, hi))
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.release_wait_timeouts = 0

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
        meta, rccl, exported = [], [], []
        for t in tensors:
            nbytes = t.numel() * t.element_size()
            self.bytes_sent += nbytes
            if not t.is_cuda:
                meta.append(("cpu", t.detach()))
                continue
            t = t.detach()
            if self.mode == "ipc":
                t = t.contiguous()
                rec = tuple(self._ipc.export_tensor(t))
                exported.append(t)
                meta.append(("ipc", tuple(t.shape), t.dtype, rec))
            elif self.mode == "rccl":
                meta.append(("rccl", tuple(t.shape), t.dtype))
                rccl.append(t.contiguous())
            else:  # host staging
                meta.append(("host", t.to("cpu")))
        if exported:
            # one readiness event per message; the mailbox lets the message out once the
            # producer kernels are done (csrc/runtime/mailbox.h GateFn)
            slot, ctx = self._ipc.record_event()
            xid = next(self._ids)
            self._held[(dst, xid)] = (exported, slot)
            self.mailbox.send_gated(dst, 0, SERVER_CHANNEL, dumps((stubbed, (xid, slot), meta)), self._gate_fn, ctx)
        else:
            self.mailbox.send(dst, 0, SERVER_CHANNEL, dumps((stubbed, None, meta)))
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
        if self._deferred:
            r = self._deferred.popleft()
        else:
            r = self._read(timeout)
            if r is None:
                return None
        src, stubbed, xfer, meta = r
        return src, stubbed, self._materialize_all(src, xfer, meta)

    def _read(self, timeout):
        """Next control message that is not a release note (release notes are applied)."""
        while True:
            r = self.mailbox.next_server_message(timeout)
            if r is None:
                return None
            src, _tid, payload = r
            stubbed, xfer, meta = loads(payload)
            if isinstance(stubbed, tuple) and stubbed and stubbed[0] == _REL:
                self._on_release(src, stubbed[1])
                continue
            return src, stubbed, xfer, meta

    def _materialize_all(self, src, xfer, meta):
        if xfer is None:
            return [self._materialize(src, m) for m in meta]
        # ipc message: every pull on the comm stream (or the compute stream), one completion
        # event for the release note
        ev = torch.cuda.Event()
        if self._comm is None:
            out = [self._materialize(src, m) for m in meta]
            ev.record()
        else:
            compute = torch.cuda.current_stream(self.device)
            # the buffers come from the comm stream's pool (no hidden ordering against compute
            # kernels still queued on a recycled block); compute waits on the pulls and
            # record_stream keeps each block from being recycled before compute used it
            with torch.cuda.stream(self._comm):
                out = [self._materialize(src, m) for m in meta]
                ev.record(self._comm)
            with comm_timer.region("p2p", self.device):
                compute.wait_event(ev)
            for t in out:
                if t.is_cuda:
                    t.record_stream(compute)
        xid, slot = xfer
        self._pending_rel.setdefault(src, []).append((xid, slot, ev))
        return out

    def _materialize(self, src, m):
        kind = m[0]
        if kind == "cpu":
            self.bytes_recv += m[1].numel() * m[1].element_size()
            return m[1]
        if kind == "host":
            self.bytes_recv += m[1].numel() * m[1].element_size()
            return m[1].to(self.device, non_blocking=False)
        if kind == "ipc":
            _, shape, dtype, rec = m
            base, gen, mh, off, nbytes = rec
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            self._ipc.import_copy(buf, src, base, gen, mh, off, nbytes)
            self.bytes_recv += nbytes
            return buf
        _, shape, dtype = m
        buf = torch.empty(shape, dtype=dtype, device=self.device)
        w = dist.irecv(buf, src, group=self.pgs.p2p[(src, self.rank)])
        with comm_timer.region("p2p", self.device):
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
                self.mailbox.send(src, 0, SERVER_CHANNEL, dumps(((_REL, done), None, [])))
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
        return bool(self._deferred) or self.mailbox.has_server_message()

    def drain(self, release_timeout=None):
        """End of step: finish RCCL sends, return release notes for every pulled tensor and
        wait until the peers have released every tensor this rank exported, so no source
        activation stays pinned into the next step.  Control messages of the next step that
        arrive meanwhile (a faster peer) are kept for the next poll()."""
        for w, _ in self._inflight:
            w.wait()
        self._inflight.clear()
        self._pump_releases(block=True)
        if not self._held:
            return
        if release_timeout is None:
            release_timeout = 30.0
        import time

        deadline = time.monotonic() + release_timeout
        while self._held:
            left = deadline - time.monotonic()
            if left <= 0:
                self.release_wait_timeouts += 1
                logger.warning(f"rank {self.rank}: {len(self._held)} exported pipeline tensors not released by "
                               f"their receivers after {release_timeout:.0f} s; keeping them until released")
                return
            r = self._read(min(left, 0.05))
            if r is not None:
                self._deferred.append(r)

    def stats(self):
        d = {"mode": self.mode, "bytes_sent": self.bytes_sent, "bytes_recv": self.bytes_recv,
             "held": len(self._held), "comm_stream": self._comm is not None,
             "release_wait_timeouts": self.release_wait_timeouts}
        if self._ipc is not None:
            d.update(self._ipc.stats())
        return d
