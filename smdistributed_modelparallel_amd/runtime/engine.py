"""Pipeline execution engine.

What it does (reference behaviour, `smp/torch/server.py`, `worker.py`, `ops.py`,
`patches/execution.py`, `sequential.py`): pp_rank 0 runs the user's step function per
microbatch; whenever a module owned by another pipeline stage is called, the call becomes
a request to that stage, the caller's coroutine is suspended and the server keeps
scheduling other microbatches -- the pipeline schedule emerges from the task priorities
(``interleaved`` / ``simple`` with the ``active_microbatches`` cap).  ``nn.Sequential``
stacks are executed as chains that hop stage to stage directly (child-to-child) and only
return to the caller at the end.

How it is built here (our design, not the reference's):

* **Coroutines are greenlets**, not OS threads handing a condition variable back and
  forth: one OS thread, zero lock hand-offs, deterministic interleaving.
* **Backward is segmented and asynchronous.** A remote call saves (requester side) the
  tensors it sent and (executor side) its outputs and its input leaves.  Autograd hooks
  (`RemoteOutput.backward`) and input-leaf gradients turn into backward *messages* to
  whichever rank holds the next segment; every segment runs
  ``torch.autograd.backward(saved, grads, retain_graph=True)`` -- gradients are linear,
  so partial segments compose exactly.  No backward function ever blocks.
* **Termination is an ack tree** (Dijkstra-Scholten): every backward message is acked
  once the work it spawned has been acked; the microbatch root on pp_rank 0 completes
  when its own children are acked.  This replaces the reference's real/dummy/sequential
  receive counting (`module_manager.py:360-720`, `server.py:162-252`).
* Microbatch state is freed when pp_rank 0 broadcasts the microbatch-end message, which
  also carries the step outputs to every stage (`MicrobatchEndResult` semantics).
* **Deterministic task order under tensor parallelism.**  The TP peers of a stage run
  separate engines fed by separate pipelines, but their modules issue TP collectives that
  must match one-to-one.  tp_rank 0 decides: before executing any event (a message, a
  locally queued result, a scheduling action) it sends the event's TP-invariant key to
  its TP peers, which execute exactly that sequence (reference `DeterministicServerQueue`,
  `server_queue.py:224-626`, forced when TP > 1).  Message ids are (pp_rank, counter),
  the counter restarting every step, so the same logical message has the same key on
  every TP peer AND in every step.
* **Record and replay.**  For the first ``SMP_REPLAY_RECORD_STEPS`` (5) steps of a step
  function every decider records its event sequence and the step time.  Then the global
  leader picks the fastest recorded step, every decider hands that step's sequence to its
  TP peers, and from then on all ranks of the model-parallel group replay it: no decision
  messages, no dynamic choices (reference `server_queue.py:224-626`, record window 5 steps
  `:245`, best step `:575-626`).  All stages replay the SAME recorded step, so the replayed
  orders are one feasible global execution.  It runs for TP > 1, ``static_mode``,
  ``fast_mode`` and activation offloading (``SMP_REPLAY=1`` opts other pipelines in); a
  replayed step whose events differ from the frozen ones raises instead of waiting.
  With the IPC transport a tensor is pulled the moment its control message is dispatched,
  so the reference's pre-registered receptions (`:488`) have nothing left to pre-post.
* **Fast mode** (``fast_mode``; reference `torch/serialization.py:365-473`, `step.py:150-230`,
  `patches/execution.py:283,362`, `worker.py:329,397,473`): during microbatch 0 of a step
  function's first step every parent records which stage / module call consumes each
  output of a remote module call (``(call target, call count), output index``), local uses
  included; the maps are merged over PP at the end of that step.  From then on a producer
  whose output is consumed only by other children sends it STRAIGHT to the consuming
  stage(s) ("dtx") and returns a dummy to the parent -- a meta-device tensor, so any real
  use by the parent fails loudly.  Passing the dummy on to the consumer sends a
  ``DirectStub``; the consumer resolves it from what it received out of band (waiting if
  the parent's request overtook the tensor), and the consumer's input gradient goes
  straight back to the producing stage ("dout").  A dummy that reaches a call the maps do
  not name raises ``NotSupportedByFastModeError(graph_change=True)``.
"""
import os
import time
from collections import Counter, deque
import itertools

import torch
from greenlet import greenlet

from ..backend.exceptions import (
    MissingPathFromComputationToModuleOutputError,
    MissingPathFromModuleInputToModuleOutputError,
    NotSupportedByFastModeError,
    PipelineParallelBWDError,
    SMPRuntimeError,
)
from ..backend.logger import get_logger
from .pipeline import MbStatus, create_pipeline
from .serialization import DirectStub, find_direct, iter_tensors, stubify, unstubify

logger = get_logger()


class RemoteOutput(torch.autograd.Function):
    """Outputs of a module executed on another stage (reference ``SMPParentRecv``).

    Forward is an identity on the received tensors; backward ships the output
    gradients to the stage that holds the producing graph segment."""

    @staticmethod
    def forward(ctx, engine, holder, key, mb, *tensors):
        ctx.set_materialize_grads(False)
        ctx.engine, ctx.holder, ctx.key, ctx.mb = engine, holder, key, mb
        return tuple(t.view_as(t) for t in tensors)

    @staticmethod
    def backward(ctx, *grads):
        if any(g is not None for g in grads):
            ctx.engine._entry_grads(ctx.mb, ("rout", ctx.key), ctx.holder, ("out", ctx.key), grads)
        return (None, None, None, None) + (None,) * len(grads)


class _Entry:
    """Tensors whose gradients go to another stage (a request's input leaves, a fast-mode
    consumer leaf, or a RemoteOutput).  Their gradients are sent ONCE per microbatch: after
    every backward wave that can reach them has run (``pending`` = number of registered
    wave sources whose graph reaches them).  So every saved segment on the peer receives
    exactly one backward message per microbatch -- which is what the GradTracker counts
    (reference: the aggregated backward of `worker.py:382-418` + `ops.py:131`).  Sending per
    wave instead broke DDP finality when an output fanned out to several consumers: the
    peer's segment then ran once per consumer, beyond its registered count, and a bucket was
    scaled and reduced before the last accumulation.  An entry that ends up with no gradient
    still sends one (empty) message: the peer's segment then knows no wave will come, and the
    entries IT holds are released in turn (an unused path must not block the used ones)."""

    __slots__ = ("targets", "pending", "grads", "dst", "key", "leaf", "flushed")

    def __init__(self, targets, dst, key, leaf):
        self.targets = targets
        self.pending = 0
        self.grads = None
        self.dst, self.key, self.leaf = dst, key, leaf
        self.flushed = False

    def take(self):
        """The accumulated gradients (None: nothing arrived), reset."""
        if self.leaf:
            gs = [t.grad for t in self.targets]
            if all(g is None for g in gs):
                return None
            for t in self.targets:
                t.grad = None
            return gs
        gs, self.grads = self.grads, None
        return gs


class _Token:
    __slots__ = ("pending", "ack_to", "remote_token", "mb", "done")

    def __init__(self, ack_to, remote_token, mb):
        self.pending = 0
        self.ack_to = ack_to
        self.remote_token = remote_token
        self.mb = mb
        self.done = False


class _Worker:
    __slots__ = ("g", "mb", "kind", "result", "exc", "wait_key", "routs")

    def __init__(self, g, mb, kind):
        self.g, self.mb, self.kind = g, mb, kind
        self.result = None
        self.exc = None
        self.wait_key = None
        self.routs = []  # (RemoteOutput result, producing module) created by this worker


class _MbState:
    __slots__ = ("sent", "leaves", "out", "out_direct", "dleaves", "entries", "reach")

    def __init__(self):
        self.sent = {}
        self.leaves = {}
        self.out = {}
        self.out_direct = {}  # (rid, mi) -> output tensor sent child-to-child   [fast mode producer]
        self.dleaves = {}  # rid -> [(leaf, producer rank, ("dout", prid, mi))]  [fast mode consumer]
        self.entries = {}  # entry id -> _Entry (gradients owed to another stage)
        self.reach = {}  # wave source key -> [entries its backward reaches]


class _FastMode:
    """Per step function: consumer maps recorded on microbatch 0 of its first step."""
    __slots__ = ("rec", "map")

    def __init__(self):
        self.rec = {}  # mi -> {(consumer pp_rank, call target, call count)}  (this rank's calls)
        self.map = None  # merged over PP after the recording step: mi -> [(pp_rank, target, count)]


class PipelineEngine:
    RECORD_STEPS = int(os.environ.get("SMP_REPLAY_RECORD_STEPS", "5"))

    def __init__(self, state):
        self.state = state
        self._ids = itertools.count()
        self._recorded = {}  # step fn id -> [(seconds, [event keys])]   (deciders only)
        self._replay = {}  # step fn id -> frozen event keys
        self._replay_mbs = {}  # step fn id -> microbatch of each frozen event (None: n/a)
        self._recording = None
        self._cur_worker = None
        self.reset_step()
        wd = getattr(state.core, "watchdog", None) if getattr(state, "core", None) is not None else None
        if wd is not None:
            wd.diagnostics.append(self.debug_state)

    def debug_state(self):
        """One line of what this rank's pipeline is waiting for (the watchdog logs it on a step
        timeout or a peer failure): microbatch statuses, open wait keys, per-microbatch
        gradient entries still owed, transport holds."""
        pl = self.pipeline
        status = [int(x) for x in pl.status] if pl is not None else None
        waits = sorted(str(k) for k in list(self.waiting))[:24]
        owed = {mb: sum(1 for e in list(st.entries.values()) if not e.flushed)
                for mb, st in list(self.mbstate.items())}
        tr = self.state.transport
        ts = tr.stats() if tr is not None and hasattr(tr, "stats") else {}
        return (f"mb_status={status} active={getattr(pl, 'active_mb', None)} waiting={waits} "
                f"local_q={len(self._local_q)} entries_owed={owed} transport={ts}")

    # ------------------------------------------------------------- plumbing
    @property
    def core(self):
        return self.state.core

    def reset_step(self):
        self.mbstate = {}
        self._callcount = {}  # (mb, call target) -> calls so far (fast-mode call identity)
        self._direct_in = {}  # (mb, mi) -> (tensor, producer rank, producer call id)
        self.tokens = {}
        self.waiting = {}  # wait key -> worker
        self.workers = []
        self.results = {}
        self.pipeline = None
        self._cur_token = None
        self._stop = False
        self._root_tokens = {}
        self._local_q = []
        self._tl = None

    def _new_id(self):
        # (pp_rank, n): identical on every TP / DP peer executing the same task sequence
        return (self.core.pp_rank(), next(self._ids))

    def _mb(self, mb):
        s = self.mbstate.get(mb)
        if s is None:
            s = self.mbstate[mb] = _MbState()
        return s

    def _pp_peer(self, pp_rank):
        return self.core.pp_rank_to_rank(pp_rank)

    def _send(self, dst, msg):
        stubbed, tensors = stubify(msg)
        self.state.transport.send(dst, stubbed, tensors)

    # ------------------------------------------------------------- tracing
    def _traced(self, mb, label, fn, *args):
        """Run one scheduler task; with SMP_TIMELINE_FILE / SMP_ROCTX=1 it becomes a
        Chrome-trace span and a roctx range (reference `server.py:366-478`
        timeline_record_pipeline_event around every request/result)."""
        tl = self._tl
        if tl is None:
            return fn(*args)
        t0 = tl.now_us()
        tl.range_push(label)
        try:
            return fn(*args)
        finally:
            tl.range_pop()
            tl.record(mb, label, t0, tl.now_us())

    def _broadcast_pp(self, msg):
        me = self.core.rank()
        for r in self.core.get_pp_group():
            if r != me:
                self._send(r, msg)

    # ============================================================= fast mode
    def _fm(self):
        """(state, recording now, maps in use) for the running step function."""
        cfg = self.state.cfg
        sf = getattr(self, "step_fn", None)
        if cfg is None or not cfg.fast_mode or sf is None or self.core.pp_size() == 1:
            return None, False, False
        fm = sf.__dict__.get("_fm")
        if fm is None:
            fm = sf.__dict__["_fm"] = _FastMode()
        recording = sf.calls == 0 and self.state.microbatch == 0
        return fm, recording, fm.map is not None

    def fm_note_local(self, obj):
        """Recording step: tensors of remote module outputs used on THIS rank (a local module
        call, the step function's outputs, model.backward) must reach the parent for real."""
        fm, recording, _ = self._fm()
        if not recording:
            return
        me = self.core.pp_rank()
        for t in iter_tensors(obj):
            mi = getattr(t, "_smp_mi", None)
            if mi is not None:
                fm.rec.setdefault(mi, set()).add((me, None, None))

    def _fm_merge(self, step_fn):
        """End of the recording step (every rank, symmetric): merge the consumer maps over PP."""
        fm = step_fn.__dict__.get("_fm")
        if fm is None or fm.map is not None:
            return
        from ..backend.collectives import CommGroup

        merged = {}
        for rec in self.state.comm.allgather(fm.rec, CommGroup.PP_GROUP):
            for mi, cons in rec.items():
                merged.setdefault(mi, set()).update(cons)
        fm.map = {mi: sorted(c, key=repr) for mi, c in merged.items()}
        logger.info(f"fast mode: direct-consumer maps merged for step function {step_fn.id} "
                    f"({len(fm.map)} module outputs)")

    def _dummy_stub(self, fm, t, owner_pp, target, count):
        """Parent side: a fast-mode dummy passed on to a remote call becomes a DirectStub."""
        if t.device.type != "meta":
            return None
        mi = getattr(t, "_smp_mi", None)
        if mi is None:
            raise NotSupportedByFastModeError(detail="a tensor transmitted child-to-child was transformed by the parent")
        if (owner_pp, target, count) not in (fm.map or {}).get(mi, ()):
            raise NotSupportedByFastModeError(graph_change=True, detail=f"{mi} reached {target} #{count}")
        return DirectStub(mi, t.shape, t.dtype, t.requires_grad)

    # ============================================================== run_step
    def run_step(self, step_fn, mb_inputs):
        model = self.state.model
        if self.core.pp_size() == 1:
            return self._run_local(step_fn, mb_inputs)
        model._ensure_partitioned(step_fn, mb_inputs)
        return self._run_pipelined(step_fn, mb_inputs)

    def _run_local(self, step_fn, mb_inputs):
        outs = []
        n = len(mb_inputs)
        model = self.state.model
        for mb, (a, k) in enumerate(mb_inputs):
            self.state.microbatch = mb
            model._begin_microbatch(mb, n)
            outs.append(step_fn.run_microbatch(mb, a, k))
        return outs

    # ------------------------------------------------------------ pipelined
    def _run_pipelined(self, step_fn, mb_inputs):
        self.reset_step()
        self._ids = itertools.count()  # step-relative ids: keys repeat step to step (replay)
        cfg = self.state.cfg
        n = cfg.microbatches
        self.num_mb = n
        leader = self.core.pp_rank() == 0
        self.server = greenlet.getcurrent()
        tl = self.core.timeline
        self._tl = tl if (tl is not None and (tl.enabled or tl.roctx_enabled)) else None
        self.step_fn = step_fn
        self.mb_inputs = mb_inputs
        if leader:
            self.pipeline = create_pipeline(cfg.pipeline, n, cfg.active_microbatches)
        failed = True
        try:
            self._serve(leader)
            failed = False
        except SMPRuntimeError:
            raise
        except BaseException as e:  # noqa: B902 - tell the other stages before dying
            self._abort(e)
        finally:
            self.state.transport.drain(release_timeout=0.0 if failed else None)
        outs = [self.results[i] for i in range(n)]
        self.reset_step()
        return outs

    # ------------------------------------------------------- record / replay
    def replay_enabled(self):
        """Record-and-replay runs where the reference forces its DeterministicServerQueue
        (`torch/server.py:57-65`): TP > 1 (collective order), ``static_mode``, ``fast_mode`` and
        ``offload_activations`` (the task-level activation prefetch needs the frozen order).
        Every other pipeline keeps the dynamic scheduler -- its module graph may change from
        step to step (static_mode=False is the default) -- unless ``SMP_REPLAY=1`` opts in.
        SMP_NONDETERMINISTIC_TP_ORDER=1 (tests) disables both.  A replayed step whose events
        differ from the frozen schedule raises (``_serve_follower``) instead of waiting
        forever."""
        core = self.core
        if core.pp_size() <= 1 or os.environ.get("SMP_NONDETERMINISTIC_TP_ORDER", "0") == "1":
            return False
        cfg = self.state.cfg
        forced = (core.tp_size() > 1 or bool(cfg.static_mode) or bool(cfg.fast_mode)
                  or bool(cfg.offload_activations))
        return forced or os.environ.get("SMP_REPLAY", "0") == "1"

    def after_step(self, step_fn, seconds):
        """Called on every rank after every pipelined step (symmetric collectives)."""
        if self.state.cfg.fast_mode:
            self._fm_merge(step_fn)
        if not self.replay_enabled():
            return
        sid = step_fn.id
        if sid in self._replay:
            return
        core, comm = self.core, self.state.comm
        from ..backend.collectives import CommGroup

        rec = self._recorded.setdefault(sid, [])
        rec.append((seconds, self._recording or []))
        self._recording = None
        if len(rec) < self.RECORD_STEPS:
            return
        # the global leader picks the fastest recorded step; every stage replays that SAME step
        ranker = core.ranker
        best = None
        if core.pp_rank() == 0 and core.tp_rank() == 0:
            best = min(range(len(rec)), key=lambda i: rec[i][0])
        if core.mp_size() > 1:
            best = comm.bcast(best, ranker.translate(0, 0, core.rdp_rank()), CommGroup.MP_GROUP)
        pairs = rec[best][1] if core.tp_rank() == 0 else None
        if core.tp_size() > 1:
            pairs = comm.bcast(pairs, ranker.translate(core.pp_rank(), 0, core.rdp_rank()), CommGroup.TP_GROUP)
        keys = [k for k, _ in pairs]
        self._replay[sid] = keys
        self._replay_mbs[sid] = [m for _, m in pairs]
        self._recorded.pop(sid, None)
        logger.info(f"pipeline schedule frozen for step function {sid}: recorded step {best} "
                    f"({len(keys)} events) is replayed from now on")

    def _serve(self, leader):
        core = self.core
        replay = self._replay.get(self.step_fn.id) if self.replay_enabled() else None
        self._det = (core.tp_size() > 1 and os.environ.get("SMP_NONDETERMINISTIC_TP_ORDER", "0") != "1") or \
            self.replay_enabled()
        if replay is not None:
            self._tp_peers = []
            return self._serve_follower(leader, replay=replay, replay_mbs=self._replay_mbs.get(self.step_fn.id))
        if self._det:
            me = core.rank()
            self._tp_peers = [r for r in core.get_tp_group() if r != me]
            if core.tp_rank() != 0:
                return self._serve_follower(leader)
            if self.replay_enabled():
                self._recording = []
        timeout = 0.05
        while not self._stop:
            progressed = False
            while self._local_q:
                result_id, payload = self._local_q.pop(0)
                self._announce(("lres", result_id))
                self._resume(self.waiting.pop(("res", result_id)), payload)
                progressed = True
            while True:
                m = self.state.transport.poll(0.0)
                if m is None:
                    break
                self._dispatch_decided(m)
                progressed = True
                if self._stop:
                    return
            if leader:
                if self.pipeline.is_done():
                    self._stop = True
                    return
                act = self.pipeline.next_action()
                if act is not None:
                    self._announce(("act",) + tuple(act), act[1])
                    self._do_action(act)
                    progressed = True
            if not progressed:
                self._idle_prefetch()
                m = self.state.transport.poll(timeout)
                if m is not None:
                    self._dispatch_decided(m)

    def _do_action(self, act):
        kind, mb = act
        if kind == "fwd":
            self._traced(mb, f"FWD mb{mb} (step fn)", self._start_microbatch, mb)
        else:
            self._prefetch_activations(mb)
            self.pipeline.set_status(mb, MbStatus.BWD)
            self._traced(mb, f"BWD mb{mb} (loss)", self._resume, self.waiting.pop(("bwd_start", mb)), None)

    def _event_key(self, src, stubbed):
        kind = stubbed[0]
        if kind in ("fwd", "res"):
            return (kind, stubbed[1])
        if kind == "bwd":
            return (kind, self.core.ranker.get_pp_rank(src), stubbed[4])
        if kind == "ack":
            return (kind, self.core.ranker.get_pp_rank(src), stubbed[1])
        if kind == "mbdone":
            return (kind, stubbed[1])
        if kind == "dtx":
            return (kind, stubbed[1], stubbed[2])
        return (kind,)

    def _announce(self, key, mb=None):
        if self._det:
            if self._recording is not None:
                self._recording.append((key, mb))
            # tagged with the step: a decider may start step t+1 while a TP peer (in
            # another pipeline) is still finishing step t
            msg = ("dec", self.state.step_count, key)
            for r in self._tp_peers:
                self.state.transport.send(r, msg, [])

    def _dispatch_decided(self, m):
        src, stubbed, tensors = m
        if stubbed[0] not in ("abort", "dec"):
            kind = stubbed[0]
            mb = stubbed[2] if kind in ("fwd", "res", "bwd") else (stubbed[1] if kind in ("mbdone", "dtx") else None)
            self._announce(self._event_key(src, stubbed), mb)
        self._dispatch(src, stubbed, tensors)

    def _serve_follower(self, leader, replay=None, replay_mbs=None):
        """TP peer of a deciding rank (or any rank replaying a frozen schedule): execute
        events strictly in the decided order."""
        pending = {}
        pos = 0  # index of decisions[0] in the replayed schedule
        step = self.state.step_count
        owed = None  # replay: how many times each key is still expected this step
        if replay is not None:
            decisions = deque(replay)
            owed = Counter(replay)
            stall_s = float(os.environ.get("SMP_REPLAY_STALL_TIMEOUT_S", "600"))
            last = time.monotonic()
        else:
            stash = getattr(self, "_dec_stash", deque())
            decisions = deque(k for st, k in stash if st == step)
            self._dec_stash = deque((st, k) for st, k in stash if st != step)
        timeout = 0.05
        while not self._stop:
            m = self.state.transport.poll(0.0 if decisions else timeout)
            while m is not None:
                src, stubbed, tensors = m
                if stubbed[0] == "dec":
                    if stubbed[1] == step:
                        decisions.append(stubbed[2])
                    else:
                        self._dec_stash.append((stubbed[1], stubbed[2]))
                elif stubbed[0] == "abort":
                    self._dispatch(src, stubbed, tensors)
                else:
                    key = self._event_key(src, stubbed)
                    if owed is not None and owed[key] <= sum(1 for k in pending if k == key):
                        self._replay_mismatch(f"event {key} from rank {src} is not in the frozen schedule", decisions)
                    pending[key] = m
                m = self.state.transport.poll(0.0)
            if replay_mbs is not None:
                self._lookahead_prefetch(replay, replay_mbs, pos)
            pos0 = pos
            while decisions and not self._stop:
                key = decisions[0]
                pos += 1
                if owed is not None and not (key[0] in ("act", "lres") or key in pending):
                    pos -= 1
                    break  # the decided message has not arrived yet
                if owed is not None:
                    owed[key] -= 1
                    if key[:2] == ("act", "bwd") and ("bwd_start", key[2]) not in self.waiting:
                        self._replay_mismatch(f"microbatch {key[2]}'s forward has not finished where the frozen "
                                              "schedule starts its backward", decisions)
                if key[0] == "act":
                    decisions.popleft()
                    self._do_action(key[1:])
                elif key[0] == "lres":
                    idx = next((i for i, (rid, _) in enumerate(self._local_q) if rid == key[1]), None)
                    if idx is None:
                        raise SMPRuntimeError(f"decided local result {key[1]} not produced on rank {self.core.rank()}")
                    decisions.popleft()
                    result_id, payload = self._local_q.pop(idx)
                    self._resume(self.waiting.pop(("res", result_id)), payload)
                elif key in pending:
                    decisions.popleft()
                    self._dispatch(*pending.pop(key))
                else:
                    pos -= 1
                    break  # the decided message has not arrived yet
            if owed is not None and not self._stop:
                now = time.monotonic()
                if pos != pos0:
                    last = now
                elif not decisions and not (leader and self.pipeline.is_done()):
                    self._replay_mismatch("the frozen schedule is exhausted but the step has not finished", decisions)
                elif now - last > stall_s:
                    self._replay_mismatch(f"no event of the frozen schedule arrived for {stall_s:.0f} s "
                                          f"(SMP_REPLAY_STALL_TIMEOUT_S)", decisions)
            if leader and self.pipeline.is_done() and not decisions:
                self._stop = True

    def _replay_mismatch(self, what, decisions):
        nxt = list(decisions)[:3]
        raise SMPRuntimeError(
            f"rank {self.core.rank()} step {self.state.step_count}: {what}; next expected events {nxt}.  The "
            "module graph changed after the pipeline schedule was frozen (record-and-replay runs for TP > 1, "
            "static_mode, fast_mode and offload_activations, or SMP_REPLAY=1): keep the per-step module calls "
            "identical, or run without those options / with SMP_REPLAY=0.")

    # ------------------------------------------------- activation prefetching
    def _offloader(self):
        st = self.state
        return st.current_offloader if (st.cfg is not None and st.cfg.offload_activations) else None

    def _prefetch_activations(self, mb):
        off = self._offloader()
        if off is not None:
            off.prefetch_microbatch(mb)

    def _lookahead_prefetch(self, keys, mbs, pos):
        """Replayed schedule (reference `server_queue.py:492-548`): start loading the
        offloaded activations of every backward among the next
        ``task_level_activation_loading_horizon`` events, so host->device copies overlap
        the tasks before them."""
        off = self._offloader()
        if off is None:
            return
        for i in range(pos, min(len(keys), pos + max(1, int(self.state.cfg.task_level_activation_loading_horizon)))):
            k = keys[i]
            if k[0] == "bwd" or (k[0] == "act" and k[1] == "bwd"):
                off.prefetch_microbatch(mbs[i] if k[0] == "bwd" else k[2])

    def _idle_prefetch(self):
        """Dynamic schedule: nothing runnable -- use the idle link to load the activations
        of the oldest microbatch whose backward has not reached this stage yet."""
        off = self._offloader()
        if off is not None:
            mb = off.next_pending_microbatch()
            if mb is not None:
                off.prefetch_microbatch(mb)

    # ----------------------------------------------------------- coroutines
    def _spawn(self, fn, mb, kind, *args):
        w = _Worker(None, mb, kind)

        def run(*_ignored):
            try:
                w.result = fn(*args)
            except BaseException as e:  # noqa: B902 - re-raised in the server
                w.exc = e
            return ("exit", w)

        w.g = greenlet(run, parent=self.server)
        self.workers.append(w)
        self._resume(w, None)

    def _resume(self, worker, value):
        prev, self._cur_worker = self._cur_worker, worker
        try:
            ret = worker.g.switch(value)
        finally:
            self._cur_worker = prev
        self._after_switch(worker, ret)

    def _after_switch(self, worker, ret):
        kind, payload = ret
        if kind == "exit":
            self.workers.remove(worker)
            if worker.exc is not None:
                self._abort(worker.exc)
            if worker.kind == "root":
                self._finish_microbatch(worker.mb, worker.result)
        elif kind == "wait":
            worker.wait_key = payload
            self.waiting[payload] = worker
            if payload[0] == "bwd_start":
                self.pipeline.set_status(payload[1], MbStatus.READY_FOR_BWD)
                self.state.model._mark_fwd_pass_done(payload[1])

    def _suspend(self, key):
        """Called from a worker: yield to the server until `key` is satisfied."""
        st = self.state
        saved = (torch.is_grad_enabled(), st.microbatch, self._cur_token)
        cur = greenlet.getcurrent()
        worker = next((w for w in self.workers if w.g is cur), None)
        if worker is None:
            raise SMPRuntimeError("remote call outside of a pipeline worker")
        value = self.server.switch(("wait", key))
        torch.set_grad_enabled(saved[0])
        st.microbatch = saved[1]
        self._cur_token = saved[2]
        return value

    def _abort(self, exc):
        try:
            self._broadcast_pp(("abort", repr(exc)))
        except Exception:  # pragma: no cover
            pass
        raise exc

    # ------------------------------------------------------------- dispatch
    def _dispatch(self, src, stubbed, tensors):
        if self._tl is not None and stubbed[0] in ("fwd", "res", "bwd"):
            kind = stubbed[0]
            mb = stubbed[2]
            if kind == "fwd":
                label = f"FWD mb{mb} {stubbed[3][1]}" + (f"[{stubbed[3][2]}:]" if stubbed[3][0] == "chain" else "")
            elif kind == "bwd":
                label = f"BWD mb{mb} {stubbed[1][0]}{stubbed[1][1]} from r{src}"
            else:
                label = f"RESULT mb{mb} from r{src}"
            return self._traced(mb, label, self._dispatch_impl, src, stubbed, tensors)
        return self._dispatch_impl(src, stubbed, tensors)

    def _dispatch_impl(self, src, stubbed, tensors):
        kind = stubbed[0]
        if kind in ("fwd", "bwd") and stubbed[2] == 0 and not self.state.has_uploaded_metrics:
            self.state.num_hops += 1  # reference server.py:366-368,449-451
        if kind == "fwd":
            self._spawn(self._exec_fwd, stubbed[2], "fwd", src, stubbed, tensors)
        elif kind == "res":
            _, result_id, mb, out_stubbed, holder, out_key, grad_enabled = stubbed
            w = self.waiting.pop(("res", result_id))
            self._resume(w, (out_stubbed, tensors, holder, out_key))
        elif kind == "bwd":
            _, key, mb, grads_stubbed, remote_token = stubbed
            # a backward request for mb: its forward is over everywhere (server.py:455)
            self.state.model._mark_fwd_pass_done(mb)
            self._prefetch_activations(mb)
            grads = unstubify(grads_stubbed, tensors)
            self._process_bwd(src, key, mb, grads, remote_token)
        elif kind == "ack":
            self._ack(stubbed[1])
        elif kind == "dtx":
            # fast mode: a module output sent straight from its producer to this consumer
            _, mb, mi, prid = stubbed
            self._direct_in[(mb, mi)] = (tensors[0], src, prid)
            w = self.waiting.pop(("dtx", mb, mi), None)
            if w is not None:
                self._resume(w, None)
        elif kind == "mbdone":
            _, mb, out_stubbed = stubbed
            self.results[mb] = unstubify(out_stubbed, tensors)
            self.state.model._mark_fwd_pass_done(mb)
            self.mbstate.pop(mb, None)
            self.state.model._on_microbatch_done(mb)
            if len(self.results) == self.num_mb:
                self._stop = True
        elif kind == "abort":
            raise SMPRuntimeError(f"peer pipeline stage (rank {src}) failed: {stubbed[1]}")
        else:
            raise SMPRuntimeError(f"unknown pipeline message {kind}")

    # ----------------------------------------------------------- microbatch
    def _start_microbatch(self, mb):
        self.pipeline.set_status(mb, MbStatus.FWD)
        a, k = self.mb_inputs[mb]
        self.state.model._begin_microbatch(mb, self.num_mb)

        def run():
            self.state.microbatch = mb
            return self.step_fn.run_microbatch(mb, a, k)

        self._spawn(run, mb, "root")

    def _finish_microbatch(self, mb, out):
        self.fm_note_local(out)
        self.pipeline.mark_done(mb)
        self.results[mb] = out
        self.mbstate.pop(mb, None)
        self.state.model._on_microbatch_done(mb)
        self._broadcast_pp(("mbdone", mb, out))

    # ------------------------------------------------------- forward (remote)
    def remote_module_call(self, module, args, kwargs):
        mm = self.state.module_manager
        name = mm.get_module_name(module)
        owner = self._pp_peer(mm.get_partition(module))
        return self._remote_call(owner, ("module", name), (args, kwargs))

    def remote_chain_call(self, seq, start, inp):
        mm = self.state.module_manager
        name = mm.get_module_name(seq)
        child = list(seq)[start]
        owner = self._pp_peer(mm.get_partition(child))
        return self._remote_call(owner, ("chain", name, start), ((inp,), {}))

    def _remote_call(self, owner, target, payload):
        st = self.state
        mb = st.microbatch
        rid = self._new_id()
        grad_enabled = torch.is_grad_enabled()
        count = self._callcount.get((mb, target), 0)
        self._callcount[(mb, target)] = count + 1
        fm, recording, using = self._fm()
        direct = None
        if fm is not None:
            owner_pp = self.core.ranker.get_pp_rank(owner)
            if recording:
                for t in iter_tensors(payload):
                    mi = getattr(t, "_smp_mi", None)
                    if mi is not None:
                        fm.rec.setdefault(mi, set()).add((owner_pp, target, count))
            if using:
                def direct(t):
                    return self._dummy_stub(fm, t, owner_pp, target, count)
        stubbed, tensors = stubify(payload, direct)
        sent = []
        if grad_enabled:
            sent = [t for t in tensors if t.requires_grad]
            if sent:
                self._mb(mb).sent[rid] = sent
                self._register_source(mb, ("in", rid), sent)
        mi_base = (target, count) if fm is not None else None
        st.transport.send(owner, ("fwd", rid, mb, target, stubbed, self.core.rank(), rid, grad_enabled, mi_base),
                          tensors)
        out_stubbed, out_tensors, holder, out_key = self._suspend(("res", rid))
        producer = target[1] if target[0] == "module" else f"{target[1]}[{target[2]}:]"
        return self._materialize_outputs(out_stubbed, out_tensors, holder, out_key, mb, grad_enabled, producer, sent)

    def _materialize_outputs(self, out_stubbed, tensors, holder, out_key, mb, grad_enabled, producer=None, sent=()):
        _, stubs = _stubs_of(out_stubbed)
        dummies = {}
        for d in find_direct(out_stubbed):
            # fast mode: the real tensor went straight to its consumer(s); any real use here fails
            t = torch.empty(d.shape, dtype=d.dtype, device="meta")
            if d.requires_grad and grad_enabled:
                t.requires_grad_(True)
            t._smp_mi = d.mi
            dummies[d.mi] = t
        rg_idx = [s.index for s in stubs if s.requires_grad] if grad_enabled else []
        if rg_idx:
            tensors = list(tensors)
            ins = []
            for i in rg_idx:
                t = tensors[i].detach()
                t.requires_grad_(True)
                ins.append(t)
            wrapped = RemoteOutput.apply(self, holder, out_key, mb, *ins)
            self._mb(mb).entries[("rout", out_key)] = _Entry(list(wrapped), holder, ("out", out_key), False)
            for i, w in zip(rg_idx, wrapped):
                tensors[i] = w
            if self._cur_worker is not None:
                self._cur_worker.routs.append((wrapped[0], producer, sent))
        for st_ in stubs:
            if st_.mi is not None:
                if not isinstance(tensors, list):
                    tensors = list(tensors)
                tensors[st_.index]._smp_mi = st_.mi
        return unstubify(out_stubbed, tensors, dummies)

    def _exec_fwd(self, src, msg, tensors):
        _, rid, mb, target, stubbed, reply_to, result_id, grad_enabled, mi_base = msg
        st = self.state
        st.microbatch = mb
        torch.set_grad_enabled(grad_enabled)
        _, stubs = _stubs_of(stubbed)
        tensors = list(tensors)
        dvals = self._resolve_direct(stubbed, mb, rid, grad_enabled)
        leaves, leaf_idx = [], []
        if grad_enabled:
            for s in stubs:
                if s.requires_grad:
                    t = tensors[s.index].detach()
                    t.requires_grad_(True)
                    tensors[s.index] = t
                    leaves.append(t)
                    leaf_idx.append(s.index)
            if leaves:
                self._mb(mb).leaves[rid] = (leaves, src)
                self._mb(mb).entries[("in", rid)] = _Entry(leaves, src, ("in", rid), True)
        args, kwargs = unstubify(stubbed, tensors, dvals)
        mm = st.module_manager
        if target[0] == "module":
            module = mm.get_module(target[1])
            out = st.model._call_local(module, args, kwargs)
            if grad_enabled:
                self.validate_frame(target[1], out, leaves, leaf_idx)
            self._send_result(reply_to, result_id, mb, out, rid, grad_enabled, mi_base)
        else:
            seq = mm.get_module(target[1])
            h = self.run_chain(seq, target[2], args[0], reply_to, result_id, mb, rid, grad_enabled, mi_base)
            if grad_enabled:
                self.validate_frame(f"{target[1]}[{target[2]}:]", h, leaves, leaf_idx)

    def _resolve_direct(self, stubbed, mb, rid, grad_enabled):
        """Consumer side of fast mode: the tensors a request names by DirectStub, waiting for
        any that has not arrived yet.  A tensor from another stage becomes a leaf whose
        gradient goes straight back to its producer."""
        directs = find_direct(stubbed)
        if not directs:
            return None
        me = self.core.rank()
        out = {}
        for d in directs:
            ent = self._direct_in.get((mb, d.mi))
            while ent is None:
                self._suspend(("dtx", mb, d.mi))
                ent = self._direct_in.get((mb, d.mi))
            t, prod, prid = ent
            if prod != me and grad_enabled and d.requires_grad:
                leaf = t.detach()
                leaf.requires_grad_(True)
                self._mb(mb).dleaves.setdefault(rid, []).append((leaf, prod, ("dout", prid, d.mi)))
                self._mb(mb).entries[("dout", rid, d.mi)] = _Entry([leaf], prod, ("dout", prid, d.mi), True)
                t = leaf
            out[d.mi] = t
        return out

    def validate_frame(self, name, out, leaves=(), leaf_idx=()):
        """Graph validation (reference `patches/execution.py:57-72`): every result of a
        remote module obtained while executing this frame (a remote request, or the main
        module on pp_rank 0) and every input that requires grad must have an autograd path
        to the frame's outputs -- else ``MissingPathFromComputationToModuleOutputError`` /
        ``MissingPathFromModuleInputToModuleOutputError``.  The reference must refuse such
        graphs (its backward would wait forever for the missing requests); this engine can
        run them -- an unused path simply receives no gradient, as without pipelining -- so
        ``SMP_SKIP_GRAPH_VALIDATION=1`` turns the check off and executes them.  The walk is
        native (``graph_reaches`` over torch::autograd::Node edges)."""
        w = self._cur_worker
        routs = w.routs if w is not None else []
        if w is not None:
            w.routs = []
        if not (routs or leaves) or os.environ.get("SMP_SKIP_GRAPH_VALIDATION", "0").lower() in ("1", "true"):
            return
        from ..ops._ext import ext

        _, tensors = stubify(out)
        roots = [t for t in tensors if t.requires_grad]
        if not roots:
            return  # outputs without grad: nothing flows back, as in the reference (execution.py:131-135)
        targets = [r[0] for r in routs] + list(leaves)
        # a reached remote result continues the walk at the tensors sent in that call (the
        # remote side validates its own inputs -> outputs path)
        hit = ext().graph_reaches(roots, targets, [list(r[2]) for r in routs])
        for (_, producer, _), ok in zip(routs, hit):
            if not ok:
                raise MissingPathFromComputationToModuleOutputError(name, producer)
        for idx, ok in zip(leaf_idx, hit[len(routs):]):
            if not ok:
                raise MissingPathFromModuleInputToModuleOutputError(name, idx)

    def begin_root_frame(self):
        if self._cur_worker is not None:
            self._cur_worker.routs = []

    def run_chain(self, seq, start, h, reply_to, result_id, mb, rid, grad_enabled, mi_base=None):
        """Execute seq's children from `start` while they are local; hand the rest to the
        next stage directly (child-to-child)."""
        mm = self.state.module_manager
        children = list(seq)  # iter(Sequential) keeps repeated modules; children() dedups them
        me = self.core.pp_rank()
        i = start
        j = i
        while j < len(children) and mm.get_partition(children[j]) == me:
            j += 1
        h = self.state.model._run_local_chain(seq, children, i, j, h)
        if j == len(children):
            self._send_result(reply_to, result_id, mb, h, rid, grad_enabled, mi_base)
            return h
        nxt = self._pp_peer(mm.get_partition(children[j]))
        rid2 = self._new_id()
        stubbed, tensors = stubify(((h,), {}))
        if grad_enabled:
            sent = [t for t in tensors if t.requires_grad]
            if sent:
                self._mb(mb).sent[rid2] = sent
                self._register_source(mb, ("in", rid2), sent)
        self.state.transport.send(
            nxt,
            ("fwd", rid2, mb, ("chain", mm.get_module_name(seq), j), stubbed, reply_to, result_id, grad_enabled,
             mi_base),
            tensors,
        )
        return h

    def _send_result(self, reply_to, result_id, mb, out, rid, grad_enabled, mi_base=None):
        if mi_base is None:
            stubbed, tensors = stubify(out)
        else:
            stubbed, tensors = self._stubify_result(reply_to, mb, out, rid, grad_enabled, mi_base)
        if grad_enabled:
            rg = [t for t in tensors if t.requires_grad]
            if rg:
                self._mb(mb).out[rid] = rg
                self._register_source(mb, ("out", rid), rg)
        msg = ("res", result_id, mb, stubbed, self.core.rank(), rid, grad_enabled)
        if reply_to == self.core.rank():
            # local delivery (a chain came back to its requester's stage): queue it for the
            # server loop -- a worker must never resume another worker directly.
            det = [t.detach() for t in tensors]
            self._local_q.append((result_id, (stubbed, det, self.core.rank(), rid)))
        else:
            self.state.transport.send(reply_to, msg, tensors)

    def _stubify_result(self, reply_to, mb, out, rid, grad_enabled, mi_base):
        """Fast mode, producer side: outputs tagged with their module info; once the consumer
        maps are merged, an output consumed only by OTHER children goes straight to them
        ("dtx") and the parent gets a DirectStub (reference `serialization.py:365-473`)."""
        fm, _, using = self._fm()
        order = {id(t): k for k, t in enumerate(iter_tensors(out))}
        direct_to = {}
        if using:
            parent_pp = self.core.ranker.get_pp_rank(reply_to)
            my_pp = self.core.pp_rank()
            for t in iter_tensors(out):
                mi = (mi_base, order[id(t)])
                cons = fm.map.get(mi)
                if cons and all(c[0] != parent_pp for c in cons):
                    # every consuming call on another stage detaches its own leaf and sends
                    # one "dout" backward; a call on this stage uses the tensor itself, so
                    # its gradient flows inside that call's own segment
                    n_remote = sum(1 for c in cons if c[0] != my_pp)
                    direct_to[id(t)] = (mi, sorted({c[0] for c in cons}), n_remote)

        def direct(t):
            d = direct_to.get(id(t))
            return None if d is None else DirectStub(d[0], t.shape, t.dtype, t.requires_grad)

        stubbed, tensors = stubify(out, direct if direct_to else None)
        _, stubs = _stubs_of(stubbed)
        for st_ in stubs:
            st_.mi = (mi_base, order[id(tensors[st_.index])])
        if direct_to:
            me = self.core.rank()
            s = self._mb(mb)
            for t in iter_tensors(out):
                d = direct_to.get(id(t))
                if d is None:
                    continue
                mi, pps, n_remote = d
                if grad_enabled and t.requires_grad:
                    s.out_direct[(rid, mi)] = [t]
                    # one expected backward segment per remote consuming call (ADVICE r3:
                    # one per tensor let PP+DDP launch a bucket after the first of two douts,
                    # and a same-stage consumer's count was never reached)
                    self._register_source(mb, ("dout", rid, mi), [t], n_remote)
                for pp in pps:
                    dst = self._pp_peer(pp)
                    if dst == me:
                        self._direct_in[(mb, mi)] = (t, me, rid)
                    else:
                        self.state.transport.send(dst, ("dtx", mb, mi, rid), [t])
        return stubbed, tensors

    # --------------------------------------------------------------- backward
    def backward_root(self, tensors, grads):
        """model.backward() on pp_rank 0 inside a microbatch worker."""
        self.fm_note_local(list(tensors))
        mb = self.state.microbatch
        # register the loss segment before the scheduler marks this microbatch's forward
        # done: the last microbatch's mark must never see an incomplete expected count
        self._register_source(mb, ("root",), [t for t in tensors if t.requires_grad])
        self._suspend(("bwd_start", mb))
        tid = self._new_token(None, None, mb)
        self._root_tokens[mb] = tid
        self._run_backward(tid, mb, tensors, grads, ("root",))
        self._maybe_finish(tid)
        if not self.tokens.get(tid, _DONE).done:
            self._suspend(("bwd_done", mb))

    def _new_token(self, ack_to, remote_token, mb):
        tid = next(self._ids)
        self.tokens[tid] = _Token(ack_to, remote_token, mb)
        return tid

    def _send_bwd(self, holder, key, mb, grads):
        parent = self._cur_token
        if parent is None:
            raise PipelineParallelBWDError("remote backward outside of a tracked backward segment")
        self.tokens[parent].pending += 1
        self._send(holder, ("bwd", key, mb, grads, parent))

    def _register_source(self, mb, skey, tensors, waves=1):
        """A saved segment whose backward will run `waves` times this microbatch (one per
        gradient message, or the loss): the GradTracker expects the accumulations it
        reaches, and every gradient entry it reaches waits for those waves."""
        if not tensors:
            return
        for _ in range(waves):
            self.state.model._track_segment(tensors)
        s = self._mb(mb)
        targets, owners = [], []
        for e in s.entries.values():
            for t in e.targets:
                targets.append(t)
                owners.append(e)
        reached = []
        if targets:
            from ..ops._ext import ext

            hit = ext().graph_reaches(list(tensors), targets, [])
            seen = set()
            for h, e in zip(hit, owners):
                if h and id(e) not in seen:
                    seen.add(id(e))
                    reached.append(e)
                    e.pending += waves
        s.reach[skey] = reached

    def _entry_grads(self, mb, eid, dst, key, grads):
        """RemoteOutput backward: accumulate the output gradients of one wave (sent at the
        end of the last wave that reaches the entry)."""
        e = self._mb(mb).entries.get(eid)
        if e is None:  # not tracked (should not happen): send right away
            self._send_bwd(dst, key, mb, list(grads))
            return
        if e.grads is None:
            e.grads = list(grads)
        else:
            e.grads = [a if b is None else (b if a is None else a + b) for a, b in zip(e.grads, grads)]

    def _wave_done(self, mb, skey):
        s = self.mbstate.get(mb)
        if s is None:
            return
        for e in s.reach.get(skey, ()):
            e.pending -= 1
        for e in s.entries.values():
            if e.pending > 0:
                continue
            gs = e.take()
            if not e.flushed:
                e.flushed = True
                self._send_bwd(e.dst, e.key, mb, gs if gs is not None else [None] * len(e.targets))
            elif gs is not None:  # a wave the counts did not foresee: never drop gradients
                self._send_bwd(e.dst, e.key, mb, gs)

    def _run_backward(self, tid, mb, tensors, grads, skey):
        pairs = [(t, g) for t, g in zip(tensors, grads) if g is not None and t.requires_grad]
        prev = self._cur_token
        self._cur_token = tid
        try:
            if pairs:
                with torch.enable_grad():
                    torch.autograd.backward([t for t, _ in pairs], [g for _, g in pairs], retain_graph=True)
            self._wave_done(mb, skey)
        finally:
            self._cur_token = prev

    def _process_bwd(self, src, key, mb, grads, remote_token):
        s = self._mb(mb)
        kind, rid = key[0], key[1]
        if kind == "dout":  # fast mode: a consumer's gradient for an output sent child-to-child
            saved = s.out_direct.get((rid, key[2]))
        else:
            saved = s.sent.get(rid) if kind == "in" else s.out.get(rid)
        if saved is None:
            raise PipelineParallelBWDError(f"no saved tensors for {key} (mb {mb}) on rank {self.core.rank()}")
        tid = self._new_token(src, remote_token, mb)
        self.state.microbatch = mb
        self.state.model._step_had_backward = True
        self._run_backward(tid, mb, saved, grads, tuple(key))
        self._maybe_finish(tid)

    def _ack(self, tid):
        t = self.tokens[tid]
        t.pending -= 1
        self._maybe_finish(tid)

    def _maybe_finish(self, tid):
        t = self.tokens[tid]
        if t.pending > 0 or t.done:
            return
        t.done = True
        del self.tokens[tid]
        if t.ack_to is not None:
            self._send(t.ack_to, ("ack", t.remote_token))
        else:
            w = self.waiting.pop(("bwd_done", t.mb), None)
            if w is not None:
                self._resume(w, None)


class _DoneSentinel:
    done = True


_DONE = _DoneSentinel()


def _stubs_of(stubbed):
    from .serialization import TensorStub

    found = []

    def walk(o, memo):
        if isinstance(o, TensorStub):
            found.append(o)
            return
        oid = id(o)
        if oid in memo:
            return
        memo.add(oid)
        if isinstance(o, (list, tuple, set)):
            for x in o:
                walk(x, memo)
        elif isinstance(o, dict):
            for x in o.values():
                walk(x, memo)
        elif hasattr(o, "__dict__") and not isinstance(o, type):
            for x in vars(o).values():
                walk(x, memo)

    walk(stubbed, set())
    uniq = {s.index: s for s in found}
    return stubbed, [uniq[i] for i in sorted(uniq)]
