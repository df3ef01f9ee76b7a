"""Process topology, native runtime bring-up and coordinated shutdown.

Reference parity: `smp/backend/core.py:165-562` (rank/size/group queries, world-size
validation, ExitHook, shutdown on exit).  MPI is replaced by the launcher environment
(``torchrun``: RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE) and the native mailbox
is wired up through a key-value store rendezvous (the torch.distributed TCPStore).
"""
import atexit
import faulthandler
import os
import socket
import sys
import threading
import time

from .collectives import CollectiveCommunicator, CommGroup
from .exceptions import InvalidEnvironmentError, NotInitializedError, WorkerSizeError
from .logger import get_logger
from .native import runtime
from .topology import Ranker

logger = get_logger()


class ExitHook:
    """Intercepts sys.exit/excepthook so shutdown can report a consistent status
    (reference `core.py:165-188`)."""

    def __init__(self):
        self.exit_code = None
        self.exception = None
        self._orig_exit = None
        self._orig_excepthook = None

    def hook(self):
        self._orig_exit = sys.exit
        self._orig_excepthook = sys.excepthook
        sys.exit = self.exit
        sys.excepthook = self.exc_handler

    def unhook(self):
        if self._orig_exit is not None:
            sys.exit = self._orig_exit
            sys.excepthook = self._orig_excepthook

    def exit(self, code=0):
        self.exit_code = code
        self._orig_exit(code)

    def exc_handler(self, exc_type, exc, *args):
        self.exception = exc
        self._orig_excepthook(exc_type, exc, *args)


class Watchdog:
    """Failure detector (new relative to the reference, which waits forever -- SURVEY §5.3).

    A daemon thread blocks in the native ``Mailbox.wait_error`` (GIL released).  When a
    peer aborts or its process vanishes, receives on the mailbox already raise in the
    main thread; a rank stuck inside an RCCL/gloo collective cannot be interrupted, so
    after ``SMP_ABORT_GRACE_S`` seconds (default 60) the watchdog dumps every thread's
    stack and ends the process with exit code 1 instead of hanging the job.

    Step timeout: with ``SMP_STEP_TIMEOUT_S`` set, a ``@smp.step`` call running longer
    than that is treated as a hang: stacks are dumped, peers get ABORT, the process exits.
    """

    def __init__(self, core):
        self.core = core
        self.grace = float(os.environ.get("SMP_ABORT_GRACE_S", "60"))
        t = os.environ.get("SMP_STEP_TIMEOUT_S")
        self.step_timeout = float(t) if t else None
        self._step_started = None
        self._stop = False
        # hang diagnostics: callables returning one line of runtime state each (the pipeline
        # engine's pending waits, transport holds, mailbox queues), logged with the stacks
        self.diagnostics = []
        self._thread = threading.Thread(target=self._run, name="smp-watchdog", daemon=True)

    def start(self):
        self._thread.start()

    def stop(self):
        self._stop = True

    def join(self):
        # Joined before interpreter finalisation: a daemon thread returning from native
        # code (GIL released) into a finalising interpreter is torn down with a forced
        # unwind, which aborts the process.
        if self._thread.is_alive() and self._thread is not threading.current_thread():
            self._thread.join(timeout=5.0)

    def step_started(self):
        self._step_started = time.monotonic()
        if self.step_timeout is not None:
            # backstop for a main thread blocked in native code WITH the GIL (the watchdog
            # thread then cannot run): faulthandler's own C thread dumps every Python stack
            # without the GIL, 30 s after the watchdog should have fired, and exits
            try:
                faulthandler.dump_traceback_later(self.step_timeout + 30.0, exit=True)
            except Exception:  # pragma: no cover
                pass

    def step_finished(self):
        self._step_started = None
        if self.step_timeout is not None:
            try:
                faulthandler.cancel_dump_traceback_later()
            except Exception:  # pragma: no cover
                pass

    def dump_state(self):
        for fn in list(self.diagnostics):
            try:
                logger.error(f"[smp watchdog] rank {self.core._rank} state: {fn()}")
            except Exception as e:  # state read racing the main thread: report and go on
                logger.error(f"[smp watchdog] rank {self.core._rank} state unavailable: {e!r}")

    def _fatal(self, why):
        logger.error(f"[smp watchdog] rank {self.core._rank}: {why}; dumping stacks and exiting")
        self.dump_state()
        try:
            faulthandler.dump_traceback(all_threads=True)
        except Exception:  # pragma: no cover
            pass
        try:
            self.core.mailbox.shutdown(False)
        except Exception:  # pragma: no cover
            pass
        os._exit(1)

    def _run(self):
        mb = self.core.mailbox
        while not self._stop:
            err = mb.wait_error(1.0)
            if self._stop:
                return
            if err:
                logger.error(f"[smp watchdog] rank {self.core._rank}: peer failure: {err}")
                self.dump_state()  # what this rank was waiting for when the peer gave up
                deadline = time.monotonic() + self.grace
                while time.monotonic() < deadline:
                    if self._stop:
                        return
                    time.sleep(0.1)
                self._fatal(f"still running {self.grace:.0f}s after peer failure ({err})")
                return
            st = self._step_started
            if self.step_timeout is not None and st is not None and time.monotonic() - st > self.step_timeout:
                self._fatal(f"step exceeded SMP_STEP_TIMEOUT_S={self.step_timeout:g}s")
                return


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def _local_ip(master_addr):
    if master_addr in ("127.0.0.1", "localhost"):
        return "127.0.0.1"
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect((master_addr, 9))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return "127.0.0.1"


_INIT_GENERATION = [0]


def _next_init_generation():
    _INIT_GENERATION[0] += 1
    return _INIT_GENERATION[0]


class ModelParallelCore:
    def __init__(self):
        self.cfg = None
        self.ranker = None
        self.mailbox = None
        self.comm = None
        self.timeline = None
        self.exit_hook = None
        self.watchdog = None
        self._initialized = False
        self._rank = 0
        self._size = 1
        self._local_rank = 0
        self._local_size = 1

    # ----------------------------------------------------------- lifecycle
    @property
    def initialized(self):
        return self._initialized

    def read_environment(self):
        self._rank = _env_int("RANK", "OMPI_COMM_WORLD_RANK", default=0)
        self._size = _env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", default=1)
        self._local_rank = _env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", default=self._rank)
        self._local_size = _env_int("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", default=self._size)
        if self._rank >= self._size or self._local_rank >= self._local_size:
            raise InvalidEnvironmentError(
                f"inconsistent launcher environment: rank {self._rank}/{self._size}, "
                f"local {self._local_rank}/{self._local_size}"
            )

    def _validate_worker_size(self, cfg):
        pp, tp = cfg.pipeline_parallel_degree, cfg.tensor_parallel_degree
        if self._size % (pp * tp) != 0:
            raise WorkerSizeError(
                f"World size {self._size} must be divisible by pipeline_parallel_degree x "
                f"tensor_parallel_degree = {pp * tp}."
            )
        if cfg.zero2d_enabled():
            if self._size % cfg.sharded_data_parallel_degree != 0:
                raise WorkerSizeError(
                    f"World size {self._size} must be divisible by sharded_data_parallel_degree "
                    f"{cfg.sharded_data_parallel_degree}."
                )
        dp = self._size // pp
        if dp > 1 and not (cfg.ddp or cfg.horovod or cfg.zero2d_enabled()):
            raise WorkerSizeError(
                f"World size {self._size} implies data parallelism of degree {dp // tp}; enable 'ddp' in the config."
            )

    def initialize(self, cfg, store, device_count=None):
        """`store` is a torch.distributed Store shared by all ranks."""
        self.cfg = cfg
        self.read_environment()
        self._validate_worker_size(cfg)
        if device_count is not None and device_count > 0 and self._local_size > device_count:
            raise InvalidEnvironmentError(
                f"{self._local_size} processes on this node but only {device_count} GPUs are visible."
            )
        pp, tp = cfg.pipeline_parallel_degree, cfg.tensor_parallel_degree
        rdp = self._size // (pp * tp)
        self.ranker = Ranker(cfg.placement_strategy, rdp, pp, tp)

        rt = runtime()
        self.mailbox = rt.Mailbox(self._rank, self._size)
        host = _local_ip(os.environ.get("MASTER_ADDR", "127.0.0.1"))
        port = self.mailbox.listen("0.0.0.0" if host != "127.0.0.1" else "127.0.0.1")
        # keys are per init generation: after smp.reset() + smp.init() a peer must never
        # read the previous mailbox's address (every rank re-initialises the same times)
        gen = _next_init_generation()
        store.set(f"smp/mailbox/{gen}/{self._rank}", f"{host}:{port}")
        hosts, ports = [], []
        for r in range(self._size):
            h, p = store.get(f"smp/mailbox/{gen}/{r}").decode().rsplit(":", 1)
            hosts.append(h)
            ports.append(int(p))
        self.mailbox.connect(hosts, ports, float(os.environ.get("SMP_CONNECT_TIMEOUT", "300")))
        self.comm = CollectiveCommunicator(self, self.mailbox)

        self.timeline = rt.Timeline(self._rank)
        tl = os.environ.get("SMP_TIMELINE_FILE")
        if tl:
            self.timeline.set_output(tl.replace("{rank}", str(self._rank)))

        if cfg.zero2d_enabled():
            cfg.construct_zero2d_config_dict(self)

        self.exit_hook = ExitHook()
        self.exit_hook.hook()
        atexit.register(self.shutdown)
        self.watchdog = Watchdog(self)
        self.watchdog.start()
        self._initialized = True

    def shutdown(self):
        if not self._initialized:
            return
        self._initialized = False
        success = True
        if self.exit_hook is not None:
            success = self.exit_hook.exception is None and self.exit_hook.exit_code in (None, 0)
            self.exit_hook.unhook()
        try:
            if self.timeline is not None:
                self.timeline.flush()
            if self.watchdog is not None:
                self.watchdog.stop()
            if self.mailbox is not None:
                if success:
                    self.mailbox.flush()
                self.mailbox.shutdown(success)
            if self.watchdog is not None:
                self.watchdog.join()
        except Exception as e:  # pragma: no cover - best effort at exit
            logger.debug(f"shutdown: {e}")

    def _check(self):
        if not self._initialized:
            raise NotInitializedError()

    # ------------------------------------------------------------- queries
    def rank(self):
        return self._rank

    def size(self):
        return self._size

    def local_rank(self):
        return self._local_rank

    def local_size(self):
        return self._local_size

    def pp_rank(self):
        return self.ranker.get_pp_rank(self._rank)

    def tp_rank(self):
        return self.ranker.get_tp_rank(self._rank)

    def rdp_rank(self):
        return self.ranker.get_rdp_rank(self._rank)

    def dp_rank(self):
        return self.ranker.get_dp_rank(self._rank)

    def mp_rank(self):
        return self.ranker.get_mp_rank(self._rank)

    def pp_size(self):
        return self.ranker.size_map["P"]

    def tp_size(self):
        return self.ranker.size_map["T"]

    def rdp_size(self):
        return self.ranker.size_map["D"]

    def dp_size(self):
        return self.ranker.size_map["D"] * self.ranker.size_map["T"]

    def mp_size(self):
        return self.ranker.size_map["P"] * self.ranker.size_map["T"]

    def get_pp_group(self):
        return self.ranker.get_pp_group(self._rank)

    def get_tp_group(self):
        return self.ranker.get_tp_group(self._rank)

    def get_rdp_group(self):
        return self.ranker.get_rdp_group(self._rank)

    def get_dp_group(self):
        return self.ranker.get_dp_group(self._rank)

    def get_mp_group(self):
        return self.ranker.get_mp_group(self._rank)

    def get_group_ranks(self, group):
        if group == CommGroup.WORLD:
            return list(range(self._size))
        return {
            CommGroup.PP_GROUP: self.get_pp_group,
            CommGroup.TP_GROUP: self.get_tp_group,
            CommGroup.RDP_GROUP: self.get_rdp_group,
            CommGroup.DP_GROUP: self.get_dp_group,
            CommGroup.MP_GROUP: self.get_mp_group,
        }[group]()

    def pp_rank_to_rank(self, pp_rank):
        return self.ranker.translate(pp_rank, self.tp_rank(), self.rdp_rank())

    def is_in_same_instance(self, other_rank):
        return (other_rank // self._local_size) == (self._rank // self._local_size)

    def instance_id(self):
        return self._rank // self._local_size

    def barrier(self):
        self.comm.barrier(CommGroup.WORLD)

    # ------------------------------------------------------------ metrics
    def get_and_reset_memory_metrics(self):
        """Reference `smp_get_and_reset_memory_metrics` (`smp/backend/core.py:538-550`):
        receive-pool peak allocated/reserved and device free/total memory, in MB.  The
        pipeline's receive buffers live in the caching allocator here (no separate D2D
        pool), so its peaks are the allocator's; free/total come from hipMemGetInfo.
        Peaks are reset."""
        import torch

        out = {"d2d_peak_allocated_mb": 0.0, "d2d_peak_reserved_mb": 0.0, "gpu_free_mb": 0.0, "gpu_total_mb": 0.0}
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            dev = torch.cuda.current_device()
            out["d2d_peak_allocated_mb"] = torch.cuda.max_memory_allocated(dev) / 2**20
            out["d2d_peak_reserved_mb"] = torch.cuda.max_memory_reserved(dev) / 2**20
            free, total = torch.cuda.mem_get_info(dev)
            out["gpu_free_mb"], out["gpu_total_mb"] = free / 2**20, total / 2**20
            torch.cuda.reset_peak_memory_stats(dev)
        return out

    def get_and_reset_alloc_metrics(self):
        """Reference `smp_get_and_reset_alloc_metrics` (`core.py:552-562`): allocation
        success / failure counters since the last call (allocator retries and OOMs count
        as failures), plus control-plane message counts of the native mailbox."""
        import torch

        out = {"alloc_success": 0, "alloc_fail": 0}
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            st = torch.cuda.memory_stats()
            allocs = st.get("allocation.all.allocated", 0)
            fails = st.get("num_alloc_retries", 0) + st.get("num_ooms", 0)
            prev = getattr(self, "_alloc_prev", (0, 0))
            out["alloc_success"], out["alloc_fail"] = allocs - prev[0], fails - prev[1]
            self._alloc_prev = (allocs, fails)
        if self.mailbox is not None:
            ms = self.mailbox.stats()
            out.update(msgs_sent=ms.msgs_sent, msgs_recv=ms.msgs_recv, bytes_sent=ms.bytes_sent,
                       bytes_recv=ms.bytes_recv)
        return out

    def timeline_start_step(self, step):
        if self.watchdog is not None:
            self.watchdog.step_started()
        if self.timeline is not None:
            self.timeline.start_step(step)

    def timeline_end_step(self):
        if self.watchdog is not None:
            self.watchdog.step_finished()
        if self.timeline is not None:
            self.timeline.end_step()

    def timeline_record_pipeline_event(self, mb, label):
        if self.timeline is not None and self.timeline.enabled:
            self.timeline.mark(mb, label)

