"""``smp.DistributedOptimizer``.

Reference parity (`smp/torch/optimizers/optimizer.py:437-549`, `fp16/fp16.py`): wraps any
torch optimizer; with fp16/bf16 keeps fp32 master weights (Bit16_Optimizer semantics),
unscales fp16 gradients with a static or dynamic loss scale and skips overflowing steps
(overflow decision shared across the model-parallel group), ``clip_master_grads``
(global L2 norm across model-parallel ranks), optimizer-state sharding
(``shard_optimizer_state``: each data-parallel rank updates only its slice, then
parameters are all-gathered), local/full state dicts, param name <-> index maps.

MI355X design: the optimizer works on *domains* -- contiguous ranges of the model's flat
parameter/gradient buffers (`parallel/flat.py`), one per gradient bucket (or this rank's
chunk of each bucket when sharded).  For Adam/AdamW/SGD/Adagrad/LAMB the whole update
(unscale + clip + moment update + fp32 master update + low-precision param write-back)
is ONE fused HIP kernel per domain.  Any other torch optimizer runs through the same
domains as fp32 "virtual parameters" (the reference's name for sharded master slices).
"""
import os

import torch
import torch.distributed as dist

from ..backend.exceptions import SMPInvalidArgumentError
from ..backend.logger import get_logger
from ..ops import multi_tensor as mt
from ..torch.state_mod import state
from .loss_scaler import DynamicLossScaler, LossScaler, any_overflow

logger = get_logger()


def _kind_of(opt):
    name = type(opt).__name__
    if name in ("AdamW",):
        return "adamw"
    if name in ("Adam",):
        return "adamw" if opt.defaults.get("decoupled_weight_decay", False) else "adam"
    if name == "FusedAdam":
        return "adamw" if getattr(opt, "adam_w_mode", True) else "adam"
    if name == "SGD" or name == "FusedSGD":
        return "sgd"
    if name == "Adagrad" or name == "FusedAdagrad":
        return "adagrad"
    if name == "FusedLAMB":
        return "lamb"
    return "generic"


class _Domain:
    __slots__ = ("key", "start", "end", "group_index", "master", "m", "v", "upd", "vparam", "params", "_lamb_chunks")

    def __init__(self, key, start, end, group_index, params):
        self.key, self.start, self.end, self.group_index, self.params = key, start, end, group_index, params
        self.master = self.m = self.v = self.upd = self.vparam = None

    @property
    def numel(self):
        return self.end - self.start


class _Staged:
    """A domain whose master/m/v are temporarily the HBM staging views."""

    def __init__(self, d, master, m, v):
        self.key, self.start, self.end, self.group_index, self.params = d.key, d.start, d.end, d.group_index, d.params
        self.master, self.m, self.v, self.upd, self.vparam = master, m, v, None, None


def _pinned_full(n, fill):
    """fp32 host array of exactly n elements, page-locked in place (hipHostRegister) so the
    offload streams copy at PCIe rate without the pinned allocator's power-of-two rounding."""
    import weakref

    from ..ops._ext import ext

    t = torch.full((n,), float(fill), dtype=torch.float32)
    if n:
        ext().host_register(t)
        weakref.finalize(t, ext().host_unregister_ptr, t.data_ptr())
    return t


class DistributedOptimizer(torch.optim.Optimizer):
    """The wrapped optimizer.  A ``torch.optim.Optimizer`` by type (the base class's ``__init__``
    is not run: param_groups / defaults / state are the inner optimizer's), so code that checks
    the type -- ``torch.optim.lr_scheduler`` schedulers, Hugging Face / accelerate training loops --
    takes it; the reference returns the user's optimizer object itself with patched methods
    (`torch/optimizers/optimizer.py:437-520`)."""

    def __init__(self, optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None):
        if state.model is None:
            raise SMPInvalidArgumentError("create smp.DistributedModel before smp.DistributedOptimizer")
        self.optimizer = optimizer
        model = state.model
        model_params = set(model.module.parameters())
        for g in optimizer.param_groups:
            for p in g["params"]:
                if p not in model_params:
                    raise SMPInvalidArgumentError("optimizer contains a parameter that is not part of the model")
        self._orig_param_groups = [dict(g, params=list(g["params"])) for g in optimizer.param_groups]
        cfg = state.cfg
        self.fp16 = cfg.fp16 or cfg.fp16_params
        self.bf16 = cfg.bf16
        if self.fp16:
            self.loss_scaler = DynamicLossScaler(**(dynamic_loss_args or {})) if dynamic_loss_scale else \
                LossScaler(static_loss_scale)
        else:
            self.loss_scaler = LossScaler(1.0)
        self.kind = _kind_of(optimizer)
        if self.kind == "lamb" and cfg.zero2d_enabled():
            raise SMPInvalidArgumentError("FusedLAMB is not supported with sharded data parallelism")
        self.domains = []
        self._step_count = [0] * len(optimizer.param_groups)
        self._clip_coef = None
        self._built = False
        self.overflow = False
        self.offload = bool(getattr(cfg, "amd_offload_optimizer_state", False)) and state.use_gpu
        if self.offload and self.kind not in ("adam", "adamw", "sgd", "adagrad"):
            raise SMPInvalidArgumentError("amd_offload_optimizer_state supports Adam/AdamW/SGD/Adagrad")
        # which fp32 fields live in pinned host memory (SMP_OFFLOAD_OPTIMIZER_FIELDS, default
        # all three): e.g. "m,v" keeps the master weights in HBM and moves 8 B/param to the host
        fields = os.environ.get("SMP_OFFLOAD_OPTIMIZER_FIELDS", "master,m,v")
        self._offload_fields = {f.strip() for f in fields.split(",") if f.strip()} if self.offload else set()
        if not self._offload_fields <= {"master", "m", "v"}:
            raise SMPInvalidArgumentError(f"SMP_OFFLOAD_OPTIMIZER_FIELDS: unknown field in {fields!r}")
        self._offload = None
        state.optimizer = self
        if model.partitioned:
            self._on_model_partitioned()
        if state.loaded_optimizer_state is not None:
            self._deferred_load = state.loaded_optimizer_state
        else:
            self._deferred_load = None

    # ----------------------------------------------------------------- props
    @property
    def loss_scale(self):
        return self.loss_scaler.loss_scale

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def defaults(self):
        return self.optimizer.defaults

    # torch names of the fused kernels' per-parameter moments
    _TORCH_STATE_NAMES = {"adam": {"m": "exp_avg", "v": "exp_avg_sq"}, "adamw": {"m": "exp_avg", "v": "exp_avg_sq"},
                          "lamb": {"m": "exp_avg", "v": "exp_avg_sq"}, "sgd": {"m": "momentum_buffer"},
                          "adagrad": {"v": "sum"}}

    @property
    def state(self):
        """``optimizer.state[param]`` as torch names it (``exp_avg`` / ``exp_avg_sq`` / ``step``,
        ``momentum_buffer``, ``sum``): views of the flat fp32 state for every parameter held whole
        by this rank, so reads and in-place edits reach the fused optimizer.  Parameters split
        across shards (shard_optimizer_state) are absent; the generic path keeps the inner
        optimizer's own state."""
        names = self._TORCH_STATE_NAMES.get(self.kind)
        if names is None or state.model is None:
            return self.optimizer.state
        from collections import defaultdict

        out = defaultdict(dict)
        for d in self.domains:
            flat = state.model.flat_groups[d.key]
            for p in d.params:
                off, n = flat.offsets[p], p.numel()
                if off < d.start or off + n > d.end:
                    continue
                lo = off - d.start
                entry = {"step": torch.tensor(float(self._step_count[d.group_index]))}
                for k, tname in names.items():
                    t = getattr(d, k)
                    if t is not None:
                        entry[tname] = t[lo:lo + n].view(p.shape)
                out[p] = entry
        return out

    # ----------------------------------------------------------------- build
    def _on_model_partitioned(self):
        model = state.model
        if not self._built:
            model._relayout_for_optimizer([g["params"] for g in self._orig_param_groups])
        self._build_domains()
        self._built = True
        if getattr(self, "_deferred_load", None) is not None:
            self.load_state_dict(self._deferred_load)
            self._deferred_load = None
            state.loaded_optimizer_state = None

    def _group_index_of(self):
        idx = {}
        for gi, g in enumerate(self._orig_param_groups):
            for p in g["params"]:
                idx.setdefault(p, gi)
        return idx

    def _build_domains(self):
        model = state.model
        gidx = self._group_index_of()
        self.domains = []
        lowp = self.fp16 or self.bf16
        for key, flat in model.flat_groups.items():
            red = model.reducers[key]
            for b in flat.buckets:
                gis = {gidx.get(p, 0) for p in b.params}
                gi = min(gis)
                if red.shard and red.group_size > 1:
                    s, e = red.shard_range(b)
                else:
                    s, e = b.start, b.end
                d = _Domain(key, s, e, gi, b.params)
                gdev = flat.data.device
                cpu = torch.device("cpu")
                off = self._offload_fields
                if "master" in off:
                    # pinned host copy; the low-precision params stay in HBM
                    d.master = _pinned_full(e - s, 0.0)
                    d.master.copy_(flat.data[s:e].float())
                elif lowp or flat.data.dtype != torch.float32:
                    d.master = flat.data[s:e].float().clone()
                else:
                    d.master = flat.data[s:e]  # fp32 model: the parameters are the master copy

                def state_buf(field, fill=0.0):
                    if field in off:
                        return _pinned_full(e - s, fill)
                    return torch.full((e - s,), float(fill), dtype=torch.float32, device=gdev)

                if self.kind in ("adam", "adamw", "lamb"):
                    d.m = state_buf("m")
                    d.v = state_buf("v")
                elif self.kind in ("sgd",):
                    d.m = state_buf("m")
                elif self.kind == "adagrad":
                    d.v = state_buf("v", self.optimizer.param_groups[gi].get("initial_accumulator_value", 0.0))
                if self.kind == "lamb":
                    d.upd = torch.empty(e - s, dtype=torch.float32, device=gdev)
                self.domains.append(d)
        if self.offload:
            from .offload import OptimizerStateOffload

            self._offload = OptimizerStateOffload(self.domains, state.device)
        if self.kind == "generic":
            # inner optimizer sees fp32 virtual parameters (one per domain)
            groups = [[] for _ in self.optimizer.param_groups]
            for d in self.domains:
                vp = torch.nn.Parameter(d.master, requires_grad=True)
                d.vparam = vp
                groups[d.group_index].append(vp)
            self.optimizer.state.clear()
            for gi, g in enumerate(self.optimizer.param_groups):
                g["params"] = groups[gi]

    def virtual_named_parameters(self):
        for i, d in enumerate(self.domains):
            yield f"{d.key}/domain{i}", d.vparam if d.vparam is not None else d.master

    # ------------------------------------------------------------------ step
    def zero_grad(self, set_to_none=False):
        model = state.model
        for flat in model.flat_groups.values():
            flat.zero_grad()
        if self.kind == "generic":
            for d in self.domains:
                if d.vparam is not None:
                    d.vparam.grad = None

    def _grad_range(self, d):
        return state.model.flat_groups[d.key].grad[d.start:d.end]

    def _param_range(self, d):
        return state.model.flat_groups[d.key].data[d.start:d.end]

    def _model_parallel_group(self):
        cfg = state.cfg
        if cfg.shard_optimizer_state or cfg.zero2d_enabled():
            return state.pgs.world
        return state.pgs.mp

    def _check_overflow(self):
        """Skip-step decision shared by every rank whose gradients differ: the model-parallel
        group, or the whole world when the gradients are sharded (optimizer-state sharding,
        sharded data parallelism) -- otherwise one shard's inf would make only its rank skip
        the step and halve its loss scale, and shards / scales would diverge."""
        grads = [self._grad_range(d) for d in self.domains]
        sharded = state.cfg.shard_optimizer_state or state.sdp is not None
        group = state.pgs.world if sharded else (self._model_parallel_group() if state.core.mp_size() > 1 else None)
        return any_overflow(grads, group)

    @staticmethod
    def _materialize_grads():
        """Sharded data parallelism zeroes gradient shards lazily (``_ShardFlat.zero_grad``):
        make sure no shard is read before its zero fill when a step ran no reduction."""
        model = state.model
        for flat in (model.flat_groups.values() if model is not None else ()):
            fill = getattr(flat, "fill_fresh", None)
            if fill is not None:
                fill()

    def clip_master_grads(self, max_norm, norm_type=2):
        """Global L2 norm of the (unscaled) gradients across all ranks holding distinct
        gradients; records the clip coefficient applied inside the next step."""
        if norm_type != 2:
            raise SMPInvalidArgumentError("only L2 norm clipping is supported")
        self._materialize_grads()
        dev = state.device
        acc = torch.zeros(1, dtype=torch.float32, device=dev)
        core = state.core
        inv = 1.0 / self.loss_scale
        for d in self.domains:
            # replicated (non-TP) params are identical on every tp_rank: count them once
            if d.key == "default" and core.tp_size() > 1 and core.tp_rank() != 0 and not state.cfg.shard_optimizer_state:
                continue
            mt.sumsq(self._grad_range(d), acc, scale=inv)
        if state.sdp is not None:
            # every replica holds identical reduced shards: the norm spans one shard group
            if state.pgs.shard is not None:
                dist.all_reduce(acc, group=state.pgs.shard)
        elif state.cfg.shard_optimizer_state and core.dp_size() > 1:
            dist.all_reduce(acc, group=state.pgs.world)
        elif core.mp_size() > 1:
            dist.all_reduce(acc, group=state.pgs.mp)
        norm = acc.sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        self._clip_coef = coef
        return norm

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._materialize_grads()
        if state.sdp is not None and self._clip_coef is None and state.cfg.sdp_gradient_clipping > 0:
            # sharded data parallelism clips to sdp_gradient_clipping on every step (the
            # DeepSpeed `gradient_clipping` the reference configures, zero_config.py)
            self.clip_master_grads(state.cfg.sdp_gradient_clipping)
        inv_scale = 1.0 / self.loss_scale
        if self.fp16:
            self.overflow = self._check_overflow()
            if self.loss_scaler.dynamic:
                self.loss_scaler.update_scale(self.overflow)
            if self.overflow:
                logger.info(f"gradient overflow: skipping step, loss scale -> {self.loss_scale}")
                self._clip_coef = None
                return loss
        gscale = inv_scale
        if self._clip_coef is not None:
            # one scalar host read per step (the coefficient is already all-reduced)
            gscale = gscale * float(self._clip_coef.item())
            self._clip_coef = None
        lowp = self.fp16 or self.bf16
        for gi in range(len(self.optimizer.param_groups)):
            self._step_count[gi] += 1
        if self.kind == "generic":
            self._generic_step(gscale, lowp)
        elif self._offload is not None:
            self._offload.run(self.domains, lambda d, st: self._fused_step(d, gscale, lowp, st))
        else:
            for d in self.domains:
                self._fused_step(d, gscale, lowp)
        self._allgather_shards()
        return loss

    def _hp(self, gi):
        return self.optimizer.param_groups[gi]

    def _fused_step(self, d, gscale, lowp, staged=None):
        """One fused update of domain d; ``staged`` = HBM (master, m, v) copies when the
        optimizer state lives in host memory (`optimizers/offload.py`)."""
        if staged is not None:
            d = _Staged(d, *staged)
        g = self._hp(d.group_index)
        step = self._step_count[d.group_index]
        grad = self._grad_range(d)
        plow = self._param_range(d) if (lowp or d.master.data_ptr() != self._param_range(d).data_ptr()) else None
        lr = float(g["lr"])
        wd = float(g.get("weight_decay", 0.0))
        if self.kind in ("adam", "adamw"):
            b1, b2 = g.get("betas", (0.9, 0.999))
            mt.fused_adam_(plow, grad, d.master, d.m, d.v, lr, float(b1), float(b2), float(g.get("eps", 1e-8)), wd,
                           step, gscale, adamw=self.kind == "adamw", bias_correction=g.get("bias_correction", True))
        elif self.kind == "sgd":
            mom = float(g.get("momentum", 0.0))
            mt.fused_sgd_(plow, grad, d.master, d.m if mom != 0.0 else None, lr, mom, float(g.get("dampening", 0.0)),
                          wd, bool(g.get("nesterov", False)), step == 1, gscale)
        elif self.kind == "adagrad":
            mt.fused_adagrad_(plow, grad, d.master, d.v, lr, float(g.get("eps", 1e-10)), wd, gscale)
        elif self.kind == "lamb":
            b1, b2 = g.get("betas", (0.9, 0.999))
            mt.lamb_stage1_(grad, d.master, d.m, d.v, d.upd, float(b1), float(b2), float(g.get("eps", 1e-6)), wd,
                            step, gscale, bias_correction=g.get("bias_correction", True))
            # per-parameter trust ratios inside the domain: one chunk table per domain (layout
            # is fixed), two launches for all of its parameters
            table = getattr(d, "_lamb_chunks", None)
            if table is None:
                flat = state.model.flat_groups[d.key]
                pieces = []
                for p in d.params:
                    o = flat.offsets[p]
                    s, e = max(o, d.start), min(o + p.numel(), d.end)
                    if s < e:
                        pieces.append((s - d.start, e - d.start))
                table = d._lamb_chunks = (mt.lamb_chunk_table(pieces, d.master.device), len(pieces))
            mt.lamb_segmented_(plow, d.master, d.upd, table[0], table[1], lr,
                               use_trust=g.get("use_nvlamb", False) or wd != 0.0)

    def _generic_step(self, gscale, lowp):
        for d in self.domains:
            gr = torch.empty_like(d.master)
            mt.cast_copy_(self._grad_range(d), gr, gscale)
            d.vparam.grad = gr
        self.optimizer.step()
        for d in self.domains:
            if d.master.data_ptr() != self._param_range(d).data_ptr():
                mt.cast_copy_(d.master, self._param_range(d))

    def _allgather_shards(self):
        model = state.model
        if state.sdp is not None:
            state.sdp.after_optimizer_step()
        for r in model.reducers.values():
            if r.shard and r.group_size > 1:
                r.allgather_params()

    # ----------------------------------------------------------- state dicts
    _STATE_KEYS = ("master", "m", "v")

    def _param_pieces(self, d):
        """(name, numel, lo, hi, dlo, dhi): elements [lo, hi) of parameter `name` live at
        [dlo, dhi) of domain d (a bucket, or this rank's shard of it)."""
        flat = state.model.flat_groups[d.key]
        out = []
        for p in d.params:
            off, n = flat.offsets[p], p.numel()
            a, b = max(off, d.start), min(off + n, d.end)
            if a < b:
                out.append((flat.name_of[p], n, a - off, b - off, a - d.start, b - d.start))
        return out

    def local_optimizer_state_dict(self):
        """Per-parameter optimizer state (reference format: a torch optimizer state_dict per
        parameter, `optimizers/optimizer.py:150-200`): fp32 master / first / second moments
        keyed by parameter NAME and element range, independent of the flat-buffer layout, so
        a checkpoint loads after a change of bucket cap or parameter-group order.  The
        generic (non-fused) path keeps the inner optimizer's domain-bound state, with the
        layout recorded and verified on load."""
        if self._offload is not None:
            self._offload.wait()  # host copies of the last step are complete
        sd = {
            "format": "smp_amd_per_param_v1",
            "kind": self.kind,
            "step_count": list(self._step_count),
            "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.optimizer.param_groups],
        }
        if self.kind == "generic" or state.sdp is not None:
            # domain-bound: the generic path's inner optimizer state, and sharded data
            # parallelism (whose files are per shard rank and need the same layout anyway)
            sd["domains"] = [
                {k: (getattr(d, k).detach().cpu() if getattr(d, k) is not None else None) for k in self._STATE_KEYS}
                | {"key": d.key, "start": d.start, "end": d.end}
                | ({"names": [(n, lo, hi) for n, _, lo, hi, _, _ in self._param_pieces(d)]} if state.sdp is None else {})
                for d in self.domains
            ]
            sd["inner"] = self.optimizer.state_dict() if self.kind == "generic" else None
            return sd
        params = {}
        for d in self.domains:
            for name, numel, lo, hi, dlo, dhi in self._param_pieces(d):
                e = params.setdefault(name, {"numel": numel, "pieces": []})
                piece = {"lo": lo, "hi": hi}
                for k in self._STATE_KEYS:
                    t = getattr(d, k)
                    if t is not None:
                        piece[k] = t[dlo:dhi].detach().to("cpu", copy=True)
                e["pieces"].append(piece)
        sd["params"] = params
        return sd

    def local_fp16_state_dict(self):
        return {"loss_scaler": self.loss_scaler.state_dict(), "fp16": self.fp16, "bf16": self.bf16}

    def local_state_dict(self):
        d = self.local_optimizer_state_dict()
        d["fp16_state"] = self.local_fp16_state_dict()
        return d

    def state_dict(self):
        return self.local_state_dict()

    def _load_per_param(self, saved):
        """Copy every saved (name, element range) piece into the domains that hold it now."""
        for d in self.domains:
            for name, numel, lo, hi, dlo, dhi in self._param_pieces(d):
                e = saved.get(name)
                if e is None:
                    raise SMPInvalidArgumentError(f"optimizer checkpoint has no state for parameter {name}")
                if e["numel"] != numel:
                    raise SMPInvalidArgumentError(
                        f"optimizer checkpoint: parameter {name} has {e['numel']} elements, the model {numel}")
                covered = 0
                for pc in e["pieces"]:
                    a, b = max(lo, pc["lo"]), min(hi, pc["hi"])
                    if a >= b:
                        continue
                    covered += b - a
                    for k in self._STATE_KEYS:
                        t = getattr(d, k)
                        if t is not None and k in pc:
                            t[dlo + (a - lo):dlo + (b - lo)].copy_(pc[k][a - pc["lo"]:b - pc["lo"]].to(t.device))
                if covered < hi - lo:
                    raise SMPInvalidArgumentError(
                        f"optimizer checkpoint covers {covered} of elements [{lo}, {hi}) of {name} on this rank "
                        "(the optimizer-state sharding layout changed; save and load with the same layout)")

    def _load_domains(self, sd):
        """Generic / legacy domain-bound state: the layout must match exactly."""
        doms = sd["domains"]
        if len(doms) != len(self.domains):
            raise SMPInvalidArgumentError(
                f"optimizer state has {len(doms)} domains, the current layout {len(self.domains)} "
                "(partition / sharding / bucket layout changed)")
        for d, s in zip(self.domains, doms):
            if (s.get("key"), s.get("start"), s.get("end")) != (d.key, d.start, d.end):
                raise SMPInvalidArgumentError(
                    f"optimizer state domain {(s.get('key'), s.get('start'), s.get('end'))} does not match the "
                    f"current layout {(d.key, d.start, d.end)}")
            if "names" in s and state.sdp is None:
                cur = [(n, lo, hi) for n, _, lo, hi, _, _ in self._param_pieces(d)]
                if [tuple(x) for x in s["names"]] != cur:
                    raise SMPInvalidArgumentError(f"optimizer state domain {d.key}[{d.start}:{d.end}] holds "
                                                  "different parameters than the current layout")
            for k in self._STATE_KEYS:
                t = getattr(d, k)
                if t is not None and s.get(k) is not None:
                    t.copy_(s[k].to(t.device))

    def load_local_optimizer_state_dict(self, sd):
        if "params" in sd:
            self._load_per_param(sd["params"])
        else:
            self._load_domains(sd)
        for d in self.domains:
            lowp = self.fp16 or self.bf16
            if lowp:
                src = d.master.to(self._param_range(d).device, non_blocking=False)
                mt.cast_copy_(src, self._param_range(d))
        self._step_count = list(sd.get("step_count", self._step_count))
        for g, saved in zip(self.optimizer.param_groups, sd.get("param_groups", [])):
            for k, v in saved.items():
                g[k] = v
        if self.kind == "generic" and sd.get("inner") is not None:
            self.optimizer.load_state_dict(sd["inner"])
        self._allgather_shards()

    def load_local_fp16_state_dict(self, sd):
        self.loss_scaler.load_state_dict(sd["loss_scaler"])

    # torch optimizer-state keys of the reference's wrapped optimizers -> our domain buffers
    _REF_KEYS = {"m": ("exp_avg", "momentum_buffer"), "v": ("exp_avg_sq", "sum")}

    @staticmethod
    def is_reference_format(sd):
        """A reference `smp` optimizer state: the wrapped torch optimizer's state_dict (partial:
        `_smp_is_partial`, `optimizers/optimizer.py:125-200`), optionally inside the fp16 wrapper
        dict (`optimizer_state_dict` + `fp32_from_fp16`, `backcompat_opt.py:136-154`)."""
        return isinstance(sd, dict) and ("optimizer_state_dict" in sd or ("state" in sd and "param_groups" in sd))

    def _from_reference_format(self, sd):
        """Reference-format state -> this optimizer's per-parameter format.  Parameter indices
        are the positions in the optimizer's parameter groups (reference `param_name_to_index`),
        so the model and the optimizer's groups must be built as in the saving job."""
        masters = sd.get("fp32_from_fp16")
        inner = sd["optimizer_state_dict"] if "optimizer_state_dict" in sd else sd
        i2n = self.param_index_to_name()
        names = {p: n for n, p in state.model.module.named_parameters()}
        master_of = {}
        if masters is not None:
            if len(masters) != len(self._orig_param_groups):
                raise SMPInvalidArgumentError("reference optimizer state: fp32_from_fp16 groups do not match the "
                                              "optimizer's parameter groups")
            for g, ms in zip(self._orig_param_groups, masters):
                # the reference builds fp32_from_fp16 from trainable params only (fp16_optimizer.py:45)
                lowp = [p for p in g["params"] if p.dtype in (torch.float16, torch.bfloat16) and p.requires_grad]
                if len(lowp) != len(ms):
                    raise SMPInvalidArgumentError("reference optimizer state: fp32_from_fp16 does not match the "
                                                  "low-precision parameters of a group")
                for p, m in zip(lowp, ms):
                    master_of[names[p]] = m
        params = {}
        steps = [0] * len(self._orig_param_groups)
        by_name = {n: p for n, p in state.model.module.named_parameters()}
        gidx = self._group_index_of()
        for idx, st in inner.get("state", {}).items():
            name = i2n.get(int(idx))
            if name is None or not st:
                continue  # not a parameter of this optimizer / state kept on another TP rank
            p = by_name[name]
            n = p.numel()
            piece = {"lo": 0, "hi": n}
            for ours, theirs in self._REF_KEYS.items():
                for k in theirs:
                    if isinstance(st.get(k), torch.Tensor):
                        piece[ours] = st[k].detach().reshape(-1).float().cpu()
                        break
            mt_ = master_of.get(name)
            piece["master"] = (mt_ if mt_ is not None else p.detach()).reshape(-1).float().cpu()
            params[name] = {"numel": n, "pieces": [piece]}
            if "step" in st:
                steps[gidx[p]] = max(steps[gidx[p]], int(float(st["step"])))
            elif "m" in piece:  # torch SGD keeps no step: a momentum buffer means >= 1 step taken
                steps[gidx[p]] = max(steps[gidx[p]], 1)
        out = {"format": "smp_amd_per_param_v1", "kind": self.kind, "params": params, "step_count": steps,
               "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in inner.get("param_groups", [])]}
        # the fp16 wrapper's dynamic loss scale (reference `fp16/fp16.py:668-700`: "loss_scaler" with
        # cur_scale / cur_iter / last_overflow_iter): carried over when readable, else it restarts
        ls = sd.get("loss_scaler") if masters is not None else None
        cur = getattr(ls, "cur_scale", None) if ls is not None and not isinstance(ls, dict) else \
            (ls.get("cur_scale") if isinstance(ls, dict) else None)
        if cur is not None:
            out["loss_scale"] = float(cur)
        return out

    def load_state_dict(self, sd):
        if not self._built:
            self._deferred_load = sd
            return
        if self.is_reference_format(sd):
            sd = self._from_reference_format(sd)
        self.load_local_optimizer_state_dict(sd)
        if "fp16_state" in sd:
            self.load_local_fp16_state_dict(sd["fp16_state"])
        elif sd.get("loss_scale") is not None and self.loss_scaler is not None:
            self.loss_scaler.cur_scale = float(sd["loss_scale"])  # a reference fp16 wrapper's scale

    def load_optimizer_checkpoint(self, sd):
        self.load_state_dict(sd)

    def param_name_to_index(self):
        names = {p: n for n, p in state.model.module.named_parameters()}
        out, i = {}, 0
        for g in self._orig_param_groups:
            for p in g["params"]:
                out[names.get(p)] = i
                i += 1
        return out

    def param_index_to_name(self):
        return {v: k for k, v in self.param_name_to_index().items()}

    def add_param_group(self, group):
        raise SMPInvalidArgumentError("add_param_group after wrapping in DistributedOptimizer is not supported")

    def __getstate__(self):
        raise TypeError("DistributedOptimizer is not picklable; use smp.save_checkpoint")
