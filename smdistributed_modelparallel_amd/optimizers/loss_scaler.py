"""Loss scaling for fp16 training.

Reference behaviour: `smp/torch/fp16/loss_scaler.py` -- static scale, or a dynamic scale
that halves on overflow (skipping the step) and doubles after ``scale_window`` clean
steps, with ``min_scale`` / ``delayed_shift`` hysteresis; the overflow decision is
all-reduced (MAX) over the model-parallel group so every stage skips together.

MI355X change: the overflow check is ONE fused device reduction over each flat gradient
buffer plus ONE all-reduce (the reference synchronises the host once per parameter,
K20 in SURVEY §2.6).
"""
import torch
import torch.distributed as dist


class LossScaler:
    def __init__(self, scale=1.0):
        self.cur_scale = float(scale)
        self.dynamic = False

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_loss(self, loss):
        return loss * self.cur_scale if self.cur_scale != 1.0 else loss

    def update_scale(self, overflow):
        pass

    def state_dict(self):
        return {"cur_scale": self.cur_scale, "dynamic": self.dynamic}

    def load_state_dict(self, sd):
        self.cur_scale = sd["cur_scale"]


class DynamicLossScaler(LossScaler):
    def __init__(self, init_scale=2.0 ** 32, scale_factor=2.0, scale_window=1000, min_scale=1.0,
                 delayed_shift=1, consecutive_hysteresis=False):
        super().__init__(init_scale)
        self.dynamic = True
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis
        self.cur_iter = 0
        self.last_overflow_iter = -1

    def update_scale(self, overflow):
        if overflow:
            if self.delayed_shift == 1 or self.cur_hysteresis == 1:
                self.cur_scale = max(self.cur_scale / self.scale_factor, self.min_scale)
            else:
                self.cur_hysteresis -= 1
            self.last_overflow_iter = self.cur_iter
        else:
            if self.consecutive_hysteresis:
                self.cur_hysteresis = self.delayed_shift
            if (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                if not self.consecutive_hysteresis:
                    self.cur_hysteresis = self.delayed_shift
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1

    def state_dict(self):
        d = super().state_dict()
        d.update(cur_iter=self.cur_iter, last_overflow_iter=self.last_overflow_iter,
                 cur_hysteresis=self.cur_hysteresis)
        return d

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        self.cur_iter = sd.get("cur_iter", 0)
        self.last_overflow_iter = sd.get("last_overflow_iter", -1)
        self.cur_hysteresis = sd.get("cur_hysteresis", self.delayed_shift)


def any_overflow(flat_grads, group=None):
    """One device reduction per buffer + one MAX all-reduce; a single host sync."""
    from ..ops import multi_tensor

    flag = None
    for g in flat_grads:
        f = multi_tensor.nonfinite_flag(g)
        flag = f if flag is None else torch.maximum(flag, f)
    collective = group is not None and dist.is_initialized() and dist.get_world_size(group) > 1
    if flag is None:
        if not collective:
            return False
        # a rank without gradients still takes part in the group's decision
        from ..torch.state_mod import state

        flag = torch.zeros(1, dtype=torch.float32, device=state.device)
    if collective:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return bool(flag.item() > 0)
