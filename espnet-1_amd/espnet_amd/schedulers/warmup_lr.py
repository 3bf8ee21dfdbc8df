"""WarmupLR — espnet2/schedulers/warmup_lr.py:11-50:
lr = base_lr * warmup^0.5 * min(step^-0.5, step * warmup^-1.5), step = last_epoch + 1.

On an arena optimizer (ArenaAdam) the schedule is evaluated on the device from the
optimizer's applied-update count (ea_adam_step_dev), which keeps a captured training step
replayable and advances exactly when the reference calls scheduler.step() — only after an
applied update (trainer.py:682-697).  The host fields mirror it for logging/state_dict."""
from __future__ import annotations

from .._lib import SCHED_WARMUP


class WarmupLR:
    def __init__(self, optimizer, warmup_steps=25000, last_epoch: int = -1):
        self.optimizer = optimizer
        self.warmup_steps = warmup_steps
        self.base_lrs = [g.get("initial_lr", g["lr"]) for g in optimizer.param_groups]
        for g, lr in zip(optimizer.param_groups, self.base_lrs):
            g["initial_lr"] = lr
        self._device = hasattr(optimizer, "attach_schedule")
        if self._device:
            optimizer.attach_schedule(SCHED_WARMUP, warmup_steps, self.base_lrs[0])
        self.last_epoch = last_epoch
        self.step()

    def get_lr(self):
        s = self.last_epoch + 1
        return [lr * self.warmup_steps ** 0.5 * min(s ** -0.5, s * self.warmup_steps ** -1.5)
                for lr in self.base_lrs]

    def step(self, epoch=None):
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        for g, lr in zip(self.optimizer.param_groups, self.get_lr()):
            g["lr"] = lr

    def state_dict(self):
        last = self.optimizer.step_count if self._device else self.last_epoch
        return dict(warmup_steps=self.warmup_steps, base_lrs=self.base_lrs, last_epoch=last)

    def load_state_dict(self, sd):
        self.__dict__.update(sd)
        if self._device:
            self.optimizer.attach_schedule(SCHED_WARMUP, self.warmup_steps, self.base_lrs[0])
            self.optimizer.step_count = int(self.last_epoch)

    def __repr__(self):
        return f"{self.__class__.__name__}(warmup_steps={self.warmup_steps})"
