"""torch.optim.Adam over the flat parameter arena (espnet2/tasks/abs_task.py:79-90 'adam').

One kernel updates all parameters (plus the bf16 weight shadow) and folds in
clip_grad_norm_ and the skip-on-non-finite rule of trainer.py:653-678, reading the grad
norm from device memory — the step never synchronises with the host.
The step count, the learning rate of the attached batch-step schedule (WarmupLR) and the
bias corrections are device state too (ea_adam_step_dev), so a whole training step can be
captured once as a hipGraph and replayed (espnet_amd/train/graph.py).
state_dict() exposes the per-parameter torch.optim.Adam layout (exp_avg / exp_avg_sq
views, step) so checkpoints interoperate with the reference's.
"""
from __future__ import annotations

import ctypes

import torch

from .. import hip_ops as ops
from .._lib import OPT_STATE_BYTES, SCHED_CONSTANT, LrSchedule, lib


class ArenaAdam(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad")
        arena = model.arena
        if arena is None:
            raise RuntimeError("call model.prepare(device) before building the optimizer")
        super().__init__(list(model.parameters()),
                         dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self.arena = arena
        # torch.optim.Adam numbers its per-parameter state by position in the param group,
        # i.e. model.parameters() order (not the arena layout order)
        self.param_names = [n for n, _ in model.named_parameters()]
        self.exp_avg = torch.zeros_like(arena.data)
        self.exp_avg_sq = torch.zeros_like(arena.data)
        # ea_opt_state: applied-update count, lr/bias corrections/clip coef of the last step
        self.state_dev = torch.zeros(OPT_STATE_BYTES // 8, dtype=torch.int64, device=arena.device)
        self.schedule = LrSchedule(SCHED_CONSTANT, 0.0, float(lr))
        self.grad_norm = torch.zeros(1, device=arena.device)
        self._ws = torch.empty(4096, dtype=torch.float64, device=arena.device)

    def attach_schedule(self, kind, warmup_steps, base_lr):
        """Batch-step LR schedule evaluated on device from the applied-update count."""
        self.schedule = LrSchedule(int(kind), float(warmup_steps), float(base_lr))

    @property
    def step_count(self) -> int:
        """Applied updates (torch Adam state['step']); reads device memory (syncs)."""
        return int(self.state_dev[0].item())

    @step_count.setter
    def step_count(self, v: int):
        self.state_dev[0] = int(v)

    def last_lr(self) -> float:
        return float(self.state_dev[1:2].view(torch.float32)[0].item())

    @torch.no_grad()
    def compute_grad_norm(self):
        """||all grads||_2 on device (clip_grad_norm_ norm_type=2)."""
        a = self.arena
        lib.ea_sqnorm(a.numel, a.grad.data_ptr(), self._ws.data_ptr(), self.grad_norm.data_ptr(), ops.stream())
        return self.grad_norm

    @torch.no_grad()
    def step(self, closure=None, grad_norm=None, max_norm=0.0):
        """Adam step; with grad_norm (device tensor) the clip coefficient
        min(1, max_norm/(norm+1e-6)) is applied and a non-finite norm skips the update
        (and does not advance the step count / schedule)."""
        g = self.param_groups[0]
        a = self.arena
        b1, b2 = g["betas"]
        if self.schedule.kind == SCHED_CONSTANT:
            self.schedule.base_lr = float(g["lr"])
        lib.ea_adam_step_dev(a.numel, a.data.data_ptr(), a.grad.data_ptr(), self.exp_avg.data_ptr(),
                             self.exp_avg_sq.data_ptr(), ops.ptr(a.shadow), ctypes.byref(self.schedule),
                             b1, b2, float(g["eps"]), float(g["weight_decay"]), self.state_dev.data_ptr(),
                             ops.ptr(grad_norm), float(max_norm), ops.stream())
        if getattr(a, "tshadow", None) is not None:  # W^T copies follow the new bf16 shadow
            a.tshadow.refresh()

    def zero_grad(self, set_to_none: bool = False):
        self.arena.grad.zero_()

    def state_dict(self):
        sd = super().state_dict()
        st = {}
        step = float(self.step_count)
        for i, n in enumerate(self.param_names):
            st[i] = dict(step=torch.tensor(step),
                         exp_avg=self.arena_view(self.exp_avg, n).clone(),
                         exp_avg_sq=self.arena_view(self.exp_avg_sq, n).clone())
        sd["state"] = st
        return sd

    def arena_view(self, buf, name):
        o = self.arena.offsets[name]
        p = self.arena._params[name]
        return buf[o:o + p.numel()].view(p.shape)

    def load_state_dict(self, state_dict):
        st = state_dict["state"]
        for i, n in enumerate(self.param_names):
            if i in st:
                self.arena_view(self.exp_avg, n).copy_(st[i]["exp_avg"])
                self.arena_view(self.exp_avg_sq, n).copy_(st[i]["exp_avg_sq"])
                self.step_count = int(st[i]["step"])
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            for k in ("lr", "betas", "eps", "weight_decay"):
                if k in sg:
                    g[k] = sg[k]
