"""Trainer step — the semantics of espnet2/train/trainer.py:train_one_epoch (:472-731) for
one minibatch, on the HIP path:

  model(**batch) -> (loss, stats, weight)                               (:567)
  DP weighting: loss*weight / sum_ranks(weight); stats weighted-averaged (:604-619)
  backward -> gradient all-reduce over RCCL (SUM; the ÷world of DDP is folded into the
  loss weight)                                                           (:632, K1)
  every accum_grad: clip_grad_norm_(grad_clip) + skip if non-finite + Adam + WarmupLR +
  zero_grad                                                              (:653-701)

The clip coefficient and the finite check live on the device (ArenaAdam), so a step
issues no host synchronisation; the grad norm is returned as a device tensor.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import torch

from ..optim.adam import ArenaAdam


class Trainer:
    @staticmethod
    def train_one_step(model, batch: Dict[str, torch.Tensor], optimizer: ArenaAdam, scheduler=None, *,
                       grad_clip: float = 5.0, accum_grad: int = 1, iiter: int = 1, dp=None, maxlens=None):
        if dp is not None and dp.world_size > 1:
            dp.broadcast_buffers()
        if maxlens is not None:
            loss, stats, weight = model(**batch, _maxlens=maxlens)
        else:
            loss, stats, weight = model(**batch)
        stats = {k: v for k, v in stats.items() if v is not None}
        if dp is not None and dp.world_size > 1:
            loss, stats, weight = dp.weighted_average(loss, stats, weight)
        loss = loss / accum_grad if accum_grad > 1 else loss
        if dp is not None and dp.world_size > 1:
            dp.begin_backward()
        loss.backward()
        if dp is not None and dp.world_size > 1:
            dp.allreduce_grads()
        grad_norm = None
        if iiter % accum_grad == 0:
            grad_norm = optimizer.compute_grad_norm()
            optimizer.step(grad_norm=grad_norm, max_norm=grad_clip)
            if scheduler is not None:
                scheduler.step()
            optimizer.zero_grad()
        return loss.detach(), stats, weight, grad_norm
