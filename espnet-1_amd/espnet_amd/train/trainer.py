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
import math
from typing import Dict, Iterable, Optional

import torch
import torch.distributed as dist

from .. import hip_ops as ops
from ..optim.adam import ArenaAdam


class Trainer:
    @staticmethod
    def train_one_step(model, batch: Dict[str, torch.Tensor], optimizer: ArenaAdam, scheduler=None, *,
                       grad_clip: float = 5.0, accum_grad: int = 1, iiter: int = 1, dp=None, maxlens=None):
        if dp is not None and dp.active:
            dp.broadcast_buffers()
        if maxlens is not None:
            loss, stats, weight = model(**batch, _maxlens=maxlens)
        else:
            loss, stats, weight = model(**batch)
        if dp is not None and dp.active:
            # every rank packs the model's full (fixed) key set, None entries flagged, so
            # the one stats all-reduce has the same size on every rank
            present = {k for k, v in stats.items() if v is not None}
            loss, stats, weight = dp.weighted_average(loss, stats, weight)
            stats = {k: v for k, v in stats.items() if k in present}
        else:
            stats = {k: v for k, v in stats.items() if v is not None}  # trainer.py:604
        loss = loss / accum_grad if accum_grad > 1 else loss
        if dp is not None and dp.active:
            dp.begin_backward()
        # the Linear weight gradients of the pass are queued and run as grouped GEMMs (at the
        # end of the pass, or per bucket from the DP hooks)
        with ops.deferred_wgrad():
            loss.backward()
        if dp is not None and dp.active:
            dp.allreduce_grads()
        grad_norm = None
        if iiter % accum_grad == 0:
            grad_norm = optimizer.compute_grad_norm()
            optimizer.step(grad_norm=grad_norm, max_norm=grad_clip)
            if scheduler is not None:
                scheduler.step()
            optimizer.zero_grad()
        return loss.detach(), stats, weight, grad_norm

    @staticmethod
    @torch.no_grad()
    def validate_one_epoch(model, iterator: Iterable, dp=None, device="cuda") -> Dict[str, float]:
        """trainer.py:735-783 plus the epoch summary of SubReporter (reporter.py aggregate,
        WeightedAverage): eval mode, one forward per minibatch (CER/WER come from the model's
        ErrorCalculator), stats weighted-averaged across ranks per batch and then across
        batches by batch weight, skipping None and non-finite values. Ranks whose iterators
        run out first stop everyone through the reference's iterator_stop all-reduce.
        `device` holds the stop flag: "cuda" for RCCL, "cpu" for gloo."""
        was_training = model.training
        model.eval()
        distributed = dp is not None and dp.active
        group = dp.group if distributed else None
        stop = torch.zeros((), dtype=torch.long, device=device)
        sums: Dict[str, float] = {}
        wsums: Dict[str, float] = {}
        exhausted = True
        for batch in iterator:
            if isinstance(batch, tuple):  # (utt_id, batch) as the reference's iterators yield
                batch = batch[1]
            if distributed:
                dist.all_reduce(stop, group=group)
                if stop.item() > 0:
                    exhausted = False
                    break
            if distributed:
                # DDP(broadcast_buffers=True) syncs the BatchNorm running stats from rank 0
                # before every forward, eval forwards included (DDP._pre_forward)
                dp.broadcast_buffers()
            loss, stats, weight = model(**batch)
            if distributed:  # full key set, None flagged: same message size on every rank
                _, stats, weight = dp.weighted_average(loss, stats, weight)
            stats = {k: v for k, v in stats.items() if v is not None}
            w = float(weight.sum())
            for k, v in stats.items():
                v = float(v.sum())
                if math.isfinite(v) and math.isfinite(w):
                    sums[k] = sums.get(k, 0.0) + v * w
                    wsums[k] = wsums.get(k, 0.0) + w
        if distributed and exhausted:
            stop.fill_(1)
            dist.all_reduce(stop, group=group)
        if was_training:
            model.train()
        return {k: (sums[k] / wsums[k] if wsums[k] else float("nan")) for k in sums}
