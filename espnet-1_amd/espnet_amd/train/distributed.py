"""Data parallelism over the parameter arena (replaces DistributedDataParallel as used by
espnet2/train/trainer.py:229-244; one process per GPU, RCCL over xGMI).

* K3: parameters broadcast from rank 0 at construction (one call: the arena is one
  buffer).
* K2: BatchNorm running stats broadcast from rank 0 before each forward
  (broadcast_buffers=True semantics).
* K1: gradients summed with all_reduce on contiguous byte ranges of the grad arena
  ("buckets"), issued back-to-front so the bucket whose gradients are complete first
  goes first; RCCL runs them on its own stream.
* K4-K6: the stats / weight all-reduces of recursive_average (recursive_op.py:8-47) are
  packed into ONE message.
Loss weighting follows trainer.py:604-619: loss_r * w_r / sum(w) on every rank, and the
SUM all-reduce of gradients then equals DDP's mean of (loss_r * w_r / sum(w) * world).
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.distributed as dist


class ArenaDataParallel:
    def __init__(self, model, bucket_mb: float = 64.0, group=None):
        self.model = model
        self.group = group
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        arena = model.arena
        self.arena = arena
        n = arena.numel
        per = max(int(bucket_mb * 1024 * 1024 / 4) // 64 * 64, 64)
        # buckets back-to-front: the tail of the arena (decoder / CTC head, whose grads
        # finish first in backward) is reduced first
        self.buckets: List[slice] = []
        end = n
        while end > 0:
            start = max(0, end - per)
            self.buckets.append(slice(start, end))
            end = start
        self._bufs = [b for _, b in sorted(model.named_buffers()) if b.is_floating_point() or b.dtype == torch.long]
        if self.world_size > 1:
            dist.broadcast(arena.data, 0, group=group)
            arena.refresh_shadow()
            self.broadcast_buffers()

    def broadcast_buffers(self):
        if self.world_size > 1:
            for b in self._bufs:
                dist.broadcast(b, 0, group=self.group)

    def weighted_average(self, loss, stats: Dict[str, torch.Tensor], weight):
        """trainer.py:604-619 + recursive_average (recursive_op.py:30-47), one all-reduce."""
        keys = sorted(stats)
        w = weight.to(torch.float32).view(1)
        pack = torch.cat([w] + [stats[k].detach().float().view(1) * w for k in keys])
        dist.all_reduce(pack, group=self.group)
        wsum = pack[0:1]
        new_stats = {k: pack[i + 1:i + 2] / wsum for i, k in enumerate(keys)}
        loss = (loss * w).sum() / wsum
        return loss, new_stats, wsum.to(torch.long)

    def allreduce_grads(self):
        g = self.arena.grad
        works = [dist.all_reduce(g[s], async_op=True, group=self.group) for s in self.buckets]
        for w in works:
            w.wait()
