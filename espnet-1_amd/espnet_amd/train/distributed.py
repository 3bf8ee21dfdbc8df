"""Data parallelism over the parameter arena — replaces DistributedDataParallel as used by
espnet2/train/trainer.py:229-244 (one process per GPU, RCCL over xGMI; gloo on CPU).

* K3: parameters broadcast from rank 0 at construction (ONE call: the arena is one buffer).
* K2: BatchNorm running stats broadcast from rank 0 before each forward
  (broadcast_buffers=True semantics) — two calls (flat f32 + int64 buffer arenas).
* K1: gradients summed with all_reduce over contiguous ranges of the grad arena
  ("buckets", default 64 MiB — fewer, larger messages suit xGMI's point-to-point links).
  Each block-level backward reports its module prefix when its gradients are final
  (`grad_ready`); a bucket whose modules are all final is all-reduced immediately
  (async), so RCCL's stream overlaps the rest of the backward pass.
* K4-K6: the stats / weight all-reduces of recursive_average (recursive_op.py:8-47) are
  packed into ONE message.
Loss weighting follows trainer.py:604-619: loss_r * w_r / sum(w); with the SUM all-reduce
of gradients this equals DDP's mean of (loss_r * w_r / sum(w) * world).
"""
from __future__ import annotations

import os
from typing import Dict, List

import torch
import torch.distributed as dist

from .. import hip_ops

class ArenaDataParallel:
    def __init__(self, model, bucket_mb: float = None, group=None, overlap: bool = True,
                 force_collectives: bool = False, check_issue: bool = None):
        # bucket size (DDP's bucket_cap_mb): EA_DP_BUCKET_MB, else 64 MiB
        if bucket_mb is None:
            bucket_mb = float(os.environ.get("EA_DP_BUCKET_MB", "64"))
        self.model = model
        self.group = group
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # `active`: the step issues its collectives.  Always for world_size > 1; with
        # force_collectives also at world_size 1 (a world-1 RCCL group exercises the same
        # code path on a one-GPU box: capture of the all-reduces, bucket hooks, packing)
        self.active = self.world_size > 1 or (force_collectives and dist.is_initialized())
        # Every backend issues the bucket all-reduces the same way (from the weight-gradient
        # side stream, overlapped with the rest of the backward): the gloo tests run the
        # ordering RCCL runs in production.  (Round 5's intermittent two-process drift, which
        # once moved gloo's all-reduces to the main stream, was a kernel's, not the ordering's:
        # the conv1 forward sometimes computed a few wrong outputs under packed-FP32 code,
        # DESIGN.md §5 round 6, tests/test_dp_ragged_gpu.py.)
        arena = model.arena
        self.arena = arena
        n = arena.numel
        per = max(int(bucket_mb * 1024 * 1024 / 4) // 64 * 64, 64)
        # module prefix -> arena span (prefixes = the block-level autograd nodes)
        self.prefixes = sorted({getattr(m, "_b").prefix for m in model.modules()
                                if getattr(m, "_b", None) is not None}, key=len, reverse=True)
        span = {}
        for name in arena.names:
            pre = next((p for p in self.prefixes if name.startswith(p)), None)
            if pre is None:
                raise RuntimeError(f"parameter {name} is not owned by a block-level node")
            o = arena.offsets[name]
            lo, hi = span.get(pre, (o, o))
            span[pre] = (min(lo, o), max(hi, o + arena._params[name].numel()))
        # buckets back-to-front: the tail of the arena (decoder / CTC head, whose grads
        # are final first in backward) is reduced first.  The front module (the subsampling
        # front end: its backward is the last of the step) gets a bucket of its own, so the
        # blocks above it are reduced while its backward runs and only its own bytes are
        # exposed after the backward ends.
        front_end = 0
        if span:
            front = min(span, key=lambda p: span[p][0])
            front_end = min(n, (span[front][1] + 63) // 64 * 64)
            if front_end >= n:
                front_end = 0
        self.buckets: List[slice] = []
        end = n
        while end > 0:
            start = max(0, end - per)
            if start < front_end < end:
                start = front_end
            self.buckets.append(slice(start, end))
            end = start
        self._bucket_mods = []
        for b in self.buckets:
            self._bucket_mods.append({p for p, (lo, hi) in span.items() if lo < b.stop and hi > b.start})
        self.overlap = overlap
        self._pending = None
        self._works = []
        # check_issue (EA_DP_CHECK_ISSUE=1; diagnostic, eager steps only): a bucket's all-reduce
        # is not started at its issue point; a copy of the bucket is taken there (on the issuing
        # stream, where the collective would read it) and allreduce_grads compares it with the
        # bucket once the backward has ended, before reducing the buckets in issue order.  A
        # gradient written into a bucket after its all-reduce was issued raises, naming the
        # parameters.
        self.check_issue = (os.environ.get("EA_DP_CHECK_ISSUE", "0") != "0") if check_issue is None else check_issue
        self._held = []
        if self.active:
            dist.broadcast(arena.data, 0, group=group)
            arena.refresh_shadow()
            self.broadcast_buffers()

    # ------------------------------------------------------------------ per step
    def broadcast_buffers(self):
        if self.active:
            for b in (self.arena.buf_f32, self.arena.buf_i64):
                if b.numel():
                    dist.broadcast(b, 0, group=self.group)

    def weighted_average(self, loss, stats: Dict[str, torch.Tensor], weight):
        """trainer.py:604-619 + recursive_average (recursive_op.py:30-47), one all-reduce.

        Every rank packs the SAME message: each key of `stats` (the model emits a fixed key
        set; None entries included) contributes (value * w, w) or (0, 0) when the value is
        None on this rank.  A key reduces to sum(v*w) / sum(w) over the ranks that had a
        value — the reference's result whenever every rank has one — and to NaN when no
        rank had one.  (The reference all-reduces per key and skips None keys, so a key that
        is None on some ranks only would mismatch its collectives.)"""
        keys = sorted(stats)
        w = weight.to(torch.float32).view(1)
        zero = torch.zeros(1, dtype=torch.float32, device=w.device)
        parts = [w]
        for k in keys:
            v = stats[k]
            parts += [zero, zero] if v is None else [v.detach().float().view(1) * w, w]
        pack = torch.cat(parts)
        dist.all_reduce(pack, group=self.group)
        wsum = pack[0:1]
        # no host read here (the step stays sync-free and capturable): a key no rank had
        # comes back NaN, which the epoch averages skip like the reference reporter skips
        # None / non-finite values
        vals = pack[1:].view(-1, 2)
        new_stats = {}
        for i, k in enumerate(keys):
            vw, ww = vals[i, 0:1], vals[i, 1:2]
            new_stats[k] = torch.where(ww > 0, vw / ww.clamp_min(1e-30), torch.full_like(vw, float("nan")))
        loss = (loss * w).sum() / wsum
        return loss, new_stats, wsum.to(torch.long)

    def begin_backward(self):
        """Arm the grad-ready hooks for one backward pass."""
        self._pending = [set(m) for m in self._bucket_mods]
        self._works = []
        if self.overlap and self.active:
            hip_ops.GRAD_READY = self.grad_ready

    def grad_ready(self, prefix: str):
        """A block's backward is done (hip_ops.grad_ready).  Its deferred weight-gradient
        GEMMs are launched on the weight-gradient side stream, and every bucket this block
        completes is all-reduced from that stream: RCCL waits for the side stream (which
        already waited for the main stream's part of the block), and the main stream goes on
        with the backward of the blocks below."""
        if self._pending is None:
            hip_ops.join_wgrad()
            return
        done = []
        for i, mods in enumerate(self._pending):
            if prefix in mods:
                mods.discard(prefix)
                if not mods:
                    done.append(i)
        if not done:
            return  # the deferred GEMMs keep accumulating until a bucket needs them
        with hip_ops.wgrad(*hip_ops.deferred_tensors(), launches=True):
            hip_ops.flush_deferred()
            for i in done:
                self._issue(i)

    def _issue(self, i):
        """Start bucket i's SUM all-reduce from the current stream (async)."""
        g = self.arena.grad[self.buckets[i]]
        if self.check_issue:
            self._held.append((i, g.clone()))
            return
        self._works.append(dist.all_reduce(g, async_op=True, group=self.group))

    def _check_held(self):
        hip_ops.join_aux()
        held, self._held = self._held, []
        bad = []
        for i, snap in held:
            b = self.buckets[i]
            g = self.arena.grad[b]
            if not torch.equal(g, snap):
                for name in self.arena.names:
                    o = self.arena.offsets[name]
                    lo, hi = max(o, b.start), min(o + self.arena._params[name].numel(), b.stop)
                    if lo < hi and not torch.equal(self.arena.grad[lo:hi], snap[lo - b.start:hi - b.start]):
                        bad.append(f"bucket {i}: {name}")
            self._works.append(dist.all_reduce(g, async_op=True, group=self.group))
        if bad:
            for w in self._works:
                w.wait()
            self._works = []
            self._pending = None
            raise RuntimeError("gradients written after their bucket's all-reduce was issued: " + "; ".join(bad))

    def allreduce_grads(self):
        """Finish the step's gradient reduction (launch what the hooks did not, wait all)."""
        hip_ops.GRAD_READY = None
        hip_ops.flush_deferred()
        hip_ops.join_wgrad()
        if self._pending is None:
            self._pending = [set(m) for m in self._bucket_mods]
        for i, mods in enumerate(self._pending):
            if mods:
                mods.clear()
                self._issue(i)
        if self._held:
            self._check_held()
        for w in self._works:
            w.wait()
        self._works = []
        self._pending = None
