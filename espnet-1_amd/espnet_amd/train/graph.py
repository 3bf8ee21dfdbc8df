"""A whole training step captured as one hipGraph and replayed.

The eager step (trainer.py's Trainer.train_one_step: forward, backward, RCCL gradient
all-reduce, clip_grad_norm_, Adam, WarmupLR, zero_grad — espnet2/train/trainer.py:567-701)
issues ~1,400 kernel launches through Python; on MI355X the host then needs longer to
issue a C3 step than the GPU needs to run it.  Every launch of the step takes its
per-step values from device memory (dropout salt: ea_rng_advance; step count, lr, bias
corrections, clip coefficient and skip flag: ea_adam_step_dev; lengths: device tensors),
so the launch sequence is identical from step to step and can be captured once per input
shape and replayed with a single host call.

Semantics per call are exactly one training step on the given batch:
  * the first `warmup` calls for a new shape run eagerly (on a side stream, as graph
    capture requires: lazy allocations, scratch buffers and the RCCL communicator are
    created there);
  * the next call captures the step (capture executes nothing) and replays it once;
  * later calls copy the batch into the graph's static input buffers and replay.
Shapes (B, T_max, F, L_max) key the graphs; lengths below the maxima vary freely since the
kernels read them from device memory.  The step's host RNG draws (SpecAug's warp and mask
parameters, MultiSequential's layer-drop uniforms) are made before each call in the
reference's order; SpecAug's land in a static device buffer the captured kernel reads, so
SpecAug (C5) steps are captured too.  Outputs (loss, stats, weight, grad_norm) are views
of graph memory, overwritten by the next replay of the same graph.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..layers import common
from ..layers.common import multisequential_draw as layerdrop_draw
from .trainer import Trainer


def _backend(group) -> str:
    import torch.distributed as dist
    try:
        return str(dist.get_backend(group))
    except (RuntimeError, ValueError):
        return ""


class _Captured:
    __slots__ = ("graph", "inputs", "outputs", "maxlens")


class CapturedTrainStep:
    def __init__(self, model, optimizer, scheduler=None, *, grad_clip: float = 5.0, dp=None,
                 warmup: int = 2, enabled: bool = True, control_group=None):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.grad_clip = grad_clip
        self.dp = dp
        self.warmup = max(1, int(warmup))
        self.enabled = enabled
        self.graphs: Dict[tuple, _Captured] = {}
        self._seen: Dict[tuple, int] = {}
        self._pool = None
        self._side = None
        self.control_group = control_group  # gloo group for the capture decision (optional)
        if dp is not None and dp.active and _backend(dp.group) == "gloo":
            self.enabled = False  # gloo collectives (host copies) cannot be captured
        # "graph" once steps replay, "eager" once capture was given up (on any rank); None
        # while the warm-up steps run
        self.mode = None if self.enabled else "eager"

    # ------------------------------------------------------------------ helpers
    def _eager(self, batch, maxlens):
        return Trainer.train_one_step(self.model, batch, self.optimizer, self.scheduler,
                                      grad_clip=self.grad_clip, dp=self.dp, maxlens=maxlens)

    def _device_batch(self, batch, maxlens):
        dev = self.model._device
        sl, tl = maxlens
        return dict(speech=batch["speech"][:, :sl].to(dev, non_blocking=True).contiguous(),
                    speech_lengths=batch["speech_lengths"].to(dev, non_blocking=True),
                    text=batch["text"][:, :tl].to(dev, non_blocking=True).contiguous(),
                    text_lengths=batch["text_lengths"].to(dev, non_blocking=True))

    @staticmethod
    def _maxlens(batch):
        return int(batch["speech_lengths"].max()), int(batch["text_lengths"].max())

    # ------------------------------------------------------------------ host draws
    def _host_draws(self, batch, maxlens, lens_host):
        """The step's host RNG draws, in the reference's order, made before the step runs
        (a replay executes no Python): SpecAug's warp / mask parameters into its static
        device buffer (SpecAug.predraw), then MultiSequential's layer-drop uniforms of the
        encoder and decoder (repeat.py:27).  The forward then skips its own draws."""
        m = self.model
        if not m.training:
            return
        if m.specaug is not None:
            B, _, F = batch["speech"].shape
            T = maxlens[0]
            if lens_host is None:
                sl = batch["speech_lengths"]
                lens_host = [int(v) for v in sl.tolist()]  # a device read if the lengths live there
            if m.frontend is not None:  # sample counts -> feature frames
                T = int(m.frontend.stft.frames_lens(T))
                F = m.frontend.output_size()
                lens_host = [int(m.frontend.stft.frames_lens(int(v))) for v in lens_host]
            m.specaug.predraw(B, T, F, lens_host, m._device)
        layerdrop_draw(len(m.encoder.encoders))
        if m.decoder is not None:
            layerdrop_draw(len(m.decoder.decoders))

    # ------------------------------------------------------------------ step
    def __call__(self, batch: Dict[str, torch.Tensor], maxlens: Optional[tuple] = None, lens_host=None):
        """One training step on `batch`; returns (loss, stats, weight, grad_norm).
        `lens_host`: the speech lengths as host ints when the batch's live on the device
        (SpecAug's per-utterance warp draws need them)."""
        if maxlens is None:
            maxlens = self._maxlens(batch)
        if not self.enabled:
            return self._eager(batch, maxlens)
        B, _, F = batch["speech"].shape
        key = (B, maxlens[0], F, maxlens[1])
        self._host_draws(batch, maxlens, lens_host)
        common.SKIP_LAYERDROP_DRAWS = True
        try:
            cap = self.graphs.get(key)
            if cap is not None:
                for k, v in cap.inputs.items():
                    v.copy_(batch[k][:, :v.shape[1]] if v.dim() > 1 else batch[k], non_blocking=True)
                cap.graph.replay()
                return cap.outputs
            n = self._seen.get(key, 0)
            self._seen[key] = n + 1
            dbatch = self._device_batch(batch, maxlens)
            if n < self.warmup:
                if self._side is None:
                    self._side = torch.cuda.Stream(device=self.model._device)
                main = torch.cuda.current_stream()
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    out = self._eager(dbatch, maxlens)
                main.wait_stream(self._side)
                return out
            err = None
            try:
                cap = self._capture(key, dbatch, maxlens)
            except RuntimeError as e:
                cap, err = None, e
                self._reset_after_failed_capture()
            # the decision is collective: every rank replays its graph or every rank runs
            # eager steps (a graph replay beside an eager step would issue the same
            # collectives, but at a different pace, and the bench would time a mixed mode)
            if self._agree(cap is not None):
                self.graphs[key] = cap
                self.mode = "graph"
                cap.graph.replay()  # capture executes nothing: run this batch's step now
                return cap.outputs
            # a stack that cannot capture this step (e.g. a collective library without graph
            # support on some node) on this rank or another: warn once and run every step
            # eagerly.  Capture executes nothing, so the step is simply run now.
            import warnings
            why = f"failed here ({err})" if err is not None else "failed on another rank"
            warnings.warn(f"hipGraph capture of the training step {why}; running eager steps")
            torch.cuda.synchronize()
            self.enabled = False
            self.mode = "eager"
            self.graphs.clear()
            return self._eager(dbatch, maxlens)
        finally:
            common.SKIP_LAYERDROP_DRAWS = False

    def _reset_after_failed_capture(self):
        """A capture that raised mid-step leaves per-pass host state behind (the deferred
        queues are dropped by their context; the DP grad-ready hook and bucket bookkeeping
        are not): clear it so the eager step starts clean."""
        from .. import hip_ops
        hip_ops.GRAD_READY = None
        if self.dp is not None:
            self.dp._pending = None
            self.dp._works = []

    def _agree(self, ok: bool) -> bool:
        """True when the capture succeeded on every rank: one MIN-style all-reduce of a failure
        count over the control group (gloo, host memory) when there is one, else over the
        data-parallel group.  Without an active DP group this rank decides alone."""
        dp = self.dp
        if dp is None or not dp.active:
            return ok
        import torch.distributed as dist
        group = self.control_group
        dev = "cpu" if group is not None else self.model._device
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, group=group if group is not None else dp.group)
        return int(flag.item()) == 0

    def _capture(self, key, dbatch, maxlens):
        cap = _Captured()
        cap.inputs = dbatch  # static input buffers (own storage)
        cap.maxlens = maxlens
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            # the warm-up steps' collectives are complete now, but the process-group watchdog
            # only retires them at its next poll (~100 ms); a poll during the capture queries an
            # event last recorded on the now-capturing RCCL stream, which HIP refuses, and the
            # watchdog aborts the process — let it retire them first
            import time
            time.sleep(0.5)
        # thread-local capture mode: other threads' HIP calls during the capture (RCCL's
        # process-group watchdog polls its events) must not invalidate it or fail themselves
        with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
            out = self._eager(cap.inputs, maxlens)
        if self._pool is None:
            self._pool = g.pool()
        cap.graph = g
        cap.outputs = out
        return cap
