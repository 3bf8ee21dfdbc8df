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


def prepare_nccl_env():
    """Call before creating an RCCL process group that will carry captured collectives.
    ProcessGroupNCCL recycles HIP events between work objects by default; fresh events keep
    every captured collective's event distinct from the eager warm-up work the watchdog
    tracked (read at process-group construction, so set here, not at package import)."""
    import os
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def _retire_pending_works(group):
    """Block until the process-group watchdog has retired every eager collective of `group`.

    The warm-up steps' collectives are complete once the device is synchronised, but the
    watchdog only drops their work objects at its next poll; a poll during the capture would
    query an event last recorded on the now-capturing RCCL stream, which HIP refuses, and the
    watchdog aborts the process.  ProcessGroupNCCL::waitForPendingWorks waits for exactly that
    retirement (no timing assumption).  gloo groups carry no device events."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    if _backend(pg) != "nccl":
        return
    pg._wait_for_pending_works()


class _Captured:
    __slots__ = ("graph", "inputs", "outputs", "maxlens", "update")


class _PseudoGraph:
    """Test double of a captured graph (CapturedTrainStep(pseudo_capture=True)): 'capture'
    executes nothing and every replay runs the eager step on the static inputs, so the capture
    bookkeeping (per-rank shape keys, warm-up counts, failure handling) runs over collectives
    a hipGraph cannot hold (gloo ranks sharing one GPU)."""

    def __init__(self, runner, cap):
        self.runner, self.cap = runner, cap

    def replay(self):
        self.cap.outputs = self.runner._eager(self.cap.inputs, self.cap.maxlens, self.cap.update)


class CapturedTrainStep:
    """Captures per input shape and replays; see the module docstring.

    Multi-rank jobs: every rank decides ALONE when it captures.  Ranks hold differently
    padded shards (the reference pads each rank's batch[rank::world] to its own maxima,
    abs_task.py:1566-1575), so their shape keys — and the steps at which they capture —
    differ.  A capture executes no collective, and a replay issues the same collectives in
    the same order as an eager step on the same communicator, so a rank replaying beside a
    rank that warms up or captures pairs its collectives correctly.  Nothing here issues a
    collective of its own.  A failed capture makes this rank run eager steps at once and sets
    `failed`; `capture_failed_flag()` is packed into the training loop's per-step control
    all-reduce (trainer.py's iterator_stop message), and `force_eager()` then turns every rank
    eager at the same step."""

    def __init__(self, model, optimizer, scheduler=None, *, grad_clip: float = 5.0, dp=None,
                 warmup: int = 2, enabled: bool = True, control_group=None, pseudo_capture: bool = False,
                 accum_grad: int = 1):
        self.model = model
        # accum_grad > 1 (trainer.py:619-653): two graphs per input shape — the micro-step
        # (forward + backward accumulating into the gradient arena) and the micro-step that ends
        # with clip + Adam + WarmupLR + zero_grad — chosen per call by iiter % accum_grad
        self.accum_grad = max(1, int(accum_grad))
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
        self.control_group = control_group  # kept for callers; the runner issues no collective
        self.pseudo = pseudo_capture
        self.failed = False       # a capture failed on this rank
        self.captures = []        # (call index, key) of every capture on this rank
        self.calls = 0
        self._fail_keys = set()   # tests: keys whose capture raises on this rank
        if dp is not None and dp.active and _backend(dp.group) == "gloo" and not pseudo_capture:
            self.enabled = False  # gloo collectives (host copies) cannot be captured
        if enabled and dp is not None and dp.active and _backend(dp.group) == "nccl":
            import os
            if os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") != "0":
                # recycled RCCL events inside captured collectives intermittently abort the
                # process: refuse instead of failing some runs later
                raise RuntimeError("TORCH_NCCL_CUDA_EVENT_CACHE is not '0' for this process group: call "
                                   "train.graph.prepare_nccl_env() before init_process_group")
        # "graph" once steps replay, "eager" once capture was given up; None while the
        # warm-up steps run
        self.mode = None if self.enabled else "eager"

    # ------------------------------------------------------------------ multi-rank control
    def capture_failed_flag(self) -> int:
        """1 when a capture failed on this rank (sent in the per-step control all-reduce)."""
        return 1 if self.failed else 0

    def force_eager(self):
        """Every later step eager (another rank's capture failed, or this one's): called at the
        same step on every rank from the control all-reduce's result."""
        if self.enabled or self.graphs:
            torch.cuda.synchronize()
        self.enabled = False
        self.mode = "eager"
        self.graphs.clear()

    # ------------------------------------------------------------------ helpers
    def _eager(self, batch, maxlens, update=True):
        return Trainer.train_one_step(self.model, batch, self.optimizer, self.scheduler,
                                      grad_clip=self.grad_clip, accum_grad=self.accum_grad,
                                      iiter=self.accum_grad if update else 1, dp=self.dp, maxlens=maxlens)

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
    def __call__(self, batch: Dict[str, torch.Tensor], maxlens: Optional[tuple] = None, lens_host=None,
                 iiter: int = 1):
        """One training step on `batch`; returns (loss, stats, weight, grad_norm).
        `lens_host`: the speech lengths as host ints when the batch's live on the device
        (SpecAug's per-utterance warp draws need them).  `iiter`: the epoch's 1-based batch
        index; with accum_grad > 1 the parameters update when iiter % accum_grad == 0."""
        if maxlens is None:
            maxlens = self._maxlens(batch)
        self.calls += 1
        update = iiter % self.accum_grad == 0
        if not self.enabled:
            return self._eager(batch, maxlens, update)
        B, _, F = batch["speech"].shape
        key = (B, maxlens[0], F, maxlens[1], update)
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
                    out = self._eager(dbatch, maxlens, update)
                main.wait_stream(self._side)
                return out
            err = None
            try:
                cap = self._capture(key, dbatch, maxlens, update)
            except RuntimeError as e:
                cap, err = None, e
                self._reset_after_failed_capture()
            if cap is not None:
                self.graphs[key] = cap
                self.captures.append((self.calls, key))
                self.mode = "graph"
                cap.graph.replay()  # capture executes nothing: run this batch's step now
                return cap.outputs
            # a stack that cannot capture this step (e.g. a collective library without graph
            # support on some node): warn once and run every step eagerly on this rank; the
            # control all-reduce turns the other ranks eager at the next step.  Capture
            # executes nothing, so the step is simply run now.
            import warnings
            warnings.warn(f"hipGraph capture of the training step failed ({err}); running eager steps")
            self.failed = True
            self.force_eager()
            return self._eager(dbatch, maxlens, update)
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

    def _capture(self, key, dbatch, maxlens, update=True):
        if key in self._fail_keys or key[:4] in self._fail_keys:
            raise RuntimeError(f"injected capture failure for {key}")
        cap = _Captured()
        cap.inputs = dbatch  # static input buffers (own storage)
        cap.maxlens = maxlens
        cap.update = update
        if self.pseudo:
            cap.graph = _PseudoGraph(self, cap)
            cap.outputs = None
            return cap
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        # the watchdog must hold no eager work of the RCCL group whose stream joins the capture
        _retire_pending_works(self.dp.group if self.dp is not None and self.dp.active else None)
        # thread-local capture mode: other threads' HIP calls during the capture (RCCL's
        # process-group watchdog polls its events) must not invalidate it or fail themselves
        with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
            out = self._eager(cap.inputs, maxlens, update)
        if self._pool is None:
            self._pool = g.pool()
        cap.graph = g
        cap.outputs = out
        return cap
