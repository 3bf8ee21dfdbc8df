"""Trainer — espnet2/train/trainer.py on the HIP path.

train_one_step (one minibatch, trainer.py:562-701):
  model(**batch) -> (loss, stats, weight)                               (:567)
  DP weighting: loss*weight / sum_ranks(weight); stats weighted-averaged (:604-619)
  loss / accum_grad; backward -> gradient all-reduce over RCCL (SUM; the /world of DDP is
  folded into the loss weight)                                           (:619-632, K1)
  every accum_grad-th call: clip_grad_norm_(grad_clip) + skip if non-finite + Adam +
  WarmupLR + zero_grad                                                   (:653-701)
The clip coefficient and the finite check live on the device (ArenaAdam), so a step
issues no host synchronisation; the grad norm is returned as a device tensor.

train_one_epoch / validate_one_epoch / run (:162-470, :472-783): the epoch loop around it
with the reference's reporter keys (iter_time, forward_time, backward_time,
optim_step_time, train_time, optim0_lr0, the model's stats), the per-step iterator_stop
all-reduce of uneven DP iterators (:507-518, :727-730), checkpoint / epoch model files /
best-model links / n-best averaging (train/checkpoint.py) and early stopping.

MI355X-first: steps whose shapes repeat are captured once as a hipGraph and replayed
(train/graph.py); the forward / backward / optimizer times come from stream-ordered
device stamps inside the step (ea_phase_stamp: they are measured on every replay), the
stats are snapshotted on the device, and the reporter reads both back in one transfer per
log line — no host synchronisation inside the step.  The iterator_stop flag travels over a
gloo group (host memory), so checking it never waits for the GPU either.
"""
from __future__ import annotations

import dataclasses
import logging
import math
import time
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Union

import torch
import torch.distributed as dist

from .. import hip_ops as ops
from .._lib import lib
from ..optim.adam import ArenaAdam


@dataclasses.dataclass
class TrainerOptions:
    """trainer.py:64-93."""
    ngpu: int
    resume: bool
    use_amp: bool
    train_dtype: str
    grad_noise: bool
    accum_grad: int
    grad_clip: float
    grad_clip_type: float
    log_interval: Optional[int]
    no_forward_run: bool
    use_matplotlib: bool
    use_tensorboard: bool
    use_wandb: bool
    output_dir: Union[Path, str]
    max_epoch: int
    seed: int
    sharded_ddp: bool
    patience: Optional[int]
    keep_nbest_models: Union[int, List[int]]
    nbest_averaging_interval: int
    early_stopping_criterion: Sequence[str]
    best_model_criterion: Sequence[Sequence[str]]
    val_scheduler_criterion: Sequence[str]
    unused_parameters: bool
    wandb_model_log_interval: int
    create_graph_in_tensorboard: bool


class PhaseTimer:
    """Device ring of per-step phase durations (ea_phase_stamp): row = step, columns =
    forward / backward / optimizer seconds and the lr the optimizer applied."""

    def __init__(self, device, cap: int = 8192):
        self.cap = cap
        self.state = torch.zeros(2, dtype=torch.int64, device=device)
        self.ring = torch.zeros(cap, 4, dtype=torch.float32, device=device)
        self.extra = None  # device float read at phase 3 (the applied lr)
        self.opt = None    # ea_opt_state (device): phase 3 reads next_lr and the skip flag
        self.count = 0     # host mirror of the device step counter

    def stamp(self, phase: int):
        if self.opt is not None:
            lib.ea_phase_stamp_opt(self.state.data_ptr(), self.ring.data_ptr(), self.cap, phase,
                                   self.opt.data_ptr(), ops.stream())
            return
        lib.ea_phase_stamp(self.state.data_ptr(), self.ring.data_ptr(), self.cap, phase,
                           None if self.extra is None else self.extra.data_ptr(), ops.stream())

    def slot(self):
        return self.count % self.cap


TIMER: Optional[PhaseTimer] = None  # set by train_one_epoch around its steps


def _stamp(phase):
    if TIMER is not None:
        TIMER.stamp(phase)


class Trainer:
    def __init__(self):
        raise RuntimeError("This class can't be instantiated.")

    @classmethod
    def build_options(cls, args) -> TrainerOptions:
        return TrainerOptions(**{f.name: getattr(args, f.name) for f in dataclasses.fields(TrainerOptions)})

    @classmethod
    def add_arguments(cls, parser):
        pass

    # ------------------------------------------------------------------ one minibatch
    @staticmethod
    def train_one_step(model, batch: Dict[str, torch.Tensor], optimizer: ArenaAdam, scheduler=None, *,
                       grad_clip: float = 5.0, accum_grad: int = 1, iiter: int = 1, dp=None, maxlens=None):
        _stamp(0)
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
        if accum_grad > 1:
            loss = loss / accum_grad
            if not (dp is not None and dp.active) and "loss" in stats:
                # the reference divides loss in place (trainer.py:619 `loss /= accum_grad`)
                # and its stats["loss"] is loss.detach() (espnet_model.py:326), the same
                # storage: single-process runs report loss / accum_grad
                stats = dict(stats, loss=stats["loss"] / accum_grad)
        _stamp(1)
        # gradients are all-reduced on the micro-step that updates (accum_grad > 1: the earlier
        # micro-steps accumulate locally).  The SUM over ranks of the accumulated gradients is
        # then sum_r sum_k g_k,r — DDP's result (trainer.py:229-244 reduces every micro-step's
        # accumulated .grad with a mean: mean_r(S + g_k,r) = S + mean_r g_k,r, the loss
        # weighting making mean and SUM agree); reducing every micro-step's SUM would count
        # the earlier micro-steps world_size times.
        reduce_now = dp is not None and dp.active and iiter % accum_grad == 0
        if reduce_now:
            dp.begin_backward()
        # the Linear weight gradients of the pass are queued and run as grouped GEMMs (at the
        # end of the pass, or per bucket from the DP hooks)
        with ops.deferred_wgrad():
            loss.backward()
        if reduce_now:
            dp.allreduce_grads()
        _stamp(2)
        grad_norm = None
        if iiter % accum_grad == 0:
            grad_norm = optimizer.compute_grad_norm()
            optimizer.step(grad_norm=grad_norm, max_norm=grad_clip)
            if scheduler is not None:
                scheduler.step()
            optimizer.zero_grad()
        _stamp(3)
        return loss.detach(), stats, weight, grad_norm

    # ------------------------------------------------------------------ epochs
    @classmethod
    def train_one_epoch(cls, model, iterator: Iterable, optimizers: Sequence, schedulers: Sequence, scaler=None,
                        reporter=None, summary_writer=None, options: TrainerOptions = None, distributed_option=None,
                        dp=None, step_runner=None) -> bool:
        """trainer.py:472-731.  Returns all_steps_are_invalid.  `step_runner` (a
        graph.CapturedTrainStep over the same model / optimizer) replays captured steps;
        without it every step is launched eagerly."""
        global TIMER
        accum_grad = options.accum_grad
        if step_runner is not None and step_runner.accum_grad != accum_grad:
            raise ValueError(f"step_runner.accum_grad={step_runner.accum_grad} != options.accum_grad={accum_grad}")
        distributed = distributed_option is not None and distributed_option.distributed
        log_interval = options.log_interval
        if log_interval is None:
            try:
                log_interval = max(len(iterator) // 20, 10)
            except TypeError:
                log_interval = 100
        model.train()
        optimizer = optimizers[0]
        scheduler = schedulers[0] if schedulers else None
        device = model._device
        timer = getattr(model, "_phase_timer", None)
        if timer is None:
            timer = model._phase_timer = PhaseTimer(device)
        # ea_opt_state: next_lr (the lr after scheduler.step(), which the reference registers)
        # and the skip flag (a skipped update's optimizer time is NaN: not registered)
        timer.opt = optimizer.state_dev
        # applied updates are counted on the device (a non-finite grad norm skips the update
        # there); read once at the end of the epoch for all_steps_are_invalid (trainer.py:681)
        applied0 = optimizer.state_dev[0].clone()
        # the reference's per-step iterator_stop all-reduce (trainer.py:507-518) over the gloo
        # control group; its message also carries "a capture failed on some rank" so every rank
        # turns eager at the same step (graph.CapturedTrainStep decides captures per rank)
        ctl = torch.zeros(2, dtype=torch.long)
        ctrl = getattr(distributed_option, "control_group", None)
        ran_no_forward = False
        unread = 0
        start = time.perf_counter()
        TIMER = timer
        try:
            for iiter, (utt_id, batch) in enumerate(reporter.measure_iter_time(iterator, "iter_time"), 1):
                assert isinstance(batch, dict), type(batch)
                if distributed:
                    ctl[0] = 0
                    ctl[1] = step_runner.capture_failed_flag() if step_runner is not None else 0
                    dist.all_reduce(ctl, group=ctrl)
                    if int(ctl[0]) > 0:
                        break
                    if int(ctl[1]) > 0 and step_runner is not None and step_runner.mode != "eager":
                        step_runner.force_eager()
                if options.no_forward_run:
                    ran_no_forward = True
                    continue
                # the padded maxima from the host copy of the lengths (no device read)
                maxlens = (int(batch["speech_lengths"].max()), int(batch["text_lengths"].max())) \
                    if "speech_lengths" in batch and "text_lengths" in batch else None
                lens_host = batch["speech_lengths"].tolist() if "speech_lengths" in batch else None
                batch = {k: v.to(device, non_blocking=True) if isinstance(v, torch.Tensor) else v
                         for k, v in batch.items()}
                update = iiter % accum_grad == 0
                if step_runner is not None:
                    loss, stats, weight, gn = step_runner(batch, maxlens, lens_host=lens_host, iiter=iiter)
                else:
                    loss, stats, weight, gn = cls.train_one_step(model, batch, optimizer, scheduler,
                                                                 grad_clip=options.grad_clip, accum_grad=accum_grad,
                                                                 iiter=iiter, dp=dp, maxlens=maxlens)
                # snapshot the step's stats on the device (replayed graph outputs are overwritten)
                keys = sorted(stats)
                snap = torch.cat([stats[k].detach().reshape(1).float() for k in keys] + [weight.reshape(1).float()])
                slot = timer.slot()
                timer.count += 1
                reporter.register({k: snap[i] for i, k in enumerate(keys)}, snap[-1])
                reporter.register({"forward_time": timer.ring[slot, 0], "backward_time": timer.ring[slot, 1]})
                if update:
                    # a non-finite gradient skips the update on the device (ArenaAdam); its
                    # optim_step_time is NaN there, which the epoch average ignores like the
                    # reference's missing entry
                    reporter.register({"optim_step_time": timer.ring[slot, 2], "optim0_lr0": timer.ring[slot, 3],
                                       "train_time": time.perf_counter() - start})
                    start = time.perf_counter()
                unread += 1
                reporter.next()
                if iiter % log_interval == 0:
                    logging.info(reporter.log_message(-log_interval))
                    unread = 0
                if unread >= timer.cap // 2:  # read the device ring before it wraps
                    for s in reporter.stats.values():
                        s.resolve(0, len(s.values))
                    unread = 0
            else:
                if distributed:
                    ctl[0] = 1
                    ctl[1] = step_runner.capture_failed_flag() if step_runner is not None else 0
                    dist.all_reduce(ctl, group=ctrl)
                    if int(ctl[1]) > 0 and step_runner is not None and step_runner.mode != "eager":
                        step_runner.force_eager()
        finally:
            TIMER = None
        applied = int((optimizer.state_dev[0] - applied0).item())
        return not (ran_no_forward or applied > 0)

    @staticmethod
    @torch.no_grad()
    def validate_one_epoch(model, iterator: Iterable, dp=None, device="cuda", reporter=None, options=None,
                           distributed_option=None) -> Dict[str, float]:
        """trainer.py:735-783 plus the epoch summary of SubReporter (reporter.py aggregate,
        WeightedAverage): eval mode, one forward per minibatch (CER/WER come from the model's
        ErrorCalculator), stats weighted-averaged across ranks per batch and then across
        batches by batch weight, skipping None and non-finite values.  Ranks whose iterators
        run out first stop everyone through the reference's iterator_stop all-reduce.
        `device` holds the stop flag: "cuda" for RCCL, "cpu" for gloo; with a
        distributed_option that has a gloo control group the flag goes over it.  With a
        reporter, every batch's stats are also registered into it."""
        was_training = model.training
        model.eval()
        distributed = dp is not None and dp.active
        group = dp.group if distributed else None
        ctrl = getattr(distributed_option, "control_group", None)
        if ctrl is not None:
            group, device = ctrl, "cpu"
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
            if reporter is not None:
                reporter.register(stats, weight)
                reporter.next()
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

    @classmethod
    def run(cls, model, optimizers, schedulers, train_iter_factory, valid_iter_factory,
            plot_attention_iter_factory, trainer_options: TrainerOptions, distributed_option) -> None:
        """trainer.py:162-470."""
        from .checkpoint import average_nbest_models, resume, save_checkpoint, save_epoch_model
        from .distributed import ArenaDataParallel
        from .graph import CapturedTrainStep
        from .reporter import Reporter
        opts = trainer_options
        keep = [opts.keep_nbest_models] if isinstance(opts.keep_nbest_models, int) else \
            (list(opts.keep_nbest_models) or [1])
        output_dir = Path(opts.output_dir)
        reporter = Reporter()
        distributed = distributed_option.distributed
        rank0 = not distributed or distributed_option.dist_rank == 0
        if opts.resume and (output_dir / "checkpoint.pth").exists():
            resume(output_dir / "checkpoint.pth", model, reporter, optimizers, schedulers, ngpu=opts.ngpu)
        start_epoch = reporter.get_epoch() + 1
        if start_epoch == opts.max_epoch + 1:
            logging.warning(f"The training has already reached at max_epoch: {start_epoch}")
        dp = ArenaDataParallel(model) if distributed else None
        # steps whose shapes repeat are captured and replayed; with accum_grad > 1 the micro-step
        # and the updating micro-step are two graphs per shape
        runner = CapturedTrainStep(model, optimizers[0], schedulers[0] if schedulers else None,
                                   grad_clip=opts.grad_clip, dp=dp, warmup=2, accum_grad=opts.accum_grad,
                                   control_group=getattr(distributed_option, "control_group", None))
        all_invalid = False
        for iepoch in range(start_epoch, opts.max_epoch + 1):
            logging.info(f"{iepoch}/{opts.max_epoch}epoch started")
            _seed_all(opts.seed + iepoch)
            reporter.set_epoch(iepoch)
            with reporter.observe("train") as sub:
                all_invalid = cls.train_one_epoch(model=model, iterator=train_iter_factory.build_iter(iepoch),
                                                  optimizers=optimizers, schedulers=schedulers, reporter=sub,
                                                  options=opts, distributed_option=distributed_option, dp=dp,
                                                  step_runner=runner)
            with reporter.observe("valid") as sub:
                cls.validate_one_epoch(model, valid_iter_factory.build_iter(iepoch), dp=dp, reporter=sub,
                                       distributed_option=distributed_option)
            if rank0:
                logging.info(reporter.log_message())
                save_checkpoint(output_dir, model, reporter, optimizers, schedulers)
                save_epoch_model(output_dir, model, iepoch)
                improved = []
                for ph, k, mode in opts.best_model_criterion:
                    if reporter.has(ph, k) and reporter.get_best_epoch(ph, k, mode) == iepoch:
                        p = output_dir / f"{ph}.{k}.best.pth"
                        if p.is_symlink() or p.exists():
                            p.unlink()
                        p.symlink_to(f"{iepoch}epoch.pth")
                        improved.append(f"{ph}.{k}")
                logging.info("The best model has been updated: " + ", ".join(improved) if improved
                             else "There are no improvements in this epoch")
                nbests = set().union(*[set(reporter.sort_epochs(ph, k, m)[: max(keep)])
                                       for ph, k, m in opts.best_model_criterion if reporter.has(ph, k)])
                if opts.nbest_averaging_interval > 0 and iepoch % opts.nbest_averaging_interval == 0:
                    average_nbest_models(output_dir, reporter, opts.best_model_criterion, keep,
                                         suffix=f"till{iepoch}epoch")
                for e in range(1, iepoch):
                    p = output_dir / f"{e}epoch.pth"
                    if p.exists() and e not in nbests:
                        p.unlink()
            if all_invalid:
                logging.warning(f"The gradients at all steps are invalid in this epoch. Something seems wrong. "
                                f"This training was stopped at {iepoch}epoch")
                break
            if opts.patience is not None and reporter.check_early_stopping(opts.patience,
                                                                           *opts.early_stopping_criterion):
                break
        else:
            logging.info(f"The training was finished at {opts.max_epoch} epochs ")
        if rank0:
            average_nbest_models(output_dir, reporter, opts.best_model_criterion, keep)


def _seed_all(seed):
    import random

    import numpy as np
    random.seed(seed)
    np.random.seed(seed)
    torch.random.manual_seed(seed)
