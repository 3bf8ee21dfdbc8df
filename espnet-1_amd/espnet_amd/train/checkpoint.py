"""Checkpoint / model-file interop with the reference trainer:

* ``save_checkpoint``  — espnet2/train/trainer.py:348-360: ``checkpoint.pth`` =
  {"model", "reporter", "optimizers", "schedulers", "scaler"}; the model state_dict has the
  reference's key layout and the optimizer state is torch.optim.Adam's per-parameter layout
  (ArenaAdam.state_dict), so a reference run resumes from it and vice versa.
* ``save_epoch_model`` — trainer.py:362-369: ``{epoch}epoch.pth`` (model state_dict) and the
  ``latest.pth`` symlink.
* ``resume`` — Trainer.resume, trainer.py:133-159.
* ``average_nbest_models`` — espnet2/main_funcs/average_nbest_models.py:13-108 (float
  entries averaged, integer entries such as BatchNorm.num_batches_tracked summed).
* ``EpochReporter`` — the part of espnet2/train/reporter.py the above read: per-epoch stats,
  ``has`` / ``sort_epochs_and_values`` / ``get_best_epoch`` and the {"stats", "epoch"} state.

Files are read with ``torch.load(weights_only=True)``: tensors, numbers, strings and
containers only, nothing is executed from a checkpoint.
"""
from __future__ import annotations

import logging
import warnings
from pathlib import Path
from typing import Collection, Dict, Optional, Sequence, Tuple, Union

import torch


from .reporter import Reporter

# the per-epoch reporter the checkpoint / averaging code reads (train/reporter.py)
EpochReporter = Reporter


def _load(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def save_checkpoint(output_dir, model, reporter, optimizers: Sequence, schedulers: Sequence, scaler=None):
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    torch.save({
        "model": model.state_dict(),
        "reporter": reporter.state_dict(),
        "optimizers": [o.state_dict() for o in optimizers],
        "schedulers": [s.state_dict() if s is not None else None for s in schedulers],
        "scaler": scaler.state_dict() if scaler is not None else None,
    }, output_dir / "checkpoint.pth")


def save_epoch_model(output_dir, model, iepoch: int):
    output_dir = Path(output_dir)
    torch.save(model.state_dict(), output_dir / f"{iepoch}epoch.pth")
    p = output_dir / "latest.pth"
    if p.is_symlink() or p.exists():
        p.unlink()
    p.symlink_to(f"{iepoch}epoch.pth")


def resume(checkpoint, model, reporter, optimizers: Sequence, schedulers: Sequence, scaler=None, ngpu: int = 0):
    """trainer.py:133-159.  The model may be prepared (arena on the device) already:
    load_state_dict copies into the arena views."""
    states = _load(checkpoint, map_location=f"cuda:{torch.cuda.current_device()}" if ngpu > 0 else "cpu")
    model.load_state_dict(states["model"])
    reporter.load_state_dict(states["reporter"])
    for optimizer, state in zip(optimizers, states["optimizers"]):
        optimizer.load_state_dict(state)
    for scheduler, state in zip(schedulers, states["schedulers"]):
        if scheduler is not None:
            scheduler.load_state_dict(state)
    if scaler is not None:
        if states["scaler"] is None:
            logging.warning("scaler state is not found")
        else:
            scaler.load_state_dict(states["scaler"])
    logging.info(f"The training was resumed using {checkpoint}")


def _relink(link: Path, target: str):
    if link.is_symlink() or link.exists():
        link.unlink()
    link.symlink_to(target)


def _sum_into(running: Dict[str, torch.Tensor], other: Dict[str, torch.Tensor]):
    for key in running:
        running[key] = running[key] + other[key]


def _divide_floats(running: Dict[str, torch.Tensor], n: int):
    """Entries become means except the torch.int* ones (BatchNorm num_batches_tracked), which
    stay sums — the reference's dtype-name test (average_nbest_models.py:90-98), so bool /
    uint8 entries are averaged too."""
    for key, v in running.items():
        if not str(v.dtype).startswith("torch.int"):
            running[key] = v / n


@torch.no_grad()
def average_nbest_models(output_dir, reporter, best_model_criterion: Sequence[Sequence[str]],
                         nbest: Union[Collection[int], int], suffix: Optional[str] = None) -> None:
    """main_funcs/average_nbest_models.py:13-108: for each criterion with values, link
    {phase}.{key}.ave_1best to the best epoch file, write {phase}.{key}.ave_{n}best as the
    mean of the n best epoch files (integer tensors summed), and link {phase}.{key}.ave to
    the largest average.

    Observable detail kept from the reference: the state dicts read from disk are cached per
    epoch and an average is accumulated INTO the cached dict of its best epoch, so a later
    (larger-n) average of the same criterion, or of another criterion whose list contains
    that epoch, starts from that already-averaged dict.  The files written are therefore
    bit-identical to the reference's (tests/test_checkpoint.py against its output)."""
    output_dir = Path(output_dir)
    sizes = [nbest] if isinstance(nbest, int) else list(nbest)
    if not sizes:
        warnings.warn("At least 1 nbest values are required")
        sizes = [1]
    tag = "" if suffix is None else suffix + "."
    cache: Dict[int, Dict[str, torch.Tensor]] = {}

    def state_of(epoch: int) -> Dict[str, torch.Tensor]:
        if epoch not in cache:
            cache[epoch] = _load(output_dir / f"{epoch}epoch.pth")
        return cache[epoch]

    for phase, key, mode in best_model_criterion:
        if not reporter.has(phase, key):
            continue
        ranked = [e for e, _ in reporter.sort_epochs_and_values(phase, key, mode)[: max(sizes)]]
        usable = [n for n in sizes if n <= len(ranked)] or [1]
        stem = f"{phase}.{key}"
        for n in usable:
            if n == 0:
                continue
            if n == 1:
                _relink(output_dir / f"{stem}.ave_1best.{tag}pth", f"{ranked[0]}epoch.pth")
                continue
            out = output_dir / f"{stem}.ave_{n}best.{tag}pth"
            logging.info(f'Averaging {n}best models: criterion="{stem}": {out}')
            running = state_of(ranked[0])
            for e in ranked[1:n]:
                _sum_into(running, state_of(e))
            _divide_floats(running, n)
            torch.save(running, out)
        _relink(output_dir / f"{stem}.ave.{tag}pth", f"{stem}.ave_{max(usable)}best.{tag}pth")
