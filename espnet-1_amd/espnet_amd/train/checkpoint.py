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


class EpochReporter:
    """reporter.py: stats[epoch][phase][key] = value; epoch = the current epoch."""

    def __init__(self, epoch: int = 0):
        self.epoch = epoch
        self.stats: Dict[int, Dict[str, Dict[str, float]]] = {}

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def get_epoch(self) -> int:
        return self.epoch

    def register(self, phase: str, values: Dict[str, float], epoch: int = None):
        e = self.epoch if epoch is None else epoch
        self.stats.setdefault(e, {}).setdefault(phase, {}).update({k: float(v) for k, v in values.items()})

    def has(self, key: str, key2: str, epoch: int = None) -> bool:
        epoch = self.get_epoch() if epoch is None else epoch
        return epoch in self.stats and key in self.stats[epoch] and key2 in self.stats[epoch][key]

    def sort_epochs_and_values(self, key: str, key2: str, mode: str):
        if mode not in ("min", "max"):
            raise ValueError(f"mode must min or max: {mode}")
        if not self.has(key, key2):
            raise KeyError(f"{key}.{key2} is not found")
        values = [(e, self.stats[e][key][key2]) for e in self.stats]
        return sorted(values, key=(lambda x: x[1]) if mode == "min" else (lambda x: -x[1]))

    def sort_epochs(self, key, key2, mode):
        return [e for e, _ in self.sort_epochs_and_values(key, key2, mode)]

    def get_best_epoch(self, key, key2, mode, nbest: int = 0) -> int:
        return self.sort_epochs(key, key2, mode)[nbest]

    def state_dict(self):
        return {"stats": self.stats, "epoch": self.epoch}

    def load_state_dict(self, state_dict):
        self.epoch = state_dict["epoch"]
        self.stats = state_dict["stats"]


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


@torch.no_grad()
def average_nbest_models(output_dir, reporter, best_model_criterion: Sequence[Sequence[str]],
                         nbest: Union[Collection[int], int], suffix: Optional[str] = None) -> None:
    """average_nbest_models.py:13-108, including its reuse of the first loaded epoch's dict
    as the accumulator (so with several nbest values a later average starts from the
    earlier sum, exactly as the reference does)."""
    output_dir = Path(output_dir)
    nbests = [nbest] if isinstance(nbest, int) else list(nbest)
    if len(nbests) == 0:
        warnings.warn("At least 1 nbest values are required")
        nbests = [1]
    suffix = suffix + "." if suffix is not None else ""
    nbest_epochs = [(ph, k, reporter.sort_epochs_and_values(ph, k, m)[: max(nbests)])
                    for ph, k, m in best_model_criterion if reporter.has(ph, k)]
    _loaded = {}
    for ph, cr, epoch_and_values in nbest_epochs:
        _nbests = [i for i in nbests if i <= len(epoch_and_values)] or [1]
        for n in _nbests:
            if n == 0:
                continue
            if n == 1:
                e, _ = epoch_and_values[0]
                op = output_dir / f"{e}epoch.pth"
                sym_op = output_dir / f"{ph}.{cr}.ave_1best.{suffix}pth"
                if sym_op.is_symlink() or sym_op.exists():
                    sym_op.unlink()
                sym_op.symlink_to(op.name)
            else:
                op = output_dir / f"{ph}.{cr}.ave_{n}best.{suffix}pth"
                logging.info(f'Averaging {n}best models: criterion="{ph}.{cr}": {op}')
                avg = None
                for e, _ in epoch_and_values[:n]:
                    if e not in _loaded:
                        _loaded[e] = _load(output_dir / f"{e}epoch.pth")
                    states = _loaded[e]
                    if avg is None:
                        avg = states
                    else:
                        for k in avg:
                            avg[k] = avg[k] + states[k]
                for k in avg:
                    if not str(avg[k].dtype).startswith("torch.int"):
                        avg[k] = avg[k] / n
                torch.save(avg, op)
        op = output_dir / f"{ph}.{cr}.ave_{max(_nbests)}best.{suffix}pth"
        sym_op = output_dir / f"{ph}.{cr}.ave.{suffix}pth"
        if sym_op.is_symlink() or sym_op.exists():
            sym_op.unlink()
        sym_op.symlink_to(op.name)
