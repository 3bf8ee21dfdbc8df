"""Reporter / SubReporter — the statistics bookkeeping of espnet2/train/reporter.py
(Reporter :283-560, SubReporter :112-280), same keys, aggregation and state layout.

MI355X-first difference: the reference converts every registered tensor with .item()
(reporter.py:27-44), a host synchronisation per stat per step.  Here a registered device
tensor is kept as-is and resolved lazily — all pending values of a window in ONE
device->host copy when a log line or the epoch summary needs them — so a training step
(a replayed hipGraph) never waits for the host.  The aggregation rules are the
reference's: Average = nanmean; WeightedAverage = sum(v*w)/sum(w) over entries whose value
and weight are finite; a key missing in a step counts as NaN for that step.
"""
from __future__ import annotations

import datetime
import logging
import time
import warnings
from contextlib import contextmanager
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

_RESERVED = {"time", "total_count"}


class _Series:
    """One stat's per-step values (floats or pending device scalars) and weights."""

    __slots__ = ("weighted", "values", "weights")

    def __init__(self, weighted: bool):
        self.weighted = weighted
        self.values: List = []
        self.weights: List = []

    def append(self, v, w):
        self.values.append(v)
        self.weights.append(w)

    def resolve(self, start: int, end: int):
        """Materialise [start, end) as float arrays; device values in one transfer."""
        vals, wts = self.values[start:end], self.weights[start:end]
        dev_idx = [i for i, v in enumerate(vals) if isinstance(v, torch.Tensor)]
        dev_w = [i for i, w in enumerate(wts) if isinstance(w, torch.Tensor)]
        if dev_idx or dev_w:
            flat = [vals[i].detach().reshape(-1)[:1].float() for i in dev_idx] + \
                   [wts[i].detach().reshape(-1)[:1].float() for i in dev_w]
            host = torch.cat([t.to(flat[0].device) for t in flat]).cpu().tolist()
            for j, i in enumerate(dev_idx):
                self.values[start + i] = vals[i] = host[j]
            for j, i in enumerate(dev_w):
                self.weights[start + i] = wts[i] = host[len(dev_idx) + j]
        return np.asarray(vals, dtype=np.float64), np.asarray(wts, dtype=np.float64)

    def aggregate(self, start: int = 0, end: Optional[int] = None) -> float:
        end = len(self.values) if end is None else end
        v, w = self.resolve(start, end)
        if len(v) == 0:
            warnings.warn("No stats found")
            return float("nan")
        if not self.weighted:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                return float(np.nanmean(v))
        ok = np.isfinite(v) & np.isfinite(w)
        if not ok.any():
            warnings.warn("No valid stats found")
            return float("nan")
        sw = float(w[ok].sum())
        if sw == 0:
            warnings.warn("weight is zero")
            return float("nan")
        return float((v[ok] * w[ok]).sum() / sw)


def _check_scalar(v, what):
    if isinstance(v, (torch.Tensor, np.ndarray)) and int(np.prod(v.shape)) != 1:
        raise ValueError(f"{what} must be 0 or 1 dimension: {len(v.shape)}")


def _fmt(key2, v):
    if abs(v) > 1.0e3:
        return f"{key2}={v:.3e}"
    if abs(v) > 1.0e-3:
        return f"{key2}={v:.3f}"
    return f"{key2}={v:.3e}"


class SubReporter:
    def __init__(self, key: str, epoch: int, total_count: int):
        self.key = key
        self.epoch = epoch
        self.start_time = time.perf_counter()
        self.stats: Dict[str, _Series] = {}
        self._finished = False
        self.total_count = total_count
        self.count = 0
        self._seen = set()

    def get_total_count(self) -> int:
        return self.total_count

    def get_epoch(self) -> int:
        return self.epoch

    def register(self, stats: Dict, weight=None) -> None:
        if self._finished:
            raise RuntimeError("Already finished")
        if not self._seen:
            self.total_count += 1
            self.count += 1
        if weight is not None:
            _check_scalar(weight, "weight")
        for key2, v in stats.items():
            if key2 in _RESERVED:
                raise RuntimeError(f"{key2} is reserved.")
            if key2 in self._seen:
                raise RuntimeError(f"{key2} is registered twice.")
            if v is None:
                v = float("nan")
            _check_scalar(v, "v")
            if isinstance(v, np.ndarray):
                v = float(v.reshape(-1)[0])
            s = self.stats.get(key2)
            if s is None:
                s = self.stats[key2] = _Series(weight is not None)
                for _ in range(self.count - 1):  # earlier steps without this key
                    s.append(float("nan"), 0.0 if weight is not None else None)
            s.append(v, weight if weight is not None else None)
            self._seen.add(key2)

    def next(self):
        """Close the step: keys not registered in it get NaN (reporter.py:135-150)."""
        for key2, s in self.stats.items():
            if key2 not in self._seen:
                s.append(float("nan"), 0.0 if s.weighted else None)
            assert len(s.values) == self.count, (key2, len(s.values), self.count)
        self._seen = set()

    def log_message(self, start: int = None, end: int = None) -> str:
        if self._finished:
            raise RuntimeError("Already finished")
        start = 0 if start is None else (self.count + start if start < 0 else start)
        end = self.count if end is None else end
        if self.count == 0 or start == end:
            return ""
        msg = f"{self.epoch}epoch:{self.key}:{start + 1}-{end}batch: "
        for idx, (k, s) in enumerate(self.stats.items()):
            # the reference separates keys with ", " except before key number `count` (it
            # compares the key index with the number of steps, reporter.py:190) - kept, so the
            # log lines are byte-identical
            if idx != 0 and idx != self.count:
                msg += ", "
            msg += _fmt(k, s.aggregate(start, end))
        return msg

    def finished(self) -> None:
        self._finished = True

    @contextmanager
    def measure_time(self, name: str):
        start = time.perf_counter()
        yield start
        self.register({name: time.perf_counter() - start})

    def measure_iter_time(self, iterable, name: str):
        it = iter(iterable)
        while True:
            start = time.perf_counter()
            try:
                item = next(it)
            except StopIteration:
                break
            self.register({name: time.perf_counter() - start})
            yield item


class Reporter:
    """stats[epoch][key][key2] = aggregated value; {"stats", "epoch"} is the checkpoint
    state (trainer.py:348-360), readable by the reference and vice versa."""

    def __init__(self, epoch: int = 0):
        if epoch < 0:
            raise ValueError(f"epoch must be 0 or more: {epoch}")
        self.epoch = epoch
        self.stats: Dict[int, Dict[str, Dict]] = {}

    def get_epoch(self) -> int:
        return self.epoch

    def set_epoch(self, epoch: int) -> None:
        if epoch < 0:
            raise ValueError(f"epoch must be 0 or more: {epoch}")
        self.epoch = epoch

    @contextmanager
    def observe(self, key: str, epoch: int = None):
        sub = self.start_epoch(key, epoch)
        yield sub
        self.finish_epoch(sub)

    def start_epoch(self, key: str, epoch: int = None) -> SubReporter:
        if epoch is not None:
            self.set_epoch(epoch)
        prev = self.stats.get(self.epoch - 1, {})
        if key not in prev:
            if self.epoch - 1 != 0:
                warnings.warn(f"The stats of the previous epoch={self.epoch - 1}doesn't exist.")
            total = 0
        else:
            total = prev[key]["total_count"]
        self.stats.pop(epoch, None)
        return SubReporter(key, self.epoch, total)

    def finish_epoch(self, sub: SubReporter) -> None:
        if self.epoch != sub.epoch:
            raise RuntimeError(f"Don't change epoch during observation: {self.epoch} != {sub.epoch}")
        stats = {k: s.aggregate() for k, s in sub.stats.items()}
        stats["time"] = datetime.timedelta(seconds=time.perf_counter() - sub.start_time)
        stats["total_count"] = sub.total_count
        if torch.cuda.is_initialized():
            stats["gpu_max_cached_mem_GB"] = torch.cuda.max_memory_reserved() / 2 ** 30
        self.stats.setdefault(self.epoch, {})[sub.key] = stats
        sub.finished()

    # ------------------------------------------------------------------ queries
    def register(self, phase: str, values: Dict[str, float], epoch: int = None):
        """Set epoch-level values directly (tests, resumed runs)."""
        e = self.epoch if epoch is None else epoch
        self.stats.setdefault(e, {}).setdefault(phase, {}).update({k: float(v) for k, v in values.items()})

    def has(self, key: str, key2: str, epoch: int = None) -> bool:
        epoch = self.get_epoch() if epoch is None else epoch
        return epoch in self.stats and key in self.stats[epoch] and key2 in self.stats[epoch][key]

    def sort_epochs_and_values(self, key: str, key2: str, mode: str) -> List[Tuple[int, float]]:
        if mode not in ("min", "max"):
            raise ValueError(f"mode must min or max: {mode}")
        if not self.has(key, key2):
            raise KeyError(f"{key}.{key2} is not found: {self.get_all_keys()}")
        values = [(e, self.stats[e][key][key2]) for e in self.stats]
        return sorted(values, key=(lambda x: x[1]) if mode == "min" else (lambda x: -x[1]))

    def sort_epochs(self, key, key2, mode) -> List[int]:
        return [e for e, _ in self.sort_epochs_and_values(key, key2, mode)]

    def sort_values(self, key, key2, mode) -> List[float]:
        return [v for _, v in self.sort_epochs_and_values(key, key2, mode)]

    def get_best_epoch(self, key, key2, mode, nbest: int = 0) -> int:
        return self.sort_epochs(key, key2, mode)[nbest]

    def check_early_stopping(self, patience: int, key1: str, key2: str, mode: str, epoch: int = None,
                             logger=None) -> bool:
        logger = logging if logger is None else logger
        epoch = self.get_epoch() if epoch is None else epoch
        best = self.get_best_epoch(key1, key2, mode)
        if epoch - best > patience:
            logger.info(f"[Early stopping] {key1}.{key2} has not been improved {epoch - best} epochs "
                        f"continuously. The training was stopped at {epoch}epoch")
            return True
        return False

    def get_value(self, key: str, key2: str, epoch: int = None):
        if not self.has(key, key2):
            raise KeyError(f"{key}.{key2} is not found in stats: {self.get_all_keys()}")
        epoch = self.get_epoch() if epoch is None else epoch
        return self.stats[epoch][key][key2]

    def get_keys(self, epoch: int = None) -> Tuple[str, ...]:
        return tuple(self.stats[self.get_epoch() if epoch is None else epoch])

    def get_keys2(self, key: str, epoch: int = None) -> Tuple[str, ...]:
        d = self.stats[self.get_epoch() if epoch is None else epoch][key]
        return tuple(k for k in d if k not in _RESERVED)

    def get_all_keys(self, epoch: int = None) -> Tuple[Tuple[str, str], ...]:
        epoch = self.get_epoch() if epoch is None else epoch
        return tuple((k, k2) for k in self.stats.get(epoch, {}) for k2 in self.stats[epoch][k])

    def log_message(self, epoch: int = None) -> str:
        epoch = self.get_epoch() if epoch is None else epoch
        blocks = []
        for key, d in self.stats.get(epoch, {}).items():
            parts = []
            for key2, v in d.items():
                if v is None:
                    continue
                if isinstance(v, float):
                    parts.append(_fmt(key2, v))
                elif isinstance(v, datetime.timedelta):
                    parts.append(f"{key2}={v.total_seconds():.3f} seconds")
                else:
                    parts.append(f"{key2}={v}")
            if parts:
                blocks.append(f"[{key}] " + ", ".join(parts))
        return (f"{epoch}epoch results: " + ", ".join(blocks)) if blocks else ""

    def state_dict(self):
        return {"stats": self.stats, "epoch": self.epoch}

    def load_state_dict(self, state_dict: dict):
        self.epoch = state_dict["epoch"]
        self.stats = state_dict["stats"]


# a checkpoint's reporter state holds datetime.timedelta values ("time"): allow exactly that
# type in torch.load(weights_only=True)
torch.serialization.add_safe_globals([datetime.timedelta])
