"""SequenceIterFactory — espnet2/iterators/sequence_iter_factory.py:28-143: the per-epoch
mini-batch iterator.  Batches are shuffled with np.random.RandomState(epoch + seed) (so a
resumed run replays the same order), --num_iters_per_epoch windows over consecutive
shuffled epochs exactly as the reference does, and a torch DataLoader runs the dataset +
collate in `num_workers` processes seeded with base_seed + worker_id."""
from __future__ import annotations

import random
from functools import partial
from typing import Any, Sequence

import numpy as np
from torch.utils.data import DataLoader


def worker_init_fn(worker_id, base_seed=0):
    seed = base_seed + worker_id
    random.seed(seed)
    np.random.seed(seed)


class RawSampler:
    def __init__(self, batches):
        self.batches = batches

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        return iter(self.batches)

    def generate(self, seed):
        return list(self.batches)


class SequenceIterFactory:
    def __init__(self, dataset, batches, num_iters_per_epoch: int = None, seed: int = 0, shuffle: bool = False,
                 num_workers: int = 0, collate_fn=None, pin_memory: bool = False):
        self.sampler = batches if hasattr(batches, "generate") else RawSampler(batches)
        self.dataset = dataset
        self.num_iters_per_epoch = num_iters_per_epoch
        self.shuffle = shuffle
        self.seed = seed
        self.num_workers = num_workers
        self.collate_fn = collate_fn
        self.pin_memory = pin_memory

    def _epoch_batches(self, e, shuffle):
        b = self.sampler.generate(e + self.seed)
        if shuffle:
            np.random.RandomState(e + self.seed).shuffle(b)
        return b

    def batches_for_epoch(self, epoch: int, shuffle: bool = None):
        """The batch list of `epoch` (sequence_iter_factory.py:72-135)."""
        shuffle = self.shuffle if shuffle is None else shuffle
        n_iter = self.num_iters_per_epoch
        if n_iter is None:
            return self._epoch_batches(epoch, shuffle)
        N = len(self.sampler)
        if n_iter < N:
            real_epoch, offset = divmod(n_iter * epoch, N)
            if offset >= n_iter:
                return self._epoch_batches(real_epoch, shuffle)[offset - n_iter: offset]
            prev = self._epoch_batches(real_epoch - 1, shuffle)
            cur = self._epoch_batches(real_epoch, shuffle)
            return prev[offset - n_iter:] + cur[:offset]
        e, cursor = divmod(n_iter * (epoch - 1), N)
        remain = n_iter
        out = []
        cur = self._epoch_batches(e, shuffle)
        while remain > 0:
            part = cur[cursor: cursor + remain]
            out += part
            if cursor + remain >= N:
                e += 1
                cursor = 0
                cur = self._epoch_batches(e, shuffle)
            else:
                cursor = cursor + remain
            remain -= len(part)
        assert len(out) == n_iter
        return out

    def build_iter(self, epoch: int, shuffle: bool = None) -> DataLoader:
        batches = self.batches_for_epoch(epoch, shuffle)
        kwargs = dict(collate_fn=self.collate_fn) if self.collate_fn is not None else {}
        return DataLoader(dataset=self.dataset, batch_sampler=batches, num_workers=self.num_workers,
                          pin_memory=self.pin_memory, worker_init_fn=partial(worker_init_fn, base_seed=epoch + self.seed),
                          **kwargs)
