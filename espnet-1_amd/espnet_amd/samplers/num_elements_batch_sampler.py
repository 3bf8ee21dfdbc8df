"""NumElementsBatchSampler — drop-in for espnet2/samplers/num_elements_batch_sampler.py:10-157
(the C5 `batch_type: numel` sampler): utterances sorted by length, cut into mini-batches
whose padded element count (batch size x longest length x feature dims, summed over the
shape files) just exceeds `batch_bins`, redistributing a short last batch.

Host logic only (it decides which utterances share a padded batch; the device never sees
it).  Same constructor, same errors, same batch list as the reference for the same shape
files — pinned by tests/golden/sampler.npz (oracle/make_goldens.py).
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Sequence, Tuple, Union

import numpy as np


def read_2column_text(path) -> Dict[str, str]:
    """espnet2/fileio/read_text.py:11-36: `key value` lines (value may contain spaces)."""
    data = {}
    with open(path, encoding="utf-8") as f:
        for linenum, line in enumerate(f, 1):
            sps = line.rstrip().split(maxsplit=1)
            if len(sps) == 1:
                k, v = sps[0], ""
            else:
                k, v = sps
            if k in data:
                raise RuntimeError(f"{k} is duplicated ({path}:{linenum})")
            data[k] = v
    return data


def load_num_sequence_text(path, loader_type: str = "csv_int") -> Dict[str, List[Union[int, float]]]:
    """espnet2/fileio/read_text.py:39-82."""
    kinds = {"text_int": (" ", int), "text_float": (" ", float), "csv_int": (",", int),
             "csv_float": (",", float)}
    if loader_type not in kinds:
        raise ValueError(f"Not supported loader_type={loader_type}")
    delim, dtype = kinds[loader_type]
    return {k: [dtype(i) for i in v.split(delim)] for k, v in read_2column_text(path).items()}


class NumElementsBatchSampler:
    def __init__(self, batch_bins: int, shape_files: Union[Tuple[str, ...], List[str]] = (),
                 min_batch_size: int = 1, sort_in_batch: str = "descending",
                 sort_batch: str = "ascending", drop_last: bool = False, padding: bool = True,
                 utt2shapes: Sequence[Dict[str, Sequence[int]]] = None):
        """`utt2shapes` (one {utt: shape} dict per shape file, in file order) may replace
        `shape_files` for in-memory corpora (the benchmark's synthetic one)."""
        assert batch_bins > 0
        if sort_batch not in ("ascending", "descending"):
            raise ValueError(f"sort_batch must be ascending or descending: {sort_batch}")
        if sort_in_batch not in ("ascending", "descending"):
            raise ValueError(f"sort_in_batch must be ascending or descending: {sort_in_batch}")
        self.batch_bins = batch_bins
        self.shape_files = shape_files
        self.sort_in_batch = sort_in_batch
        self.sort_batch = sort_batch
        self.drop_last = drop_last
        if utt2shapes is None:
            utt2shapes = [load_num_sequence_text(s, loader_type="csv_int") for s in shape_files]
            names = list(shape_files)
        else:
            utt2shapes = [dict(d) for d in utt2shapes]
            names = [f"<shapes {i}>" for i in range(len(utt2shapes))]
        first = utt2shapes[0]
        for s, d in zip(names, utt2shapes):
            if set(d) != set(first):
                raise RuntimeError(f"keys are mismatched between {s} != {names[0]}")
        # ascending by length; sorted() is stable, so ties keep the file order
        keys = sorted(first, key=lambda k: first[k][0])
        if len(keys) == 0:
            raise RuntimeError(f"0 lines found: {names[0]}")
        feat_dims = [np.prod(d[keys[0]][1:]) for d in utt2shapes] if padding else None

        batch_sizes = []
        current = []
        for key in keys:
            current.append(key)
            if padding:
                for d, s in zip(utt2shapes, names):
                    if tuple(d[key][1:]) != tuple(d[keys[0]][1:]):
                        raise RuntimeError(f"If padding=True, the feature dimension must be unified: {s}")
                # keys ascend, so the newest key is the batch's longest
                bins = sum(len(current) * sh[key][0] * fd for sh, fd in zip(utt2shapes, feat_dims))
            else:
                bins = sum(np.prod(d[k]) for k in current for d in utt2shapes)
            if bins > batch_bins and len(current) >= min_batch_size:
                batch_sizes.append(len(current))
                current = []
        if current and (not self.drop_last or len(batch_sizes) == 0):
            batch_sizes.append(len(current))
        if len(batch_sizes) == 0:
            raise RuntimeError("0 batches")
        # a too-small last batch is spread over the others, from the back
        if len(batch_sizes) > 1 and batch_sizes[-1] < min_batch_size:
            for i in range(batch_sizes.pop(-1)):
                batch_sizes[-(i % len(batch_sizes)) - 1] += 1
        if not self.drop_last:
            assert sum(batch_sizes) == len(keys), f"{sum(batch_sizes)} != {len(keys)}"

        self.batch_list = []
        pos = 0
        for bs in batch_sizes:
            mb = keys[pos:pos + bs]
            pos += bs
            if len(mb) < bs:  # drop_last with a trailing remainder
                break
            if sort_in_batch == "descending":
                mb = mb[::-1]
            self.batch_list.append(tuple(mb))
        if sort_batch == "descending":
            self.batch_list.reverse()

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_bins={self.batch_bins}, "
                f"sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")

    def __len__(self):
        return len(self.batch_list)

    def __iter__(self) -> Iterator[Tuple[str, ...]]:
        return iter(self.batch_list)
