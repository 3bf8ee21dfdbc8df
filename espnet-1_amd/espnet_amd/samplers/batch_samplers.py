"""The other mini-batch samplers of espnet2/samplers/ and build_batch_sampler
(build_batch_sampler.py:72-162; BATCH_TYPES unsorted / sorted / folded / numel / length).

Host logic: they only decide which utterances share a padded batch.  Each returns the
reference's batch list for the same shape files — including its corner cases (the
unsorted sampler slices by the total key count, a too-small last folded batch is spread
from the second-to-last batch backwards, a length batch from the last) — pinned by
tests/golden/sampler.npz.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Sequence, Tuple, Union

from .num_elements_batch_sampler import NumElementsBatchSampler, load_num_sequence_text, read_2column_text

BATCH_TYPES = dict(
    unsorted="UnsortedBatchSampler has nothing in particular feature and just creates mini-batches which has "
             "constant batch_size.",
    sorted="SortedBatchSampler sorts samples by the length of the first input and makes mini-batches which "
           "has constant batch_size.",
    folded="FoldedBatchSampler makes mini-batches whose batch sizes are shrunk by the lengths "
           "(batch_size / (1 + L // fold_length)).",
    length="LengthBatchSampler makes mini-batches of variable size whose summed lengths are below batch_bins.",
    numel="NumElementsBatchSampler makes mini-batches whose padded element count is below batch_bins.",
)


class _Sampler:
    batch_list: List[Tuple[str, ...]]

    def __len__(self):
        return len(self.batch_list)

    def __iter__(self) -> Iterator[Tuple[str, ...]]:
        return iter(self.batch_list)

    def generate(self, seed):
        """AbsSampler.generate (abs_sampler.py:17-18): the batches (seed unused)."""
        return list(self.batch_list)


def _check_orders(sort_in_batch, sort_batch):
    if sort_batch not in ("ascending", "descending"):
        raise ValueError(f"sort_batch must be ascending or descending: {sort_batch}")
    if sort_in_batch not in ("ascending", "descending"):
        raise ValueError(f"sort_in_batch must be ascending or descending: {sort_in_batch}")


def _categories(keys, utt2category_file, ref_keys, what):
    """{category: keys in `keys` order}; one default category without a category file."""
    if utt2category_file is None:
        return {"default_category": list(keys)}
    utt2cat = read_2column_text(utt2category_file)
    if set(utt2cat) != set(ref_keys):
        raise RuntimeError(f"keys are mismatched between {utt2category_file} != {what}")
    out: Dict[str, List[str]] = {}
    for k in keys:
        out.setdefault(utt2cat[k], []).append(k)
    return out


def _load_shapes(shape_files):
    shapes = [load_num_sequence_text(s, loader_type="csv_int") for s in shape_files]
    for s, d in zip(shape_files, shapes):
        if set(d) != set(shapes[0]):
            raise RuntimeError(f"keys are mismatched between {s} != {shape_files[0]}")
    return shapes


def _cut(keys: Sequence[str], sizes: Sequence[int], descending: bool) -> List[Tuple[str, ...]]:
    out, pos = [], 0
    for bs in sizes:
        mb = list(keys[pos:pos + bs])
        pos += bs
        out.append(tuple(mb[::-1] if descending else mb))
    return out


class UnsortedBatchSampler(_Sampler):
    """unsorted_batch_sampler.py:10-88: key-file order, constant batch size."""

    def __init__(self, batch_size: int, key_file: str, drop_last: bool = False, utt2category_file: str = None):
        assert batch_size > 0
        self.batch_size, self.key_file, self.drop_last = batch_size, key_file, drop_last
        keys = list(read_2column_text(key_file))
        if len(keys) == 0:
            raise RuntimeError(f"0 lines found: {key_file}")
        self.batch_list = []
        for ckeys in _categories(keys, utt2category_file, keys, key_file).values():
            n = max(len(ckeys) // batch_size, 1)
            if drop_last:
                self.batch_list += [tuple(ckeys[i * batch_size:(i + 1) * batch_size]) for i in range(n)]
            else:
                # the reference slices each category by the TOTAL key count
                total = len(keys)
                self.batch_list += [ckeys[i * total // n:(i + 1) * total // n] for i in range(n)]

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, "
                f"key_file={self.key_file}, ")


class SortedBatchSampler(_Sampler):
    """sorted_batch_sampler.py:10-95: sorted by the first shape dimension, constant batch size."""

    def __init__(self, batch_size: int, shape_file: str, sort_in_batch: str = "descending",
                 sort_batch: str = "ascending", drop_last: bool = False):
        assert batch_size > 0
        self.batch_size, self.shape_file = batch_size, shape_file
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        shape = load_num_sequence_text(shape_file, loader_type="csv_int")
        if sort_in_batch == "descending":
            keys = sorted(shape, key=lambda k: -shape[k][0])
        elif sort_in_batch == "ascending":
            keys = sorted(shape, key=lambda k: shape[k][0])
        else:
            raise ValueError(f"sort_in_batch must be either one of ascending, descending, or None: {sort_in_batch}")
        if len(keys) == 0:
            raise RuntimeError(f"0 lines found: {shape_file}")
        n = max(len(keys) // batch_size, 1)
        if drop_last:
            self.batch_list = [tuple(keys[i * batch_size:(i + 1) * batch_size]) for i in range(n)]
        else:
            self.batch_list = [keys[i * len(keys) // n:(i + 1) * len(keys) // n] for i in range(n)]
        if sort_in_batch != sort_batch:
            if sort_batch not in ("ascending", "descending"):
                raise ValueError(f"sort_batch must be ascending or descending: {sort_batch}")
            self.batch_list.reverse()
        if len(self.batch_list) == 0:
            raise RuntimeError("0 batches")

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, "
                f"shape_file={self.shape_file}, sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


class FoldedBatchSampler(_Sampler):
    """folded_batch_sampler.py:12-156: batch size shrinks with length,
    max(min_batch_size, batch_size // (1 + max_i L_i // fold_length_i)) at each batch's
    shortest utterance (keys ascend)."""

    def __init__(self, batch_size: int, shape_files: Union[Tuple[str, ...], List[str]], fold_lengths: Sequence[int],
                 min_batch_size: int = 1, sort_in_batch: str = "descending", sort_batch: str = "ascending",
                 drop_last: bool = False, utt2category_file: str = None):
        assert batch_size > 0
        _check_orders(sort_in_batch, sort_batch)
        self.batch_size, self.shape_files = batch_size, shape_files
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        shapes = _load_shapes(shape_files)
        first = shapes[0]
        keys = sorted(first, key=lambda k: first[k][0])
        if len(keys) == 0:
            raise RuntimeError(f"0 lines found: {shape_files[0]}")
        self.batch_list = []
        for ckeys in _categories(keys, utt2category_file, first, shape_files[0]).values():
            sizes, start = [], 0
            while True:
                k = ckeys[start]
                factor = max(int(d[k][0] / m) for d, m in zip(shapes, fold_lengths))
                bs = max(min_batch_size, int(batch_size / (1 + factor)))
                if drop_last and start + bs > len(ckeys) and len(self.batch_list) > 0:
                    break
                bs = min(len(ckeys) - start, bs)
                sizes.append(bs)
                start += bs
                if start >= len(ckeys):
                    break
            if len(sizes) == 0:
                raise RuntimeError("0 batches")
            if len(sizes) > 1 and sizes[-1] < min_batch_size:
                for i in range(sizes.pop(-1)):
                    sizes[-(i % len(sizes)) - 2] += 1
            if not drop_last:
                assert sum(sizes) == len(ckeys), f"{sum(sizes)} != {len(ckeys)}"
            batches = _cut(ckeys, sizes, sort_in_batch == "descending")
            if sort_batch == "descending":
                batches.reverse()
            self.batch_list += batches

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_size={self.batch_size}, "
                f"shape_files={self.shape_files}, sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


class LengthBatchSampler(_Sampler):
    """length_batch_sampler.py:12-146: variable batch size, sum of lengths (x batch size
    with padding) just above batch_bins."""

    def __init__(self, batch_bins: int, shape_files: Union[Tuple[str, ...], List[str]], min_batch_size: int = 1,
                 sort_in_batch: str = "descending", sort_batch: str = "ascending", drop_last: bool = False,
                 padding: bool = True):
        assert batch_bins > 0
        _check_orders(sort_in_batch, sort_batch)
        self.batch_bins, self.shape_files = batch_bins, shape_files
        self.sort_in_batch, self.sort_batch, self.drop_last = sort_in_batch, sort_batch, drop_last
        shapes = _load_shapes(shape_files)
        first = shapes[0]
        keys = sorted(first, key=lambda k: first[k][0])
        if len(keys) == 0:
            raise RuntimeError(f"0 lines found: {shape_files[0]}")
        sizes, cur = [], []
        for key in keys:
            cur.append(key)
            if padding:
                bins = sum(len(cur) * sh[key][0] for sh in shapes)
            else:
                bins = sum(d[k][0] for k in cur for d in shapes)
            if bins > batch_bins and len(cur) >= min_batch_size:
                sizes.append(len(cur))
                cur = []
        if cur and (not drop_last or len(sizes) == 0):
            sizes.append(len(cur))
        if len(sizes) == 0:
            raise RuntimeError("0 batches")
        if len(sizes) > 1 and sizes[-1] < min_batch_size:
            for i in range(sizes.pop(-1)):
                sizes[-(i % len(sizes)) - 1] += 1
        if not drop_last:
            assert sum(sizes) == len(keys), f"{sum(sizes)} != {len(keys)}"
        self.batch_list = [b for b in _cut(keys, sizes, sort_in_batch == "descending")]
        if sort_batch == "descending":
            self.batch_list.reverse()

    def __repr__(self):
        return (f"{self.__class__.__name__}(N-batch={len(self)}, batch_bins={self.batch_bins}, "
                f"sort_in_batch={self.sort_in_batch}, sort_batch={self.sort_batch})")


NumElementsBatchSampler.generate = _Sampler.generate


def build_batch_sampler(type: str, batch_size: int, batch_bins: int, shape_files: Union[Tuple[str, ...], List[str]],
                        sort_in_batch: str = "descending", sort_batch: str = "ascending", drop_last: bool = False,
                        min_batch_size: int = 1, fold_lengths: Sequence[int] = (), padding: bool = True,
                        utt2category_file: str = None):
    """build_batch_sampler.py:72-162."""
    if len(shape_files) == 0:
        raise ValueError("No shape file are given")
    if type == "unsorted":
        return UnsortedBatchSampler(batch_size=batch_size, key_file=shape_files[0], drop_last=drop_last)
    if type == "sorted":
        return SortedBatchSampler(batch_size=batch_size, shape_file=shape_files[0], sort_in_batch=sort_in_batch,
                                  sort_batch=sort_batch, drop_last=drop_last)
    if type == "folded":
        if len(fold_lengths) != len(shape_files):
            raise ValueError(f"The number of fold_lengths must be equal to the number of shape_files: "
                             f"{len(fold_lengths)} != {len(shape_files)}")
        return FoldedBatchSampler(batch_size=batch_size, shape_files=shape_files, fold_lengths=fold_lengths,
                                  sort_in_batch=sort_in_batch, sort_batch=sort_batch, drop_last=drop_last,
                                  min_batch_size=min_batch_size, utt2category_file=utt2category_file)
    if type == "numel":
        return NumElementsBatchSampler(batch_bins=batch_bins, shape_files=shape_files, sort_in_batch=sort_in_batch,
                                       sort_batch=sort_batch, drop_last=drop_last, padding=padding,
                                       min_batch_size=min_batch_size)
    if type == "length":
        return LengthBatchSampler(batch_bins=batch_bins, shape_files=shape_files, sort_in_batch=sort_in_batch,
                                  sort_batch=sort_batch, drop_last=drop_last, padding=padding,
                                  min_batch_size=min_batch_size)
    raise ValueError(f"Not supported: {type}")
