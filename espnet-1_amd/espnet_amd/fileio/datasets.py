"""Data readers of espnet2/train/dataset.py DATA_TYPES used with the ASR task's synthetic
and precomputed-feature corpora:

* ``rand_float`` — FloatRandomGenerateDataset (espnet2/fileio/rand_gen_dataset.py:11-45):
  `np.random.randn(*shape)` per utterance from a shape file ("uttA 123,83").
* ``rand_int_<low>_<high>`` — IntRandomGenerateDataset (:48-86): `np.random.randint(low, high)`.
* ``npy`` — NpyScpReader (espnet2/fileio/npy_scp.py): "uttA /path/a.npy", numpy.load with
  allow_pickle=False.
* ``text_int`` / ``text_float`` / ``csv_int`` / ``csv_float`` — load_num_sequence_text
  (espnet2/fileio/read_text.py:39-82).

Types that need third-party decoders or a tokenizer (sound, kaldi_ark, text with a
preprocessor, hdf5, ...) raise NotImplementedError naming the type.
"""
from __future__ import annotations

import collections.abc
import re
from typing import Dict, Tuple

import numpy as np

from ..samplers.num_elements_batch_sampler import load_num_sequence_text, read_2column_text


class FloatRandomGenerateDataset(collections.abc.Mapping):
    def __init__(self, shape_file, dtype="float32", loader_type: str = "csv_int"):
        self.utt2shape = load_num_sequence_text(shape_file, loader_type)
        self.dtype = np.dtype(dtype)

    def __iter__(self):
        return iter(self.utt2shape)

    def __len__(self):
        return len(self.utt2shape)

    def __getitem__(self, item) -> np.ndarray:
        return np.random.randn(*self.utt2shape[item]).astype(self.dtype)


class IntRandomGenerateDataset(collections.abc.Mapping):
    def __init__(self, shape_file, low: int, high: int = None, dtype="int64", loader_type: str = "csv_int"):
        self.utt2shape = load_num_sequence_text(shape_file, loader_type)
        self.dtype = np.dtype(dtype)
        self.low, self.high = low, high

    def __iter__(self):
        return iter(self.utt2shape)

    def __len__(self):
        return len(self.utt2shape)

    def __getitem__(self, item) -> np.ndarray:
        return np.random.randint(self.low, self.high, size=self.utt2shape[item], dtype=self.dtype)


class NpyScpReader(collections.abc.Mapping):
    def __init__(self, fname):
        self.data = read_2column_text(fname)

    def __getitem__(self, key) -> np.ndarray:
        return np.load(self.data[key], allow_pickle=False)

    def __iter__(self):
        return iter(self.data)

    def __len__(self):
        return len(self.data)


class _NumSequence(collections.abc.Mapping):
    def __init__(self, path, loader_type):
        self.data = load_num_sequence_text(path, loader_type)

    def __getitem__(self, key):
        return np.array(self.data[key])

    def __iter__(self):
        return iter(self.data)

    def __len__(self):
        return len(self.data)


def build_loader(path: str, loader_type: str):
    """dataset.py:_build_loader (:421-455) for the supported types."""
    if loader_type == "rand_float":
        return FloatRandomGenerateDataset(path)
    m = re.fullmatch(r"rand_int_(\d+)_(\d+)", loader_type)
    if m:  # dataset.py:rand_int_loader: low / high from the type name
        return IntRandomGenerateDataset(path, low=int(m.group(1)), high=int(m.group(2)))
    if loader_type == "npy":
        return NpyScpReader(path)
    if loader_type in ("text_int", "text_float", "csv_int", "csv_float"):
        return _NumSequence(path, loader_type)
    raise NotImplementedError(f"loader_type={loader_type} is outside the build's data path "
                              "(supported: rand_float, rand_int_<low>_<high>, npy, text_int, text_float, "
                              "csv_int, csv_float)")


class ESPnetDataset:
    """dataset.py:ESPnetDataset (:356-541): uid -> {name: ndarray}, float arrays cast to
    float_dtype and integer arrays to int64."""

    def __init__(self, path_name_type_list, preprocess=None, float_dtype: str = "float32",
                 int_dtype: str = "long", max_cache_size=0.0, max_cache_fd: int = 0):
        if len(path_name_type_list) == 0:
            raise ValueError('1 or more elements are required for "path_name_type_list"')
        self.preprocess = preprocess
        self.float_dtype = float_dtype
        self.int_dtype = "int64" if int_dtype == "long" else int_dtype
        self.loader_dict: Dict[str, collections.abc.Mapping] = {}
        self.debug_info: Dict[str, Tuple[str, str]] = {}
        for path, name, _type in path_name_type_list:
            if name in self.loader_dict:
                raise RuntimeError(f'"{name}" is duplicated for data-key')
            loader = build_loader(path, _type)
            if len(loader) == 0:
                raise RuntimeError(f"{path} has no samples")
            self.loader_dict[name] = loader
            self.debug_info[name] = (path, _type)

    def has_name(self, name) -> bool:
        return name in self.loader_dict

    def names(self) -> Tuple[str, ...]:
        return tuple(self.loader_dict)

    def __iter__(self):
        return iter(next(iter(self.loader_dict.values())))

    def __repr__(self):
        items = "".join(f'\n  {n}: {{"path": "{p}", "type": "{t}"}}' for n, (p, t) in self.debug_info.items())
        return f"{self.__class__.__name__}({items}\n  preprocess: {self.preprocess})"

    def __getitem__(self, uid):
        if isinstance(uid, int):
            uid = list(next(iter(self.loader_dict.values())))[uid]
        data = {}
        for name, loader in self.loader_dict.items():
            v = loader[uid]
            if isinstance(v, list):
                v = np.array(v)
            elif isinstance(v, (int, float)):
                v = np.array([v])
            data[name] = v
        if self.preprocess is not None:
            data = self.preprocess(uid, data)
        for name, v in data.items():
            if not isinstance(v, np.ndarray):
                raise RuntimeError(f"All values must be converted to np.ndarray object by preprocessing, "
                                   f'but "{name}" is still {type(v)}.')
            if v.dtype.kind == "f":
                data[name] = v.astype(self.float_dtype)
            elif v.dtype.kind == "i":
                data[name] = v.astype(self.int_dtype)
            else:
                raise NotImplementedError(f"Not supported dtype: {v.dtype}")
        return uid, data
