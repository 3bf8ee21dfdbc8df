"""CommonCollateFn — espnet2/train/collate_fn.py:11-40, 160-218: pad each key's arrays to
(B, Lmax, ...) with float_pad_value / int_pad_value (the ASR task uses 0.0 / -1,
tasks/asr.py:398) and add "<key>_lengths" (int64)."""
from __future__ import annotations

from typing import Collection, Dict, List, Tuple

import numpy as np
import torch


def common_collate_fn(data, float_pad_value=0.0, int_pad_value: int = -32768,
                      not_sequence: Collection[str] = ()) -> Tuple[List[str], Dict[str, torch.Tensor]]:
    uttids = [u for u, _ in data]
    data = [d for _, d in data]
    assert all(set(data[0]) == set(d) for d in data), "dict-keys mismatching"
    assert all(not k.endswith("_lengths") for k in data[0]), f"*_lengths is reserved: {list(data[0])}"
    out = {}
    for key in data[0]:
        arrays = [d[key] for d in data]
        pad = int_pad_value if arrays[0].dtype.kind == "i" else float_pad_value
        lmax = max(a.shape[0] for a in arrays)
        buf = np.full((len(arrays), lmax) + arrays[0].shape[1:], pad, dtype=arrays[0].dtype)
        for i, a in enumerate(arrays):
            buf[i, : a.shape[0]] = a
        out[key] = torch.from_numpy(buf)
        if key not in not_sequence:
            out[key + "_lengths"] = torch.tensor([a.shape[0] for a in arrays], dtype=torch.long)
    return uttids, out


class CommonCollateFn:
    def __init__(self, float_pad_value=0.0, int_pad_value: int = -32768, not_sequence: Collection[str] = ()):
        self.float_pad_value = float_pad_value
        self.int_pad_value = int_pad_value
        self.not_sequence = set(not_sequence)

    def __repr__(self):
        return (f"{self.__class__}(float_pad_value={self.float_pad_value}, "
                f"int_pad_value={self.float_pad_value})")

    def __call__(self, data):
        return common_collate_fn(data, float_pad_value=self.float_pad_value, int_pad_value=self.int_pad_value,
                                 not_sequence=self.not_sequence)
