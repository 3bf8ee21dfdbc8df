"""SpecAug — drop-in for espnet2/asr/specaug/specaug.py:9-102 (TimeWarp + MaskAlongAxis +
MaskAlongAxisVariableMaxWidth), applied on the device by ONE kernel (ea_specaug).

The reference draws its random parameters with torch.randint (time_warp.py:28-29 on the CPU
generator; mask_along_axis.py:33-43 on the features' device) and then runs an
interpolate / masked_fill per op (and a per-utterance Python loop when lengths differ,
time_warp.py:76-86).  Here the same torch.randint calls are made on the host CPU generator,
in the reference's order and with the reference's arguments — so under one torch seed the
warp points and mask spans are exactly the reference CPU path's — and the whole
augmentation of a batch is one fused launch over the features in HBM.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Union

import torch
from torch import nn

from .. import hip_ops as ops
from .._lib import lib
from .abs_modules import AbsSpecAug


def _width_range(r, name):
    if isinstance(r, (int, float)):
        r = (0, r)
    if len(r) != 2:
        raise TypeError(f"{name} must be a tuple of two values: {r}")
    assert r[1] > r[0]
    return tuple(r)


def _dim(dim):
    if isinstance(dim, str):
        if dim == "time":
            return 1
        if dim == "freq":
            return 2
        raise ValueError("dim must be int, 'time' or 'freq'")
    return dim


class TimeWarp(nn.Module):
    """layers/time_warp.py:49-88: parameters only; applied inside SpecAug's kernel."""

    def __init__(self, window: int = 80, mode: str = "bicubic"):
        super().__init__()
        if mode != "bicubic":
            raise NotImplementedError("time_warp_mode: only bicubic (the reference default) is on the path")
        self.window = window
        self.mode = mode

    def draw_one(self, t: int):
        """time_warp.py:24-29 for an axis of t frames -> (center, warped) or (0, 0)."""
        w = self.window
        if t - w <= w:
            return 0, 0
        center = int(torch.randint(w, t - w, (1,))[0])
        warped = int(torch.randint(center - w, center + w, (1,))[0]) + 1
        return center, warped

    def draw(self, B: int, T: int, lens):
        """time_warp.py:65-88: one warp for the batch when all lengths are equal, else one
        per utterance over its own length (drawn in batch order)."""
        if lens is None or all(le == lens[0] for le in lens):
            c, w = self.draw_one(T)
            return [(c, w)] * B, 0
        return [self.draw_one(int(le)) for le in lens], 1


class MaskAlongAxis(nn.Module):
    """layers/mask_along_axis.py:71-129 (replace_with_zero=True)."""

    def __init__(self, mask_width_range: Union[int, Sequence[int]] = (0, 30), num_mask: int = 2,
                 dim: Union[int, str] = "time", replace_with_zero: bool = True):
        super().__init__()
        if not replace_with_zero:
            raise NotImplementedError("replace_with_zero=False (mean fill) is not on the recipe path")
        self.mask_width_range = _width_range(mask_width_range, "mask_width_range")
        self.num_mask = num_mask
        self.dim = _dim(dim)
        self.replace_with_zero = replace_with_zero

    def draw(self, B: int, D: int):
        return _draw_spans(B, D, self.mask_width_range, self.num_mask)


class MaskAlongAxisVariableMaxWidth(nn.Module):
    """layers/mask_along_axis.py:132-204: widths in [floor(r0*D), floor(r1*D))."""

    def __init__(self, mask_width_ratio_range: Union[float, Sequence[float]] = (0.0, 0.05),
                 num_mask: int = 2, dim: Union[int, str] = "time", replace_with_zero: bool = True):
        super().__init__()
        if not replace_with_zero:
            raise NotImplementedError("replace_with_zero=False (mean fill) is not on the recipe path")
        self.mask_width_ratio_range = _width_range(mask_width_ratio_range, "mask_width_ratio_range")
        self.num_mask = num_mask
        self.dim = _dim(dim)
        self.replace_with_zero = replace_with_zero

    def draw(self, B: int, D: int):
        lo = max(0, math.floor(D * self.mask_width_ratio_range[0]))
        hi = min(D, math.floor(D * self.mask_width_ratio_range[1]))
        if hi > lo:
            return _draw_spans(B, D, (lo, hi), self.num_mask)
        return None


def _draw_spans(B, D, width_range, num_mask):
    """mask_along_axis.py:33-43 -> (B, num_mask, 2) int32 (position, width)."""
    length = torch.randint(width_range[0], width_range[1], (B, num_mask))
    pos = torch.randint(0, max(1, D - int(length.max())), (B, num_mask))
    return torch.stack([pos, length], dim=-1).to(torch.int32)


class SpecAug(AbsSpecAug):
    """specaug.py:9-102 with the same constructor arguments and ValueErrors."""

    def __init__(self, apply_time_warp: bool = True, time_warp_window: int = 5,
                 time_warp_mode: str = "bicubic", apply_freq_mask: bool = True,
                 freq_mask_width_range: Union[int, Sequence[int]] = (0, 20), num_freq_mask: int = 2,
                 apply_time_mask: bool = True,
                 time_mask_width_range: Optional[Union[int, Sequence[int]]] = None,
                 time_mask_width_ratio_range: Optional[Union[float, Sequence[float]]] = None,
                 num_time_mask: int = 2):
        if not apply_time_warp and not apply_time_mask and not apply_freq_mask:
            raise ValueError("Either one of time_warp, time_mask, or freq_mask should be applied")
        if apply_time_mask and time_mask_width_range is not None and time_mask_width_ratio_range is not None:
            raise ValueError('Either one of "time_mask_width_range" or "time_mask_width_ratio_range" can be used')
        super().__init__()
        self.apply_time_warp = apply_time_warp
        self.apply_freq_mask = apply_freq_mask
        self.apply_time_mask = apply_time_mask
        self.time_warp = TimeWarp(window=time_warp_window, mode=time_warp_mode) if apply_time_warp else None
        self.freq_mask = (MaskAlongAxis(dim="freq", mask_width_range=freq_mask_width_range,
                                        num_mask=num_freq_mask) if apply_freq_mask else None)
        if apply_time_mask:
            if time_mask_width_range is not None:
                self.time_mask = MaskAlongAxis(dim="time", mask_width_range=time_mask_width_range,
                                               num_mask=num_time_mask)
            elif time_mask_width_ratio_range is not None:
                self.time_mask = MaskAlongAxisVariableMaxWidth(
                    dim="time", mask_width_ratio_range=time_mask_width_ratio_range, num_mask=num_time_mask)
            else:
                raise ValueError('Either one of "time_mask_width_range" or '
                                 '"time_mask_width_ratio_range" should be used.')
        else:
            self.time_mask = None

    def draw(self, B: int, T: int, F: int, lens):
        """All of one forward's random parameters, in the reference's call order
        (specaug.py:95-101).  lens: host list of ints or None."""
        if self.time_warp is not None:
            warp, per_utt = self.time_warp.draw(B, T, lens)
        else:
            warp, per_utt = [(0, 0)] * B, 0
        fm = self.freq_mask.draw(B, F) if self.freq_mask is not None else None
        tm = self.time_mask.draw(B, T) if self.time_mask is not None else None
        return (torch.tensor(warp, dtype=torch.int32).reshape(B, 2), per_utt, fm, tm)

    # ------------------------------------------------------------------ captured steps
    def predraw(self, B: int, T: int, F: int, lens_host, device):
        """Draw this step's parameters now (host RNG, the reference's order) into a static
        device buffer for the shape (B, T, F): a hipGraph-captured step then reads them
        from there on every replay (train/graph.py), so SpecAug steps capture.  The next
        forward of that shape uses the buffer instead of drawing."""
        warp, per_utt, fm, tm = self.draw(B, T, F, lens_host)
        nf = 0 if fm is None else fm.shape[1]
        nt = 0 if tm is None else tm.shape[1]
        # the per-utterance warp over each utterance's own length equals the batch warp when
        # all lengths equal T (time_warp.py:73-86), so a captured kernel always runs per-utterance
        host = torch.cat([warp.reshape(-1)] + [a.reshape(-1) for a in (fm, tm) if a is not None]).pin_memory()
        key = (B, T, F)
        static = getattr(self, "_static", None)
        if static is None:
            static = self._static = {}
        buf = static.get(key)
        if buf is None or buf[0].numel() != host.numel():
            buf = static[key] = (torch.empty(host.numel(), dtype=torch.int32, device=device), nf, nt)
        buf[0].copy_(host, non_blocking=True)
        self._pending = key

    def forward(self, x: torch.Tensor, x_lengths: torch.Tensor = None, lens_host=None):
        """x (B, T, F) f32 on the device -> (augmented copy, x_lengths).  `lens_host` (list of
        ints) spares the device->host read of x_lengths that the equal-length test needs."""
        B, T, F = x.shape
        dev = x.device
        pending = getattr(self, "_pending", None)
        if pending == (B, T, F):
            self._pending = None
            params, nf, nt = self._static[pending]
            per_utt = 1
        else:
            if lens_host is None and x_lengths is not None:
                lens_host = [int(v) for v in x_lengths.tolist()]
            warp, per_utt, fm, tm = self.draw(B, T, F, lens_host)
            nf = 0 if fm is None else fm.shape[1]
            nt = 0 if tm is None else tm.shape[1]
            params = torch.cat([warp.reshape(-1)] + [a.reshape(-1) for a in (fm, tm) if a is not None])
            params = params.pin_memory().to(dev, non_blocking=True) if x.is_cuda else params
        warp_d = params[: 2 * B]
        fm_d = params[2 * B: 2 * B + 2 * B * nf]
        tm_d = params[2 * B + 2 * B * nf:]
        if per_utt and x_lengths is None:
            raise ValueError("per-utterance warp needs x_lengths")
        lens_d = None
        if x_lengths is not None:
            lens_d = x_lengths.to(dev, torch.long) if x_lengths.device != dev else x_lengths.long()
        x = x.contiguous()
        y = torch.empty_like(x)
        lib.ea_specaug(B, T, F, x.data_ptr(), ops.ptr(lens_d), warp_d.data_ptr(), per_utt,
                       fm_d.data_ptr() if nf else None, nf, tm_d.data_ptr() if nt else None, nt,
                       y.data_ptr(), ops.stream())
        return y, x_lengths
