"""DefaultFrontend — drop-in for espnet2/asr/frontend/default.py:17-140 (Stft -> power ->
LogMel), plus GlobalMVN (espnet2/layers/global_mvn.py), on the device.

MI355X design: the STFT is a framing kernel (reflect padding + window, one row per frame)
and ONE exact-f32 MFMA GEMM against the real DFT basis [cos | -sin]; the power spectrum is a
pass over that output, the mel projection a second f32 GEMM, and log + padding masks one
elementwise pass (include/espnet_amd.h, ea_stft_frames ... ea_logmel_mvn).  The frontend has
no parameters and the reference runs it outside autocast, so it is forward-only and f32.

The mel matrix is librosa.filters.mel (setup.py pins librosa>=0.8.0; librosa is not in this
image): `mel_filterbank` restates its published algorithm (Slaney or HTK mel scale, "slaney"
area normalisation, float32 weights), with the reference's buffer name and layout
(LogMel.melmat = melmat.T, (n_fft//2+1, n_mels)).
"""
from __future__ import annotations

import copy
import math
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch
from torch import nn

from ... import hip_ops as ops
from ..._lib import lib
from ..abs_modules import AbsFrontend, AbsNormalize


# ----------------------------------------------------------------------------- librosa mel
def _hz_to_mel(f, htk):
    f = np.asanyarray(f, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        t = f >= min_log_hz
        mels[t] = min_log_mel + np.log(f[t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def _mel_to_hz(m, htk):
    m = np.asanyarray(m, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        t = m >= min_log_mel
        freqs[t] = min_log_hz * np.exp(logstep * (m[t] - min_log_mel))
    elif m >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel_filterbank(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk, norm="slaney", dtype=float32)."""
    if fmax is None:
        fmax = float(sr) / 2
    n_mels = int(n_mels)
    weights = np.zeros((n_mels, int(1 + n_fft // 2)), dtype=np.float32)
    fftfreqs = np.linspace(0, float(sr) / 2, int(1 + n_fft // 2), endpoint=True)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin, htk), _hz_to_mel(fmax, htk), n_mels + 2), htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


# ----------------------------------------------------------------------------- modules
class Stft(nn.Module):
    """layers/stft.py:22-115 (torch.stft path, single channel, onesided, not normalized)."""

    def __init__(self, n_fft: int = 512, win_length: int = None, hop_length: int = 128,
                 window: Optional[str] = "hann", center: bool = True, normalized: bool = False,
                 onesided: bool = True):
        super().__init__()
        if normalized or not onesided:
            raise NotImplementedError("Stft: normalized / two-sided spectra are not on the recipe path")
        self.n_fft = n_fft
        self.win_length = n_fft if win_length is None else win_length
        self.hop_length = hop_length
        self.center = center
        self.normalized = normalized
        self.onesided = onesided
        if window is not None and not hasattr(torch, f"{window}_window"):
            raise ValueError(f"{window} window is not implemented")
        self.window = window
        self._cache = {}

    def _consts(self, device):
        c = self._cache.get(device)
        if c is None:
            n, nb = self.n_fft, self.n_fft // 2 + 1
            if self.window is not None:
                w = getattr(torch, f"{self.window}_window")(self.win_length, dtype=torch.float32)
            else:
                w = torch.ones(self.win_length)
            left = (n - self.win_length) // 2  # torch.stft centres a shorter window
            win = torch.zeros(n)
            win[left:left + self.win_length] = w
            k = np.arange(n, dtype=np.float64)[:, None]
            j = np.arange(nb, dtype=np.float64)[None, :]
            ang = 2.0 * np.pi * ((k * j) % n) / n  # exact phase reduction before cos/sin
            basis = np.concatenate([np.cos(ang), -np.sin(ang)], axis=1).T.astype(np.float32)  # (2nb, n)
            c = (win.to(device), torch.from_numpy(np.ascontiguousarray(basis)).to(device))
            self._cache[device] = c
        return c

    def frames_lens(self, ilens):
        pad = self.n_fft // 2 if self.center else 0
        return (ilens + 2 * pad - self.n_fft) // self.hop_length + 1

    def power(self, x: torch.Tensor, ilens: torch.Tensor):
        """x (B, Ns) f32 -> power spectrum (B*nF, nbins) f32 (padded frames zero), nF, olens."""
        B, Ns = x.shape
        n, nb = self.n_fft, self.n_fft // 2 + 1
        pad = n // 2 if self.center else 0
        nF = (Ns + 2 * pad - n) // self.hop_length + 1
        win, basis = self._consts(x.device)
        olens = self.frames_lens(ilens)
        M = B * nF
        frames = torch.empty(M, n, device=x.device)
        lib.ea_stft_frames(B, Ns, nF, n, self.hop_length, int(self.center), x.data_ptr(), win.data_ptr(),
                           frames.data_ptr(), ops.stream())
        spec = torch.empty(M, 2 * nb, device=x.device)
        ops.linear(frames, basis, spec)
        pw = torch.empty(M, nb, device=x.device)
        lib.ea_power_spectrum(M, nF, nb, spec.data_ptr(), 2 * nb, olens.data_ptr(), pw.data_ptr(), nb, ops.stream())
        return pw, nF, olens


class LogMel(nn.Module):
    """layers/log_mel.py:9-84 (log_base None: natural log)."""

    def __init__(self, fs: int = 16000, n_fft: int = 512, n_mels: int = 80, fmin: float = None,
                 fmax: float = None, htk: bool = False, log_base: float = None):
        super().__init__()
        if log_base is not None:
            raise NotImplementedError("LogMel: only the natural log (log_base None, the default)")
        fmin = 0 if fmin is None else fmin
        fmax = fs / 2 if fmax is None else fmax
        self.mel_options = dict(sr=fs, n_fft=n_fft, n_mels=n_mels, fmin=fmin, fmax=fmax, htk=htk)
        self.log_base = log_base
        self.register_buffer("melmat", torch.from_numpy(mel_filterbank(**self.mel_options).T).float())


class DefaultFrontend(AbsFrontend):
    """frontend/default.py:17-140 with frontend_conf's WPE / beamformer off (their defaults)."""

    def __init__(self, fs: Union[int, str] = 16000, n_fft: int = 512, win_length: int = None,
                 hop_length: int = 128, window: Optional[str] = "hann", center: bool = True,
                 normalized: bool = False, onesided: bool = True, n_mels: int = 80, fmin: int = None,
                 fmax: int = None, htk: bool = False, frontend_conf: Optional[dict] = None,
                 apply_stft: bool = True):
        super().__init__()
        if isinstance(fs, str):
            fs = int(float(fs.lower().rstrip("k")) * (1000 if fs.lower().endswith("k") else 1))
        conf = copy.deepcopy(frontend_conf) or {}
        if conf.get("use_wpe") or conf.get("use_beamformer"):
            raise NotImplementedError("multi-channel enhancement (WPE / beamformer) is outside the path")
        if not apply_stft:
            raise NotImplementedError("apply_stft=False (precomputed complex input)")
        self.hop_length = hop_length
        self.stft = Stft(n_fft=n_fft, win_length=win_length, hop_length=hop_length, center=center,
                         window=window, normalized=normalized, onesided=onesided)
        self.apply_stft = apply_stft
        self.frontend = None
        self.logmel = LogMel(fs=fs, n_fft=n_fft, n_mels=n_mels, fmin=fmin, fmax=fmax, htk=htk)
        self.n_mels = n_mels
        self.frontend_type = "default"

    def output_size(self) -> int:
        return self.n_mels

    @torch.no_grad()
    def forward(self, input: torch.Tensor, input_lengths: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if input.dim() != 2:
            raise NotImplementedError("multi-channel input is outside the path")
        x = input.contiguous().float()
        B = x.shape[0]
        pw, nF, olens = self.stft.power(x, input_lengths.to(x.device, torch.long))
        nm = self.n_mels
        mel = torch.empty(B * nF, nm, device=x.device)
        melmat_t = self.logmel.melmat.t().contiguous()  # (n_mels, nbins): the GEMM's K-major B
        ops.linear(pw, melmat_t, mel)
        feats = torch.empty(B, nF, nm, device=x.device)
        lib.ea_logmel_mvn(B * nF, nF, nm, mel.data_ptr(), nm, olens.data_ptr(), None, None, feats.data_ptr(),
                          ops.stream())
        return feats, olens


class GlobalMVN(AbsNormalize):
    """layers/global_mvn.py:13-104: mean/std buffers from a stats file (.npy array or .npz
    with count/sum/sum_square), loaded with numpy's default allow_pickle=False."""

    def __init__(self, stats_file: Union[Path, str], norm_means: bool = True, norm_vars: bool = True,
                 eps: float = 1.0e-20):
        super().__init__()
        self.norm_means = norm_means
        self.norm_vars = norm_vars
        self.eps = eps
        self.stats_file = Path(stats_file)
        stats = np.load(self.stats_file)
        if isinstance(stats, np.ndarray):
            count = stats[0].flatten()[-1]
            mean = stats[0, :-1] / count
            var = stats[1, :-1] / count - mean * mean
        else:
            count = stats["count"]
            mean = stats["sum"] / count
            var = stats["sum_square"] / count - mean * mean
        std = np.sqrt(np.maximum(var, eps))
        mean = torch.from_numpy(mean) if isinstance(mean, np.ndarray) else torch.tensor(mean).float()
        std = torch.from_numpy(std) if isinstance(std, np.ndarray) else torch.tensor(std).float()
        self.register_buffer("mean", mean)
        self.register_buffer("std", std)

    def forward(self, x: torch.Tensor, ilens: torch.Tensor = None):
        B, T, D = x.shape
        if ilens is None:
            ilens = torch.full((B,), T, dtype=torch.long, device=x.device)
        lens = ilens.to(x.device, torch.long)
        mean = self.mean.to(x.device, torch.float32) if self.norm_means else None
        std = self.std.to(x.device, torch.float32) if self.norm_vars else None
        y = torch.empty_like(x)
        lib.ea_global_mvn(B, T, D, x.contiguous().data_ptr(), lens.data_ptr(), ops.ptr(mean), ops.ptr(std),
                          y.data_ptr(), ops.stream())
        return y, ilens
