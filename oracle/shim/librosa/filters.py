"""TEST INFRASTRUCTURE: restatement of librosa.filters.mel (librosa >= 0.8, the version
range setup.py pins; the package itself is absent from this image): Slaney (default) or HTK
mel scale, "slaney" area normalisation, float32 weights (n_mels, 1 + n_fft // 2).
PARITY UNPINNED against librosa itself (no librosa output is available here); the frontend
goldens pin everything downstream of the mel matrix to the reference's code path."""
import numpy as np


def _hz_to_mel(f, htk=False):
    f = np.asanyarray(f, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_mel = 1000.0 / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        t = f >= 1000.0
        mels[t] = min_log_mel + np.log(f[t] / 1000.0) / logstep
    elif f >= 1000.0:
        mels = min_log_mel + np.log(f / 1000.0) / logstep
    return mels


def _mel_to_hz(m, htk=False):
    m = np.asanyarray(m, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_mel = 1000.0 / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        t = m >= min_log_mel
        freqs[t] = 1000.0 * np.exp(logstep * (m[t] - min_log_mel))
    elif m >= min_log_mel:
        freqs = 1000.0 * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel(sr=22050, n_fft=2048, n_mels=128, fmin=0.0, fmax=None, htk=False, norm="slaney", dtype=np.float32):
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((int(n_mels), int(1 + n_fft // 2)), dtype=dtype)
    fftfreqs = np.linspace(0, float(sr) / 2, int(1 + n_fft // 2), endpoint=True)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin, htk), _hz_to_mel(fmax, htk), int(n_mels) + 2), htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(int(n_mels)):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    if norm == "slaney":
        enorm = 2.0 / (mel_f[2:int(n_mels) + 2] - mel_f[:int(n_mels)])
        weights *= enorm[:, np.newaxis]
    return weights
