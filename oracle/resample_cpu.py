"""ORACLE — test infrastructure only.  CPU restatement of the resampler of
`distilcodec_nabeel_amd/resample.py` (scipy.signal.resample_poly's polyphase form and default
filter), used by tests/ to check the GPU kernel.

Parity with the reference is UNPINNED for this row: the reference resamples with librosa's
soxr_hq (distil_codec.py:108-110, :676; meldataset.py:18-20), and neither librosa nor soxr is
installed here.  What is pinned: this restatement against scipy.signal.resample_poly
(tests/test_resample.py), and the GPU kernel against this restatement (tests/test_gpu_resample.py).
"""
from __future__ import annotations

from math import gcd

import numpy as np


def design(up: int, down: int):
    """resample_poly defaults (scipy/signal/_signaltools.py): firwin(2*half+1, 1/max_rate,
    window=('kaiser', 5.0)) * up, half = 10*max_rate, pre-padded to put outputs at the centre."""
    max_rate = max(up, down)
    f_c = 1.0 / max_rate
    half = 10 * max_rate
    taps = 2 * half + 1
    m = np.arange(taps) - half
    h = f_c * np.sinc(f_c * m) * np.kaiser(taps, 5.0)
    h = h / h.sum() * up
    pad = down - half % down
    return np.concatenate([np.zeros(pad), h]), (half + pad) // down


def resample(x: np.ndarray, sr_in: int, sr_out: int) -> np.ndarray:
    """Polyphase FIR along the last axis, fp64: y[i] = sum_m h[(i + pre) * down - up * m] x[m]."""
    g = gcd(sr_in, sr_out)
    up, down = sr_out // g, sr_in // g
    x = np.asarray(x, dtype=np.float64)
    if up == down:
        return x.copy()
    h, pre = design(up, down)
    return apply_poly(x, h, pre, up, down)


def apply_poly(x: np.ndarray, h: np.ndarray, pre: int, up: int, down: int) -> np.ndarray:
    """The polyphase form of dcx_resample_poly in fp64 for any prototype filter h."""
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[-1]
    no = -(-n * up // down)
    t = (np.arange(no) + pre) * down
    out = np.zeros(x.shape[:-1] + (no,))
    for k in range(len(h)):  # vectorised over outputs, one filter tap at a time
        num = t - k
        m = num // up
        ok = (num >= 0) & (num % up == 0) & (m < n)
        if ok.any():
            out[..., ok] += h[k] * x[..., m[ok]]
    return out


def torchaudio_resample(waveform, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                        rolloff: float = 0.99):
    """`torchaudio.functional.resample` with its defaults (resampling_method="sinc_interp_hann"),
    the resampler of LogMelSpectrogram.forward(sample_rate=...) (mel_spec.py:112-113; torchaudio
    2.4.1 pinned at requirements.txt:17).  Restated from torchaudio's published
    `_get_sinc_resample_kernel` / `_apply_sinc_resample_kernel`: the kernel is built in the input's
    dtype, the signal zero-padded by (width, width + orig) and convolved with stride orig, one output
    channel per phase.  torchaudio is not installed here, so parity is UNPINNED (no reference-held
    output exists); tests pin the GPU path to this restatement."""
    import math

    import torch

    x = torch.as_tensor(waveform)
    if orig_freq == new_freq:
        return x
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    dtype = x.dtype
    base_freq = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base_freq)
    idx = torch.arange(-width, width + orig, dtype=dtype)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=dtype)[:, None, None] / new + idx
    t *= base_freq
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base_freq / orig
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels *= window * scale
    shape = x.shape
    w = x.reshape(-1, shape[-1])
    n = w.shape[-1]
    w = torch.nn.functional.pad(w, (width, width + orig))
    y = torch.nn.functional.conv1d(w[:, None], kernels, stride=orig)
    y = y.transpose(1, 2).reshape(w.shape[0], -1)
    target = int(math.ceil(new * n / orig))
    return y[..., :target].reshape(shape[:-1] + (-1,))
