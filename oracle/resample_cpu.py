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
