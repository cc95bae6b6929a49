"""Sample-rate conversion for input audio that is not at the model rate (24 kHz).

Two filters run on the same GPU polyphase kernel (`dcx_resample_poly`):
* `resample`: file / raw-audio inputs (librosa's role in the reference), described below;
* `resample_sinc_hann`: torchaudio's default `F.resample`, which the reference's
  `LogMelSpectrogram.forward(sample_rate=...)` calls (mel_spec.py:112-113).

The reference resamples with `librosa.resample(..., res_type='soxr_hq')` (distil_codec.py:108-110,
:676) and `librosa.load(path, sr=...)` (meldataset.py:18-20).  librosa / soxr are not available
here, so this module implements the polyphase FIR resampler of `scipy.signal.resample_poly` with
its default filter (Kaiser-windowed sinc, beta 5, half length 10 * max(up, down), cutoff at the
lower Nyquist rate) and runs it on the GPU (`dcx_resample_poly`, csrc/dcx_misc.hip).  Output
length = ceil(n * up / down), as librosa's.  The result differs from soxr_hq's filter (a
deliberate difference); it matches scipy's resample_poly to fp32 rounding
(tests/test_gpu_resample.py).
"""
from __future__ import annotations

import ctypes
from functools import lru_cache
from math import gcd

import numpy as np
import torch

from . import _native


def ratio(sr_in: int, sr_out: int) -> tuple[int, int]:
    """(up, down) in lowest terms."""
    if sr_in <= 0 or sr_out <= 0:
        raise ValueError(f"sample rates must be positive, got {sr_in} -> {sr_out}")
    g = gcd(int(sr_in), int(sr_out))
    return int(sr_out) // g, int(sr_in) // g


def n_out(n_in: int, up: int, down: int) -> int:
    return -(-n_in * up // down)


@lru_cache(maxsize=32)
def design(up: int, down: int) -> tuple[np.ndarray, int]:
    """Filter (fp64, pre-padded, gain `up`) and the output offset `pre` of resample_poly's
    default design: firwin(2 * half + 1, 1 / max(up, down), window=('kaiser', 5.0)) * up with
    half = 10 * max(up, down); the filter is shifted by down - half % down zeros so that output
    sample i sits at the filter centre, and the first (half + pad) // down outputs are dropped."""
    max_rate = max(up, down)
    f_c = 1.0 / max_rate
    half = 10 * max_rate
    taps = 2 * half + 1
    m = np.arange(taps, dtype=np.float64) - half
    h = f_c * np.sinc(f_c * m) * np.kaiser(taps, 5.0)
    h = h / h.sum() * up  # unit gain at DC (firwin scale=True), times the zero-stuffing factor
    pad = down - half % down
    h = np.concatenate([np.zeros(pad), h])
    return np.ascontiguousarray(h), (half + pad) // down


_filters: dict = {}


def _device_filter(up: int, down: int, device: torch.device, kind: str = "poly", rates=None) -> tuple[torch.Tensor, int]:
    key = (kind, up, down, device.index)
    if key not in _filters:
        h, pre = design(up, down) if kind == "poly" else design_sinc_hann(*rates)
        _filters[key] = (torch.from_numpy(h).to(device), pre)
    return _filters[key]


@lru_cache(maxsize=32)
def design_sinc_hann(sr_in: int, sr_out: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """torchaudio.functional.resample's default kernel (`_get_sinc_resample_kernel`,
    sinc_interp_hann) as one prototype filter for `dcx_resample_poly` (up = new, down = orig in
    lowest terms).  torchaudio weights input m for output i by
        f(t) = sinc(t) * cos^2(pi t / (2 w)) * base / orig,  t = clamp(base (m new - i orig) / (orig new), -w, w)
    with base = rolloff * min(orig, new), w = lowpass_filter_width.  The kernel reads
    h[(i + pre) down - up m], so h[n] = f at (m new - i orig) = pre * orig - n; every tap with
    |t| < w is inside h (outside, torchaudio's clamped taps are below 1e-20).  fp64 taps."""
    up, down = ratio(sr_in, sr_out)
    new, orig = up, down
    base = min(orig, new) * rolloff
    half = int(np.ceil(lowpass_filter_width * orig * new / base))
    pre = -(-half // orig)
    c = pre * orig
    n = np.arange(2 * c + 1, dtype=np.float64)
    t = np.clip(base * (c - n) / (orig * new), -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * np.pi / lowpass_filter_width / 2) ** 2
    tp = t * np.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(tp == 0, 1.0, np.sin(tp) / np.where(tp == 0, 1.0, tp))
    return np.ascontiguousarray(k * window * (base / orig)), pre


def resample_sinc_hann(x, sr_in: int, sr_out: int, device="cuda") -> torch.Tensor:
    """torchaudio.functional.resample(x, sr_in, sr_out) with its defaults, on the GPU, along the last
    axis; output length ceil(n * sr_out / sr_in) like torchaudio's."""
    return _run(x, sr_in, sr_out, device, lambda up, down, dev: _device_filter(up, down, dev, "sinc_hann", (sr_in, sr_out)))


def resample(x, sr_in: int, sr_out: int, device="cuda") -> torch.Tensor:
    """Resample along the last axis.  `x`: (n,) or (rows, n) array / tensor; returns a float32
    tensor on `device` with the last axis ceil(n * sr_out / sr_in) long (a copy when the rates match)."""
    return _run(x, sr_in, sr_out, device, lambda up, down, dev: _device_filter(up, down, dev))


def _run(x, sr_in: int, sr_out: int, device, filt) -> torch.Tensor:
    dev = torch.device(device)
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise _native.NativeUnavailable("resampling runs on the GPU (dcx_resample_poly); no GPU device")
    if dev.index is None:  # normalise "cuda" to the indexed current device (filter cache, launch guard)
        dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.as_tensor(x, dtype=torch.float32).to(dev).contiguous()
    if sr_in == sr_out:
        return t.clone()
    up, down = ratio(sr_in, sr_out)
    shape = t.shape
    rows = t.reshape(-1, shape[-1]) if t.ndim > 1 else t.reshape(1, -1)
    n = rows.shape[-1]
    if n == 0:
        return torch.empty(*shape[:-1], 0, device=dev)
    no = n_out(n, up, down)
    h, pre = filt(up, down, dev)
    out = torch.empty(rows.shape[0], no, device=dev)
    L = _native.lib()
    with torch.cuda.device(dev):  # the kernel launches on the current device: make it `dev`
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for r0 in range(0, rows.shape[0], 65535):
            r1 = min(rows.shape[0], r0 + 65535)
            rc = L.dcx_resample_poly(ctypes.c_void_p(rows[r0].data_ptr()), r1 - r0, n, n, ctypes.c_void_p(h.data_ptr()),
                                     h.numel(), up, down, pre, ctypes.c_void_p(out[r0].data_ptr()), no, no, stream)
            if rc != _native.DCX_OK:
                raise _native.NativeError(rc, "dcx_resample_poly failed")
    return out.reshape(*shape[:-1], no)
