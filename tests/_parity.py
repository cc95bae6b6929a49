"""Shared parity checks of the GPU path against the reference's outputs (fixtures or the oracle).

Waveform parity is asserted unconditionally.  When every code matches, the end-to-end waveform is
compared with the reference's.  When a non-decisive code differs (allowed: the fp64 top-2 gap is
below 1e-4 relative, where the CPU reference itself flips codes between thread counts), the
REFERENCE's codes are decoded on the GPU (vq_decode + generator, distil_codec.py:581-594) and that
waveform is held to the same SNR, so a code flip can never turn the waveform check into a pass.
"""
from __future__ import annotations

import numpy as np
import torch


def snr_db(x, ref) -> float:
    x = np.asarray(x.detach().cpu() if torch.is_tensor(x) else x, np.float64).reshape(-1)
    ref = np.asarray(ref.detach().cpu() if torch.is_tensor(ref) else ref, np.float64).reshape(-1)
    return float(10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300)))


def check_codes(gpu_codes, ref_codes, decisive, min_match: float = 0.97) -> float:
    """Exact on decisive frames, >= min_match exact overall; returns the exact-match rate."""
    gc = np.asarray(gpu_codes.cpu() if torch.is_tensor(gpu_codes) else gpu_codes).astype(np.int64)
    rc = np.asarray(ref_codes.cpu() if torch.is_tensor(ref_codes) else ref_codes).astype(np.int64)
    assert gc.shape == rc.shape, (gc.shape, rc.shape)
    assert np.array_equal(gc[decisive], rc[decisive]), "codes differ on decisive frames"
    match = float((gc == rc).mean()) if gc.size else 1.0
    assert match >= min_match, match
    return match


def check_wave(eng, gpu_codes, ref_codes, gpu_wav, ref_wav, min_db: float) -> float:
    """SNR of the GPU waveform against the reference's, unconditionally (see module docstring).
    Returns the SNR that was asserted."""
    gc = np.asarray(gpu_codes.cpu() if torch.is_tensor(gpu_codes) else gpu_codes).astype(np.int64)
    rc = np.asarray(ref_codes.cpu() if torch.is_tensor(ref_codes) else ref_codes).astype(np.int64)
    ref_wav = np.asarray(ref_wav, np.float64).reshape(gc.shape[0], -1)
    if np.array_equal(gc, rc):
        wav = gpu_wav
    else:
        wav = eng.generate(eng.vq_decode(torch.from_numpy(rc).to(torch.int32)))
    wav = np.asarray(wav.detach().cpu(), np.float64).reshape(ref_wav.shape)
    snr = snr_db(wav, ref_wav)
    assert snr >= min_db, f"waveform SNR {snr:.1f} dB < {min_db} dB (codes identical: {np.array_equal(gc, rc)})"
    return snr
