"""Resampling front end on the CPU: the oracle restatement against
scipy.signal.resample_poly, the package's filter design against the oracle's, output lengths, and
the C ABI's argument checks.  Parity with the reference's librosa/soxr_hq is unpinned (absent here);
see oracle/resample_cpu.py.  Tolerance vs scipy: 1e-12 relative (both fp64)."""
from math import gcd

import numpy as np
import pytest
import scipy.signal as ss

from oracle import resample_cpu as R

RATES = [8000, 16000, 22050, 32000, 44100, 48000, 96000, 24000, 12345]


@pytest.mark.parametrize("sr", RATES)
@pytest.mark.parametrize("n", [1, 7, 160, 4801])
def test_oracle_matches_scipy(sr, n):
    x = np.random.default_rng(sr + n).standard_normal((2, n))
    g = gcd(sr, 24000)
    up, down = 24000 // g, sr // g
    ref = ss.resample_poly(x, up, down, axis=-1) if up != down else x
    got = R.resample(x, sr, 24000)
    assert got.shape == ref.shape == (2, -(-n * up // down))
    assert np.abs(got - ref).max() <= 1e-12 * max(np.abs(ref).max(), 1.0)


@pytest.mark.parametrize("sr", [16000, 44100, 48000])
def test_package_design_equals_oracle(sr):
    from distilcodec_nabeel_amd import resample

    up, down = resample.ratio(sr, 24000)
    h, pre = resample.design(up, down)
    h0, pre0 = R.design(up, down)
    assert pre == pre0 and np.array_equal(h, h0)
    assert resample.n_out(441000, *resample.ratio(44100, 24000)) == 240000


def test_abi_rejects_bad_arguments():
    from distilcodec_nabeel_amd import _native

    L = _native.lib()
    bad = _native.DCX_ERR_INVALID_ARG
    assert L.dcx_resample_poly(None, 1, 10, 10, None, 5, 3, 2, 0, None, 15, 15, None) == bad
    assert L.dcx_resample_poly(1, 0, 10, 10, 1, 5, 3, 2, 0, 1, 15, 15, None) == bad  # batch 0
    assert L.dcx_resample_poly(1, 1, 10, 9, 1, 5, 3, 2, 0, 1, 15, 15, None) == bad  # stride < n
    assert L.dcx_resample_poly(1, 1, 10, 10, 1, 5, 0, 2, 0, 1, 15, 15, None) == bad  # up 0


@pytest.mark.parametrize("sr", [8000, 16000, 22050, 44100, 48000, 12345])
def test_sinc_hann_design_equals_torchaudio_form(sr):
    """SpecTransform(sample_rate=...) resamples like torchaudio.functional.resample (mel_spec.py:112-113).
    The package's prototype filter for dcx_resample_poly, applied in fp64, equals the oracle's
    restatement of torchaudio's conv1d formulation (fp64) to 1e-12; torchaudio's fp32 kernel differs
    from it by fp32 rounding.  Parity with torchaudio itself is unpinned (not installed)."""
    import torch

    from distilcodec_nabeel_amd import resample

    x = np.random.default_rng(sr).standard_normal((2, 3001))
    up, down = resample.ratio(sr, 24000)
    h, pre = resample.design_sinc_hann(sr, 24000)
    got = R.apply_poly(x, h, pre, up, down)
    ref64 = R.torchaudio_resample(torch.from_numpy(x), sr, 24000).numpy()
    assert got.shape == ref64.shape == (2, -(-3001 * 24000 // sr))
    assert np.abs(got - ref64).max() <= 1e-12 * np.abs(ref64).max()
    ref32 = R.torchaudio_resample(torch.from_numpy(x.astype(np.float32)), sr, 24000).numpy()
    assert np.abs(got - ref32).max() <= 1e-4 * np.abs(ref64).max()  # torchaudio fp32 kernel rounding
    # DC gain ~1 away from the edges (rolloff 0.99 sinc, Hann window)
    dc = R.apply_poly(np.ones((1, 4000)), h, pre, up, down)[0]
    mid = dc[len(dc) // 4: 3 * len(dc) // 4]
    assert np.abs(mid - 1).max() < 2e-2
