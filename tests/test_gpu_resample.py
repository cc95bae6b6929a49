"""GPU resampling front end (dcx_resample_poly) against the CPU restatement (oracle/resample_cpu.py,
itself pinned to scipy.signal.resample_poly in tests/test_resample.py), and its use by the
drop-in's input paths.  Parity with the reference's librosa/soxr_hq is unpinned (absent here).

Tolerance: max |gpu - cpu| <= 1e-6 * max |cpu| (fp64 taps and accumulation, fp32 output)."""
import wave

import numpy as np
import pytest
import scipy.signal as ss
import torch

from oracle import resample_cpu as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sr", [8000, 16000, 22050, 32000, 44100, 48000, 96000, 12345])
@pytest.mark.parametrize("n", [1, 7, 4801])
def test_kernel_matches_oracle(sr, n):
    from distilcodec_nabeel_amd import resample

    x = np.random.default_rng(sr * 7 + n).standard_normal((3, n)).astype(np.float32)
    got = resample.resample(x, sr, 24000).cpu().numpy()
    ref = R.resample(x, sr, 24000)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-6 * max(np.abs(ref).max(), 1e-30)


def test_full_size_batch():
    # 32 x 10 s at 44.1 kHz in one launch (grid.y = rows), checked on a few rows against scipy
    from distilcodec_nabeel_amd import resample

    x = torch.randn(32, 441000, device="cuda") * 0.1
    y = resample.resample(x, 44100, 24000)
    assert y.shape == (32, 240000)
    up, down = resample.ratio(44100, 24000)
    for r in (0, 17, 31):
        ref = ss.resample_poly(x[r].double().cpu().numpy(), up, down)
        assert np.abs(y[r].double().cpu().numpy() - ref).max() <= 1e-6 * np.abs(ref).max()


def _write_wav(path, x, sr):
    pcm = np.clip(np.round(x * 32767), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(x.shape[1] if x.ndim == 2 else 1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())


def test_input_paths_resample(tmp_path, cfg):
    from distilcodec_nabeel_amd import DistilCodec, audio_io, codec as codec_mod, resample

    rng = np.random.default_rng(5)
    t = np.arange(16000 * 2) / 16000.0
    mono16 = (0.3 * np.sin(2 * np.pi * 220 * t) + 0.05 * rng.standard_normal(t.size)).astype(np.float32)
    dc = DistilCodec(cfg)
    dc.move_to_cuda()
    # raw audio at 16 kHz == the same clip resampled first and passed at 24 kHz
    a, _, _ = dc.encode([[mono16, 16000]], raw_audio=True, codes_only=True)
    x24 = resample.resample(mono16, 16000, 24000).cpu().numpy()
    assert np.abs(x24 - R.resample(mono16, 16000, 24000)).max() <= 1e-6 * np.abs(x24).max()
    b, _, _ = dc.encode([[x24, 24000]], raw_audio=True, codes_only=True)
    assert torch.equal(a.codes, b.codes)
    # a 48 kHz stereo file: librosa.load(mono=True) averages, then resamples
    st = np.stack([mono16[:8000], -0.5 * mono16[:8000]], axis=1)
    p = tmp_path / "s48.wav"
    _write_wav(p, st, 48000)
    y, sr = audio_io.load_wav(str(p), 24000)
    xm, _ = audio_io.load_wav_mono(str(p))
    assert sr == 24000 and y.shape == (4000,)
    assert np.abs(y - R.resample(xm, 48000, 24000)).max() <= 1e-6 * np.abs(y).max()
    # load_and_resample_audio: every channel resampled, then the mean (distil_codec.py:676-680)
    z, zsr, dur = codec_mod.load_and_resample_audio(str(p), 24000)
    chans, _ = audio_io.read_wav(str(p))
    ref = R.resample(chans.T, 48000, 24000).mean(axis=0, keepdims=True)
    assert zsr == 24000 and z.shape == (1, 4000) and abs(dur - 8000 / 48000) < 1e-12
    assert np.abs(z - ref).max() <= 1e-6 * np.abs(ref).max()
