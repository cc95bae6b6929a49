"""GPU parity of every stage of the HIP path against the reference fixtures and the CPU oracle.

Tolerances (fp32 path, identical inputs per stage):
  mel: max |log-mel diff| < 2e-3 and mean < 2e-5 (direct fp32 DFT vs pocketfft FFT)
  encoder / VQ features / quantized: max relative error < 2e-4
  codes: exact on decisive frames (fp64 relative top-2 gap > 1e-4), >= 97 % exact overall
  waveform: SNR >= 80 dB vs the reference, always (tests/_parity.py: when a non-decisive code
    differs, the reference's codes are decoded on the GPU and held to the same bound)
"""
import numpy as np
import pytest
import torch
from _parity import check_codes, check_wave

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-30)


def _snr(x, ref):
    x = np.asarray(x.detach().cpu() if torch.is_tensor(x) else x, np.float64)
    ref = np.asarray(ref, np.float64)
    return 10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300))


@pytest.fixture(scope="module", params=["x6", "f32"])
def eng(cfg, state, request):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return NativeCodec(cfg, state, "cuda:0", gemm=request.param)


def _decisive(g):
    gap = (g["gap_second"] - g["gap_best"]) / g["gap_best"]
    return (gap > 1e-4).reshape(g["codes"].shape)


@pytest.mark.parametrize("name", ["e2e_batch", "e2e_3s", "e2e_real"])
def test_mel(eng, golden, name):
    g = golden[name]
    mel = eng.mel(torch.from_numpy(g["audio"]))
    d = (mel.transpose(1, 2).cpu().numpy().astype(np.float64) - g["mel"])
    assert np.abs(d).max() < 2e-3, np.abs(d).max()
    assert np.abs(d).mean() < 2e-5, np.abs(d).mean()


def test_encoder(eng, golden):
    g = golden["e2e_batch"]
    feat = eng.encode(torch.from_numpy(g["mel"]).transpose(1, 2))
    assert _rel(feat.transpose(1, 2), g["feat"]) < 2e-4


def test_vq_encode_on_reference_features(eng, golden, state):
    g = golden["e2e_batch"]
    feat = torch.from_numpy(g["feat"]).transpose(1, 2)
    codes, pin, fup, q = eng.vq_encode(feat)
    codes = codes.cpu().numpy()
    dec = _decisive(g)
    assert np.array_equal(codes[dec], g["codes"][dec])
    assert (codes == g["codes"]).mean() >= 0.97
    assert _rel(pin[:1], g["x_pjt_in"]) < 2e-4
    from oracle import reference_cpu as R

    emb = R.codebook(state["quantizer"])
    assert np.array_equal(fup.cpu().numpy(), emb[torch.from_numpy(codes).long()].numpy())
    # `quantized` unconditionally: from our codes when they all match, else decode the reference's
    qz = q if (codes == g["codes"]).all() else eng.vq_decode(torch.from_numpy(g["codes"]))
    assert _rel(qz.transpose(1, 2), g["quantized"]) < 2e-4


def test_vq_decode(eng, golden):
    for name in ("e2e_batch", "e2e_3s", "e2e_real"):
        g = golden[name]
        z = eng.vq_decode(torch.from_numpy(g["codes"]))
        assert _rel(z.transpose(1, 2), g["quantized"]) < 2e-4, name


def test_generator(eng, golden):
    for name in ("e2e_batch", "e2e_3s", "e2e_real"):
        g = golden[name]
        wav = eng.generate(torch.from_numpy(g["quantized"]).transpose(1, 2))
        assert wav.shape == g["wav"].shape
        snr = _snr(wav, g["wav"])
        assert snr >= 80, (name, snr)


@pytest.mark.parametrize("name", ["e2e_batch", "e2e_3s", "e2e_real"])
def test_encode_decode_end_to_end(eng, golden, name):
    g = golden[name]
    codes, wav = eng.encode_decode(torch.from_numpy(g["audio"]))
    check_codes(codes, g["codes"], _decisive(g))
    check_wave(eng, codes, g["codes"], wav, g["wav"], 80)
