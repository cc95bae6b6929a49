"""bf16 GEMM mode: the reference's enable_bfloat16 (torch.autocast bf16, distil_codec.py:550).

The mode's dtypes are pinned to the reference run under CUDA autocast's op policy by
tests/test_gpu_bf16_autocast.py (tests/golden/bf16.npz).  Here, measured on MI355X with margin:
  conv primitive: result == bf16(fp64 conv of the bf16-rounded operands, bias included) to 1 bf16 ulp
    (2^-7 relative), < 1 % of elements differing (measured 0.003-0.035 %)
  codes vs the fp32 reference fixtures: >= 90 % of frames (measured 94-99 %; the reference's own bf16
    codes agree with its fp32 codes on 95 % of e2e_batch's frames)
  VQ search on the bf16-valued x_pjt_in: the exact nearest code on every frame (no tolerance)
  decode of the reference's fp32 codes in bf16 vs the fp32 reference waveform: SNR >= 30 dB
    (the reference's own bf16 decode of the same codes is 39.2 dB from its fp32 one)
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


@pytest.mark.parametrize("case", [(512, 512, 11, 5, 300), (1024, 4096, 1, 1, 190), (64, 64, 7, 3, 700),
                                  (32, 32, 3, 1, 500), (32, 32, 7, 3, 2048), (32, 32, 11, 5, 2048),
                                  (64, 64, 11, 5, 1024), (128, 256, 7, 1, 93),
                                  (256, 1024, 1, 1, 1100)], ids=lambda c: "x".join(map(str, c)))
def test_conv_bf16(case):
    from distilcodec_nabeel_amd.engine import NativeConv

    cin, cout, k, d, L = case
    r = np.random.default_rng(cin + k)
    w = (r.standard_normal((cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
    b = (0.1 * r.standard_normal(cout)).astype(np.float32)
    x = r.standard_normal((2, L, cin)).astype(np.float32)
    y = NativeConv(w, b, dilation=d)(torch.from_numpy(x).cuda(), gemm="bf16").cpu().double()
    # autocast casts the bias with the other operands (the bf16 mode's b16)
    ref = F.conv1d(_bf(torch.from_numpy(x).double()).transpose(1, 2), _bf(torch.from_numpy(w).double()),
                   _bf(torch.from_numpy(b).double()), dilation=d, padding=d * (k - 1) // 2).transpose(1, 2)
    assert torch.equal(y, _bf(y))  # outputs are bf16 values
    err = (y - _bf(ref.float()).double()).abs()
    print(f"\nconv {case}: differing {float((err > 0).double().mean()):.5f}, max rel {float((err / ref.abs().clamp_min(1e-30)).max()):.3e}")
    assert bool((err <= 2.0 ** -7 * ref.abs() + 1e-6 * ref.abs().max()).all())
    assert float((err > 0).double().mean()) < 0.01


@pytest.mark.parametrize("case", [(256, 1024, 1100), (768, 3072, 300)], ids=lambda c: "x".join(map(str, c)))
def test_conv_gelu_bf16(case):
    """pwconv1 + GELU in bf16 mode (the encoder's hidden): bf16(gelu(v)) for v = bf16(conv + b) of the
    same kernel (test_conv_bf16 pins v), with torch's fp32 GELU 0.5 v (1 + erf(v / sqrt 2)), to 1 bf16
    ulp.  The kernel's branch-free erf (gelu_bf16_f) may differ from torch's erf in the last fp32
    bits, which moves a bf16 rounding on a small fraction of elements (mostly the cancelling tail
    v < -2)."""
    from distilcodec_nabeel_amd.engine import NativeConv

    cin, cout, L = case
    r = np.random.default_rng(cin)
    w = (r.standard_normal((cout, cin, 1)) / np.sqrt(cin)).astype(np.float32)
    b = (0.1 * r.standard_normal(cout)).astype(np.float32)
    x = (1.5 * r.standard_normal((2, L, cin))).astype(np.float32)
    conv = NativeConv(w, b)
    y = conv(torch.from_numpy(x).cuda(), gemm="bf16", epi=1).cpu()
    pre = conv(torch.from_numpy(x).cuda(), gemm="bf16", epi=0).cpu()  # bf16(conv + b), same kernel
    ref = _bf(F.gelu(pre))
    assert torch.equal(y, _bf(y))
    err = (y.double() - ref.double()).abs()
    assert bool((err <= 2.0 ** -7 * ref.double().abs() + 1e-6 * ref.double().abs().max()).all())
    assert float((err > 0).double().mean()) < 0.02


@pytest.fixture(scope="module")
def beng(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return NativeCodec(cfg, state, "cuda:0", gemm="bf16")


@pytest.mark.parametrize("name", ["e2e_batch", "e2e_3s", "e2e_real"])
def test_encode_bf16(beng, golden, state, name):
    from oracle import reference_cpu as R

    g = golden[name]
    feat = beng.encode(beng.mel(torch.from_numpy(g["audio"])))
    codes, pin, _, _ = beng.vq_encode(feat, want_fup=False, want_quantized=False)
    assert torch.equal(pin, _bf(pin))  # x_pjt_in is bf16-valued, like autocast's Linear output
    codes = codes.cpu().numpy()
    assert (codes == g["codes"]).mean() >= 0.90
    E = R.codebook(state["quantizer"]).to("cuda:0", torch.float64)
    P = pin.reshape(-1, pin.shape[-1]).double()
    d = (P ** 2).sum(1)[:, None] + (E ** 2).sum(1)[None] - 2.0 * P @ E.T
    assert np.array_equal(codes.reshape(-1), torch.argmin(d, 1).cpu().numpy())


@pytest.mark.parametrize("name", ["e2e_batch", "e2e_real"])
def test_decode_bf16(beng, golden, name):
    g = golden[name]
    wav = beng.generate(beng.vq_decode(torch.from_numpy(g["codes"]))).cpu().double().numpy()
    ref = np.asarray(g["wav"], np.float64)
    snr = 10 * np.log10((ref ** 2).sum() / ((wav - ref) ** 2).sum())
    print(f"\nbf16 decode vs fp32 reference: snr {snr:.2f} dB")
    assert snr >= 35  # measured 39.2-39.7 dB; the reference's own bf16 decode: 39.2 dB


@pytest.fixture(scope="module")
def codec(cfg):
    from distilcodec_nabeel_amd import DistilCodec

    c = DistilCodec(cfg)
    c.move_to_cuda()
    return c


def test_codec_flag_switches_and_restores(codec, golden):
    eng = codec._engine()
    assert eng.gemm == "x6"
    g = golden["e2e_3s"]
    a = g["audio"][0, 1:]
    r16, _, _ = codec.encode([[a, 24000]], enable_bfloat16=True, raw_audio=True, codes_only=True)
    assert eng.gemm == "x6"
    r32, _, _ = codec.encode([[a, 24000]], raw_audio=True, codes_only=True)
    assert (r32.codes.cpu().numpy()[0, :, :, 0] == g["codes"]).mean() >= 0.97
    assert (r16.codes == r32.codes).double().mean() >= 0.90


@pytest.mark.parametrize("B,secs", [(2, 3), (4, 11)])
def test_compact_layout_same_bits(beng, cfg, state, B, secs):
    """bf16 mode stores the activations read by conv_gemm_bf16dm and vq_prefilter_b1 in the compact
    layout (hi plane only, 2 B per element).  The GEMMs read the same hi values either way, so the
    encoder features and x_pjt_in equal the planes-layout run (DCX_NO_COMPACT=1) bit for bit, and the
    codes too (both exact argmins).  4 x 11 s puts every 1x1 conv on conv_gemm_bf16dm; 2 x 3 s mixes
    compact and planes consumers (the narrow 4C -> C convs fall back to planes kernels)."""
    import os

    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.engine import NativeCodec

    os.environ["DCX_NO_COMPACT"] = "1"
    try:
        plain = NativeCodec(cfg, {"encoder": state["encoder"], "quantizer": state["quantizer"]}, "cuda:0",
                            with_generator=False, gemm="bf16")
    finally:
        del os.environ["DCX_NO_COMPACT"]
    n = 24000 * secs
    audio = torch.zeros(B, n + 1)
    for i, c in enumerate(synth.clips(B, n, seed=11, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    outs = []
    for eng in (beng, plain):
        feat = eng.encode(eng.mel(audio))
        codes, pin, _, q = eng.vq_encode(feat, want_fup=False)
        outs.append((feat, codes, pin, q))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_register_epilogue_same_bits(beng):
    """conv_gemm_bf16dm's register epilogue for the pwconv1 launches (MFMA operands swapped, bias +
    GELU + compact stores from the accumulators) against the LDS-staged epilogue
    (DCX_BF16_REG_EPI=0 through dcx_set_knob): encoder features, x_pjt_in and codes bit for bit on a
    batch that puts every 1x1 conv on conv_gemm_bf16dm (4 x 11 s)."""

    from distilcodec_nabeel_amd import synth

    n = 24000 * 11
    audio = torch.zeros(4, n + 1)
    for i, c in enumerate(synth.clips(4, n, seed=12, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    outs = []
    for flag in (1, 0):
        with beng.knobs(DCX_BF16_REG_EPI=flag):
            feat = beng.encode(beng.mel(audio))
            codes, pin, _, q = beng.vq_encode(feat, want_fup=False)
            torch.cuda.synchronize()
        outs.append((feat.clone(), codes.clone(), pin.clone(), q.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_persistent_same_bits(beng):
    """conv_gemm_bf16dp (the pwconv1 launches as one persistent step stream, GELU from the LDS table)
    against conv_gemm_bf16dm<true> (DCX_BF16_PERSIST=0): encoder features, x_pjt_in and codes bit for
    bit, with the table (default), with table limits that send waves with a pre-GELU |x| >= 4
    (DCX_GELU_LUT=8448, a few) or >= 1 (7936, nearly all) through the evaluated epilogue over the
    table's stores, and evaluated throughout (DCX_GELU_LUT=0).  4 x 11 s clips, every 1x1 conv on the bf16 kernels."""

    from distilcodec_nabeel_amd import synth

    n = 24000 * 11
    audio = torch.zeros(4, n + 1)
    for i, c in enumerate(synth.clips(4, n, seed=13, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    outs = []
    for kn in ({"DCX_BF16_PERSIST": 0}, {}, {"DCX_GELU_LUT": 8448}, {"DCX_GELU_LUT": 7936}, {"DCX_GELU_LUT": 0}):
        with beng.knobs(**kn):
            feat = beng.encode(beng.mel(audio))
            codes, pin, _, q = beng.vq_encode(feat, want_fup=False)
            torch.cuda.synchronize()
        outs.append((feat.clone(), codes.clone(), pin.clone(), q.clone()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
