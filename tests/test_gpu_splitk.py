"""Split-K latency mode (dcx_set_split_k): few-tile x6 convs split over input-channel chunks into
partial GEMMs plus one reduce kernel that applies the conv's epilogue (BASELINE configs[4], the
streaming latency path).  The arithmetic is the x6 one; only the fp32 summation order changes, so
the stated fp32 tolerances apply:
  * generator against the fp64 oracle (generators.py:118-147): SNR >= 80 dB;
  * encoder features against the unsplit engine: relative error < 2e-5, codes equal on every frame
    whose fp64 top-2 gap exceeds 1e-4 (decisive frames);
  * a graph-captured hop on the split engine replays bit-equal to its eager run.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _snr(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return 10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300))


@pytest.fixture(scope="module")
def engines(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    split = NativeCodec(cfg, state, "cuda:0", gemm="x6")
    split.set_split_k(16)
    plain = NativeCodec(cfg, state, "cuda:0", gemm="x6")
    return split, plain


@pytest.mark.parametrize("T", [3, 24, 139])
def test_generator_matches_oracle(engines, cfg, state, T):
    from oracle import reference_cpu as R

    split, plain = engines
    g = torch.Generator().manual_seed(T)
    z = torch.randn(1, T, 1024, generator=g) * 0.5
    split.profile(True)
    split.profile_reset()
    wav = split.generate(z).cpu().reshape(-1)
    names = split.profile_read()
    split.profile(False)
    assert any(k.startswith("splitk:") for k in names), "no conv was split"
    with torch.no_grad():
        ref = R.generator(z.transpose(1, 2).double(), state["generator"], cfg["decoder"], torch.float64).reshape(-1)
    snr = _snr(wav, ref)
    print(f"T={T}: split-K generator vs fp64 oracle {snr:.1f} dB; "
          f"vs unsplit {_snr(wav, plain.generate(z).cpu().reshape(-1)):.1f} dB")
    assert snr >= 80


def test_encoder_and_codes(engines, state):
    from distilcodec_nabeel_amd import synth
    from oracle import reference_cpu as R

    split, plain = engines
    n = 2 * 24000
    audio = torch.zeros(1, n + 1)
    audio[0, 1:] = torch.from_numpy(synth.clips(1, n, seed=21, kind="speech")[0])
    audio = audio.cuda()
    fa = split.encode(split.mel(audio))
    fb = plain.encode(plain.mel(audio))
    rel = float((fa - fb).abs().max() / fb.abs().max())
    assert rel < 2e-5, rel
    ca, pa, _, _ = split.vq_encode(fa, want_fup=False, want_quantized=False)
    cb, pb, _, _ = plain.vq_encode(fb, want_fup=False, want_quantized=False)
    best, second, _ = R.top2_gap_fp64(pb.cpu().double(), R.codebook(state["quantizer"]))
    decisive = (((second - best) / best) > 1e-4).numpy().reshape(-1)
    a, b = ca.cpu().numpy().reshape(-1), cb.cpu().numpy().reshape(-1)
    assert np.array_equal(a[decisive], b[decisive])


def test_graph_hop_on_split_engine(engines):
    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.streaming import GraphedHop

    split, _ = engines
    hop = GraphedHop(split, 24000)
    x = torch.from_numpy(synth.clips(1, 24000, seed=5, kind="speech")[0]).float().cuda()[None]
    codes, wav = hop(x)
    codes, wav = codes.clone(), wav.clone()
    c2, w2 = split.encode_decode(torch.nn.functional.pad(x, (1, 0)))
    assert torch.equal(codes, c2) and torch.equal(wav, w2)


@pytest.mark.parametrize("T", [24, 93])
def test_grouped_split_launches(engines, cfg, state, T):
    """The three ResBlocks' convs of one dilation index as one grouped split-K launch plus one
    grouped reduce (round 4): the grouped kernel runs (profile), the generator output is within the
    fp32 summation-order distance of the per-conv split launches (DCX_SPLIT_GROUP_OFF=1 through
    dcx_set_knob) and of the fp64 oracle (>= 80 dB)."""

    from oracle import reference_cpu as R

    split, _ = engines
    g = torch.Generator().manual_seed(100 + T)
    z = torch.randn(1, T, 1024, generator=g) * 0.5
    split.profile(True)
    split.profile_reset()
    wav = split.generate(z).cpu().reshape(-1)
    names = split.profile_read()
    split.profile(False)
    assert any("x6pp_group" in k for k in names), sorted(names)
    with split.knobs(DCX_SPLIT_GROUP_OFF=1):
        wav_single = split.generate(z).cpu().reshape(-1)
    with torch.no_grad():
        ref = R.generator(z.transpose(1, 2).double(), state["generator"], cfg["decoder"], torch.float64).reshape(-1)
    s1, s2 = _snr(wav, ref), _snr(wav, wav_single)
    print(f"T={T}: grouped split-K vs fp64 oracle {s1:.1f} dB, vs per-conv split {s2:.1f} dB")
    assert s1 >= 80 and s2 >= 100


def test_grouped_split_respects_split_k(cfg, state):
    """dcx_set_split_k(2) caps the grouped split launches too (round-4 ADVICE: they allocated up to 16
    K-slices per member whatever the handle's limit).  With at most 2 slices per member the grouped and
    the per-conv split launches (DCX_SPLIT_GROUP_OFF=1) give every conv 2 slices, the same partial sums
    and the same reduce order: the same bits.  A grouped launch that ignored the cap would not."""
    from distilcodec_nabeel_amd.engine import NativeCodec

    e = NativeCodec(cfg, state, "cuda:0", gemm="x6")
    e.set_split_k(2)
    g = torch.Generator().manual_seed(77)
    z = torch.randn(1, 93, 1024, generator=g) * 0.5
    e.profile(True)
    e.profile_reset()
    wav = e.generate(z)
    names = e.profile_read()
    e.profile(False)
    assert any("x6pp_group" in k for k in names), sorted(names)
    with e.knobs(DCX_SPLIT_GROUP_OFF=1):
        wav_single = e.generate(z)
    torch.cuda.synchronize()
    assert torch.isfinite(wav).all()
    assert torch.equal(wav, wav_single)
