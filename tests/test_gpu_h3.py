"""The h3 arithmetic of the wide generator stages (Knobs::h3, the default; DCX_H3=0 gives x6).

The ResBlock convs of the C = 512 / 256 / 128 stages take their inputs as two fp16 values
(h = fp16(x), l = fp16(x - h): 22 significant bits) and the weights likewise after a power-of-two
scale, and sum hh' + hl' + lh' in fp32 (half the MFMAs of x6).  Bounds:
  * a stage's ParallelBlock against the fp64 oracle: max relative error < 2e-4, the bound the x6
    path is held to (tests/test_gpu_modules.py), and within 4x of the x6 path's own error;
  * the generator output against the x6 path on the same input: SNR >= 100 dB (fp32-level
    agreement; two fp32-accurate sums in different orders), and against the reference's waveform
    fixtures >= 80 dB as the x6 path (tests/test_gpu_stages.py).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-30)


def _snr(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    return 10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300))


@pytest.fixture(scope="module")
def eng(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return NativeCodec(cfg, state, "cuda:0", gemm="x6")


def _cl(x):
    return torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 1))).to("cuda:0")


@pytest.mark.parametrize("stage", [0, 1, 2])
def test_parallel_block_h3_vs_oracle(eng, state, cfg, stage):
    from oracle import reference_cpu as R

    C = cfg["decoder"]["upsample_initial_channel"] >> (stage + 1)
    x = torch.from_numpy(np.random.default_rng(10 + stage).standard_normal((2, C, 300)).astype(np.float32))
    ref = torch.nn.functional.silu(R.parallel_block(x.double(), state["generator"], stage, cfg["decoder"], torch.float64))
    ref = ref.numpy()
    with eng.knobs(DCX_H3=0):
        y6 = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    with eng.knobs(DCX_H3=1):
        y3 = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    e6, e3 = _rel(y6, ref), _rel(y3, ref)
    print(f"\nstage {stage} (C = {C}): x6 rel err {e6:.3g}, h3 rel err {e3:.3g}")
    assert e3 < 2e-4
    assert e3 < 4 * max(e6, 1e-7)


@pytest.mark.parametrize("stage", [0, 2])
def test_resblock_h3_vs_oracle(eng, state, cfg, stage):
    """One ResBlock1 (the per-module path: silu_act writes the h2 input)."""
    from oracle import reference_cpu as R

    C = cfg["decoder"]["upsample_initial_channel"] >> (stage + 1)
    x = torch.from_numpy(np.random.default_rng(20 + stage).standard_normal((1, C, 257)).astype(np.float32))
    d = cfg["decoder"]
    k, dils = d["resblock_kernel_sizes"][2], d["resblock_dilation_sizes"][2]
    ref = R._resblock1(x.double(), state["generator"], f"resblocks.{stage}.blocks.2", k, dils, torch.float64).numpy()
    with eng.knobs(DCX_H3=1):
        y3 = eng.module(f"generator.resblocks.{stage}.blocks.2", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    assert _rel(y3, ref) < 2e-4


def test_generator_h3_vs_x6(eng, golden):
    for name in ("e2e_batch", "e2e_real"):
        g = golden[name]
        z = torch.from_numpy(g["quantized"]).transpose(1, 2)
        with eng.knobs(DCX_H3=0):
            w6 = eng.generate(z).cpu().numpy()
        w3 = eng.generate(z).cpu().numpy()
        s36, s3r = _snr(w3, w6), _snr(w3, g["wav"])
        print(f"\n{name}: h3 vs x6 {s36:.1f} dB, h3 vs reference {s3r:.1f} dB (x6 vs reference {_snr(w6, g['wav']):.1f})")
        assert s36 >= 100, (name, s36)
        assert s3r >= 80, (name, s3r)


def test_h3_knob_switches_back(eng, golden):
    """The knob switches kernels only where it says: x6, h3, x6 again gives the first bits, and h3
    runs are reproducible."""
    g = golden["e2e_3s"]
    z = torch.from_numpy(g["quantized"]).transpose(1, 2)
    with eng.knobs(DCX_H3=0):
        a = eng.generate(z).cpu().numpy()
    c = eng.generate(z).cpu().numpy()
    with eng.knobs(DCX_H3=0):
        b = eng.generate(z).cpu().numpy()
    assert np.array_equal(a, b)
    assert np.array_equal(c, eng.generate(z).cpu().numpy())
    assert not np.array_equal(a, c)


def test_split_issue_same_bits_and_reproducible(eng):
    """conv_gemm_x3dw's split DMA issue (Knobs::h3_split) changes only who issues the copies: same
    bits as the unsplit issue, and run-to-run identical (round 5: before group 0's step-0 reads were
    in the handshake, the last clip of a 32-clip batch differed between runs)."""
    from distilcodec_nabeel_amd import synth

    n, L = 16, 72000
    audio = torch.zeros(n, L + 1)
    for i, c in enumerate(synth.clips(n, L, seed=3, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.to("cuda:0")
    c0, w0 = eng.encode_decode(audio)
    for _ in range(3):
        c, w = eng.encode_decode(audio)
        assert torch.equal(c, c0) and torch.equal(w, w0)
    with eng.knobs(DCX_H3_SPLIT=0):
        c, w = eng.encode_decode(audio)
    assert torch.equal(c, c0) and torch.equal(w, w0)


@pytest.mark.parametrize("stage,bn", [(0, 128), (0, 256), (2, 128)])
def test_tilings_agree(eng, state, cfg, stage, bn):
    """Every h3 tiling (x3dw 256 x 256 / 384 x 128 by default, x3dq 256 x 128 and 128 x 256 with
    DCX_H3_BN) sums every output in the same order: same bits."""
    C = cfg["decoder"]["upsample_initial_channel"] >> (stage + 1)
    x = torch.from_numpy(np.random.default_rng(5).standard_normal((1, C, 900)).astype(np.float32))
    ref = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy()
    with eng.knobs(DCX_H3_BN=bn):
        y = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy()
    assert np.array_equal(y, ref)


def test_encoder_h3_vs_x6(eng, golden):
    """The ConvNeXt blocks' 1x1 convs (conv_gemm_x3dm, Knobs::h3_1x1): encoder features against
    the reference within the x6 bound, and within 4x of the x6 path's own error."""
    g = golden["e2e_batch"]
    mel = torch.from_numpy(g["mel"]).transpose(1, 2)
    with eng.knobs(DCX_H3_1X1=0):
        f6 = eng.encode(mel).transpose(1, 2).cpu().numpy()
    f3 = eng.encode(mel).transpose(1, 2).cpu().numpy()
    e6, e3 = _rel(f6, g["feat"]), _rel(f3, g["feat"])
    print(f"\nencoder rel err: x6 {e6:.3g}, h3 {e3:.3g}")
    assert e3 < 2e-4
    assert e3 < 4 * max(e6, 1e-7)


def test_convnext_block_h3_vs_oracle(eng, golden, state):
    m = golden["modules"]
    x = _cl(m["convnext256_in"])
    with eng.knobs(DCX_H3_1X1=0):
        y6 = eng.module("encoder.stages.0.0", x).transpose(1, 2).cpu().numpy()
    y3 = eng.module("encoder.stages.0.0", x).transpose(1, 2).cpu().numpy()
    assert _rel(y3, m["convnext256_out"]) < 2e-4
    assert not np.array_equal(y3, y6)  # the h3 path ran


@pytest.mark.parametrize("i", [0, 1, 2])
def test_wide_conv_transpose_h3(eng, golden, i):
    """ups[0] / ups[1] / ups[2] (Cout 512 / 256 / 128, 2 / 3 / 2 polyphase taps) on conv_gemm_x3dw
    (256 x 256 tiles, 384 x 128 for Cout 128) against the reference's fixture, as the x6 path."""
    m = golden["modules"]
    x = _cl(m[f"ups{i}_in"])
    with eng.knobs(DCX_H3=0):
        y6 = eng.module(f"generator.ups.{i}", x).transpose(1, 2).cpu().numpy()
    y3 = eng.module(f"generator.ups.{i}", x).transpose(1, 2).cpu().numpy()
    e6, e3 = _rel(y6, m[f"ups{i}_out"]), _rel(y3, m[f"ups{i}_out"])
    assert e3 < 2e-4 and e3 < 4 * max(e6, 1e-7), (e3, e6)
    assert not np.array_equal(y3, y6)  # the h3 path ran


def test_conv_pre_h3(eng, state, cfg):
    """conv_pre (k 13, 1024 -> 1024) on conv_gemm_x3dw against an fp64 conv1d of the same weights."""
    from oracle import reference_cpu as R

    d = cfg["decoder"]
    sd = state["generator"]
    x = torch.from_numpy(np.random.default_rng(7).standard_normal((2, cfg["quantizer"]["input_dim"], 300))
                         .astype(np.float32))
    k = d["pre_conv_kernel_size"]
    ref = torch.nn.functional.conv1d(x.double(), R._w(sd, "conv_pre", torch.float64), R._t(sd, "conv_pre.bias", torch.float64),
                                     padding=(k - 1) // 2).numpy()
    with eng.knobs(DCX_H3=0):
        y6 = eng.module("generator.conv_pre", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    y3 = eng.module("generator.conv_pre", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    e6, e3 = _rel(y6, ref), _rel(y3, ref)
    print(f"\nconv_pre rel err: x6 {e6:.3g}, h3 {e3:.3g}")
    assert e3 < 2e-5 and e3 < 4 * max(e6, 1e-7)


@pytest.mark.parametrize("stage", [3, 4])
def test_pair_kernels_h3_vs_oracle(eng, state, cfg, stage):
    """The C = 64 / 32 ParallelBlocks on conv_res_pair_h3 (Knobs::h3_pairs) against the fp64 oracle,
    as the x6 pair kernels."""
    from oracle import reference_cpu as R

    C = cfg["decoder"]["upsample_initial_channel"] >> (stage + 1)
    x = torch.from_numpy(np.random.default_rng(30 + stage).standard_normal((2, C, 1000)).astype(np.float32))
    ref = torch.nn.functional.silu(R.parallel_block(x.double(), state["generator"], stage, cfg["decoder"], torch.float64))
    ref = ref.numpy()
    with eng.knobs(DCX_H3_PAIRS=0):
        y6 = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    with eng.knobs(DCX_H3_PAIRS=1):
        y3 = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy())).cpu().numpy().transpose(0, 2, 1)
    e6, e3 = _rel(y6, ref), _rel(y3, ref)
    print(f"\nstage {stage} (C = {C}) pairs: x6 rel err {e6:.3g}, h3 rel err {e3:.3g}")
    assert e3 < 2e-4 and e3 < 4 * max(e6, 1e-7)
    assert not np.array_equal(y3, y6)


def test_generator_h3_pairs_vs_x6(eng, golden):
    g = golden["e2e_batch"]
    z = torch.from_numpy(g["quantized"]).transpose(1, 2)
    with eng.knobs(DCX_H3=0, DCX_H3_1X1=0, DCX_H3_PAIRS=0):
        w6 = eng.generate(z).cpu().numpy()
    w3 = eng.generate(z).cpu().numpy()
    s36, s3r = _snr(w3, w6), _snr(w3, g["wav"])
    print(f"\nh3 + h3 pairs: vs x6 {s36:.1f} dB, vs reference {s3r:.1f} dB")
    assert s36 >= 100 and s3r >= 80
