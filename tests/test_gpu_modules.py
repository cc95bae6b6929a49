"""Per-module GPU parity against the reference's OWN module outputs (tests/golden/modules.npz, made by
tests/golden/make_golden.py from the reference's modules with the synthetic weights), through
`dcx_module_forward`: each module runs on the handle's packed weights through the same launches the
stages use, in x6 (default) and IEEE-fp32 arithmetic.  A stage regression is localised here instead
of only end to end.  Reference: convnext_utils.py:106-142,186-282, generators.py:29-147,
vector_quantize_pytorch.py:41-45,496-506, residual_vq.py:120-127, mel_spec.py:109-122.

Tolerances: max relative error < 2e-4 (the stage tolerance of DESIGN.md §4) for convs / blocks,
< 2e-5 for LayerNorm, codes exact against an fp64 argmin and equal to the reference's on decisive rows.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEY = "grvq.rvqs.0.layers.0._codebook.embed"


def _rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-30)


def _cl(x):  # reference (B, C, L) -> channels-last (B, L, C) on the GPU
    return torch.from_numpy(np.ascontiguousarray(np.swapaxes(x, 1, 2))).cuda()


def _cf(y):
    return y.transpose(1, 2).cpu().numpy()


@pytest.fixture(scope="module", params=["x6", "f32"])
def eng(cfg, state, request):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return NativeCodec(cfg, state, "cuda:0", gemm=request.param)


def test_convnext_block(eng, golden):
    m = golden["modules"]
    y = eng.module("encoder.stages.0.0", _cl(m["convnext256_in"]))
    assert _rel(_cf(y), m["convnext256_out"]) < 2e-4


def test_layer_norm(eng, golden):
    m = golden["modules"]
    y = eng.module("encoder.downsample_layers.1.0", _cl(m["convnext256_in"]))
    assert _rel(_cf(y), m["ln256_out"]) < 2e-5


def test_resblock1(eng, golden):
    m = golden["modules"]
    y = eng.module("generator.resblocks.3.blocks.2", _cl(m["resblock64_in"]))
    assert _rel(_cf(y), m["resblock64_out"]) < 2e-4


def test_parallel_block_fused(eng, golden):
    """ParralelBlock(32) of stage 4 as the generator runs it (fused pair kernels in x6 mode), with
    the SiLU that follows it in the generator: silu of the reference's ParallelBlock output."""
    m = golden["modules"]
    y = eng.module("generator.resblocks.4", _cl(m["parallel32_in"]))
    ref = torch.nn.functional.silu(torch.from_numpy(m["parallel32_out"]).double()).numpy()
    assert _rel(_cf(y), ref) < 2e-4


@pytest.mark.parametrize("i", range(5))
def test_conv_transpose(eng, golden, i):
    m = golden["modules"]
    y = eng.module(f"generator.ups.{i}", _cl(m[f"ups{i}_in"]))
    assert _rel(_cf(y), m[f"ups{i}_out"]) < 2e-4


@pytest.mark.parametrize("stage", [0, 3])
def test_parallel_block_other_stages(eng, state, cfg, stage):
    """The grouped per-conv path (stage 0, C = 512) and the C = 64 pair kernel (stage 3) against the
    oracle's ParallelBlock (pinned to the reference by tests/test_oracle.py)."""
    from oracle import reference_cpu as R

    C = cfg["decoder"]["upsample_initial_channel"] >> (stage + 1)
    x = torch.from_numpy(np.random.default_rng(stage).standard_normal((2, C, 300)).astype(np.float32))
    ref = torch.nn.functional.silu(R.parallel_block(x.double(), state["generator"], stage, cfg["decoder"], torch.float64))
    y = eng.module(f"generator.resblocks.{stage}", _cl(x.numpy()))
    assert _rel(_cf(y), ref.numpy()) < 2e-4


def test_masked_decode_fixture(eng, golden):
    """quantizer.decode of codes holding the masked code -1 (residual_vq.py:120-127)."""
    m = golden["modules"]
    z = eng.vq_decode(torch.from_numpy(m["masked_codes"])[None])
    assert _rel(_cf(z), m["masked_z"]) < 2e-4


def test_return_linear(eng, golden):
    m, g = golden["modules"], golden["e2e_batch"]
    mel, lin = eng.mel(torch.from_numpy(g["audio"][:1]), linear=True)
    assert np.abs(_cf(lin) - m["linear_log"]).max() < 2e-3
    assert np.abs(_cf(mel) - m["linear_mel"]).max() < 2e-3


def _fp64_top2(x, E):
    x64, E64 = torch.from_numpy(x).cuda().double(), E.cuda().double()
    d = (x64 ** 2).sum(1)[:, None] + (E64 ** 2).sum(1)[None, :] - 2 * x64 @ E64.T
    v, i = torch.topk(d, 2, dim=1, largest=False)
    return i[:, 0].cpu().numpy(), ((v[:, 1] - v[:, 0]) / v[:, 0]).cpu().numpy()


@pytest.mark.parametrize("gemm", ["x6", "f32"])
def test_search_1024_codes(cfg, state, golden, gemm):
    """The reference's EuclideanCodebook on a 1024-code slice of the codebook.  In fp32 mode the handle
    holds exactly those 1024 codes.  The x6 prefilter tiles 4096-code groups, so there the other 31744
    rows are set far away (|e| > 2 max|x| + max|e|: never nearest) and the same 1024 codes compete."""
    from distilcodec_nabeel_amd.engine import NativeCodec

    m = golden["modules"]
    q = dict(state["quantizer"])
    E = q[KEY][0, :1024]
    c2 = {k: dict(v) if isinstance(v, dict) else v for k, v in cfg.items()}
    if gemm == "f32":
        c2["quantizer"]["codebook_size"] = 1024
        q[KEY] = q[KEY][:, :1024]
    else:
        big = q[KEY].copy()
        far = 4.0 * (np.linalg.norm(m["vq1024_in"], axis=1).max() + np.linalg.norm(E, axis=1).max())
        big[0, 1024:] = far / np.sqrt(big.shape[2])
        q[KEY] = big
    e = NativeCodec(c2, {"encoder": state["encoder"], "quantizer": q}, "cuda:0", with_generator=False, gemm=gemm)
    codes = e.module("quantizer.search", torch.from_numpy(m["vq1024_in"])[None].cuda())[0].cpu().numpy()
    best, gap = _fp64_top2(m["vq1024_in"], torch.from_numpy(E))
    assert np.array_equal(codes, best)
    dec = gap > 1e-4
    assert np.array_equal(codes[dec], m["vq1024_codes"][dec])
    assert (codes == m["vq1024_codes"]).mean() >= 0.97


def test_spec_transform_sample_rate(cfg, state):
    """LogMelSpectrogram.forward(x, sample_rate=16000) (mel_spec.py:112-113): torchaudio's default
    resampler on the GPU, then the mel front end, against the oracle's restatement of torchaudio's
    resample + log-mel.  Parity with torchaudio itself is unpinned (not installed here)."""
    from distilcodec_nabeel_amd import DistilCodec, synth
    from oracle import reference_cpu as R
    from oracle import resample_cpu as RS

    codec = DistilCodec(cfg)
    codec.move_to_cuda()
    x = torch.from_numpy(np.stack([synth.speech_like(16000, 3), synth.music_like(16000, 4)]).astype(np.float32))
    mel = codec.spec_transform(x.cuda()[:, None, :], sample_rate=16000)
    ref = R.log_mel(RS.torchaudio_resample(x.double(), 16000, 24000).float())
    assert mel.shape == ref.shape
    d = np.abs(mel.cpu().numpy() - ref.numpy())
    assert d.max() < 2e-3 and d.mean() < 2e-5
    mel2, lin = codec.spec_transform(x.cuda(), return_linear=True)
    assert lin.shape == (2, 513, mel2.shape[2])


def test_unknown_module_raises(eng):
    with pytest.raises(ValueError):
        eng.module("generator.nonexistent", torch.zeros(1, 4, 32).cuda())


@pytest.mark.parametrize("gemm", ["x6", "bf16"])
@pytest.mark.parametrize("B,secs", [(10, 10.0), (24, 10.0), (72, 10.0)])
def test_dwconv_run_same_bits_as_tiled(cfg, state, gemm, B, secs):
    """dwconv_ln_run (one wave per run of rows, register window; launches of >= 8192 rows) against
    the round-2 tiled kernel (DCX_DWCONV_TILED=1 through dcx_set_knob): the same per-row arithmetic,
    so the encoder features are bit-identical, for runs of 4 (10 x 10 s: 9370 rows), 8 (24 x 10 s)
    and 32 rows (72 x 10 s: 67464 rows), in the x6 and bf16 modes (fp32 / planes / compact outputs)."""

    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.engine import NativeCodec

    e = NativeCodec(cfg, {"encoder": state["encoder"], "quantizer": state["quantizer"]}, "cuda:0",
                    with_generator=False, gemm=gemm)
    n = int(24000 * secs)
    audio = torch.zeros(B, n + 1)
    for i, c in enumerate(synth.clips(B, n, seed=21, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    mel = e.mel(audio.cuda())
    a = e.encode(mel).clone()
    with e.knobs(DCX_DWCONV_TILED=1):
        b = e.encode(mel)
        torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)


def test_module_in_split_k_mode(cfg, state, golden):
    """dcx_module_workspace_size counts the split-K partial-sum scratch that every stage call carves
    ahead of its buffers when the latency mode is on (round 4: without it a module call in that mode
    failed with 'workspace too small'); the split ConvNeXt block stays within the module tolerance."""
    from distilcodec_nabeel_amd.engine import NativeCodec

    e = NativeCodec(cfg, state, "cuda:0", gemm="x6", with_generator=False)
    e.set_split_k(16)
    m = golden["modules"]
    y = e.module("encoder.stages.0.0", _cl(m["convnext256_in"]))
    assert _rel(_cf(y), m["convnext256_out"]) < 2e-4
