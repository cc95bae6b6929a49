"""Fused ResBlock pairs (conv_res_pair: the C = 64 and C = 32 generator stages, dcx_resblock.hip).

The fused kernel replaces, per ParallelBlock pair index, six conv launches (c1 and c2 of three
ResBlock1s, convnext_utils.py:106-113) and the ParallelBlock mean (:137-138).  Checked:
  * against the CPU oracle's generator in fp64 (generators.py:118-147): waveform SNR >= 80 dB,
    the fp32 tolerance of DESIGN.md §4;
  * against the per-conv launches of the same library (DCX_NO_RESPAIR=1 at handle creation): SNR
    >= 110 dB (both fp32-accurate; only the summation order differs);
  * on clip lengths around the tile edges (stage lengths 128 T / 256 T against tiles of 176 / 496
    rows, shorter than one tile, and ragged), and a clip alone equal bit-for-bit to the same clip in a
    batch of equal-length clips.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _snr(x, ref):
    x = np.asarray(x.detach().cpu() if torch.is_tensor(x) else x, np.float64)
    ref = np.asarray(ref.detach().cpu() if torch.is_tensor(ref) else ref, np.float64)
    return 10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300))


@pytest.fixture(scope="module")
def engines(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    fused = NativeCodec(cfg, state, "cuda:0", gemm="x6")
    os.environ["DCX_NO_RESPAIR"] = "1"
    try:
        plain = NativeCodec(cfg, state, "cuda:0", gemm="x6")
    finally:
        del os.environ["DCX_NO_RESPAIR"]
    return fused, plain


def _z(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, T, 1024, generator=g) * 0.5


@pytest.mark.parametrize("T", [1, 2, 3, 4, 7, 31, 93])
def test_fused_matches_per_conv_launches(engines, T):
    fused, plain = engines
    z = _z(2, T, 100 + T)
    a = fused.generate(z)
    b = plain.generate(z)
    assert torch.isfinite(a).all()
    snr = _snr(a, b)
    print(f"T={T}: fused vs per-conv SNR {snr:.1f} dB")
    assert snr >= 110, snr


@pytest.mark.parametrize("T", [1, 5, 24])
def test_fused_matches_oracle_fp64(engines, cfg, state, T):
    from oracle import reference_cpu as R

    fused, _ = engines
    z = _z(1, T, 7 + T)
    wav = fused.generate(z)
    with torch.no_grad():
        ref = R.generator(z.transpose(1, 2).double(), state["generator"], cfg["decoder"], torch.float64)
    snr = _snr(wav.reshape(-1), ref.reshape(-1))
    print(f"T={T}: fused vs oracle fp64 SNR {snr:.1f} dB")
    assert snr >= 80, snr


def test_fused_batch_invariance(engines):
    fused, _ = engines
    z = _z(3, 40, 5)
    full = fused.generate(z)
    for i in range(3):
        one = fused.generate(z[i: i + 1])
        assert torch.equal(one[0], full[i])


@pytest.mark.parametrize("B,T", [(1, 1), (2, 7), (3, 40), (8, 200)])
def test_pair_kernels_same_bits(engines, B, T):
    """The shipped pair kernels (the barrier-free conv_res_pair_g at C = 32, the step schedule
    conv_res_pair at C = 64) against conv_res_pair_w4 (DCX_RP_W4=1: 4-wave workgroups, two per CU), the
    step schedule at both (DCX_RP_OLD=1) and the barrier-free kernel at both (DCX_RP_G64=1), switched
    per engine with dcx_set_knob: the same MFMAs in the same order per
    accumulator, so the same bits, also over many tiles per workgroup (B=8, T=200: the persistent tile
    loop and the weight stream's wrap-around past the last tile)."""
    fused, _ = engines
    z = _z(B, T, 300 + T)
    with fused.knobs(DCX_H3_PAIRS=0):  # the x6 pair kernels (h3: conv_res_pair_h3, the default)
        a = fused.generate(z)
    outs = []
    for kn in ({"DCX_RP_W4": 1}, {"DCX_RP_OLD": 1}, {"DCX_RP_G64": 1}):
        with fused.knobs(DCX_H3_PAIRS=0, **kn):
            outs.append(fused.generate(z))
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    for b in outs:
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T", [(1, 93), (2, 31), (1, 7)])
def test_tile_rows_same_bits(engines, B, T):
    """The pair kernels on every tile height they are instantiated for (conv_res_pair_w4: 304 / 112 / 48
    rows at C = 32, 112 / 48 at C = 64; the 8-wave kernels: 496 / 240 / 112 at C = 32, 176 / 112 / 48
    at C = 64), which the launcher picks by tile rounds (smaller ones for the C5 hop): every output
    row is computed with the same arithmetic whatever the tile, so every size (DCX_RP_R) gives the
    same bits as the default, on the w4, step-schedule and barrier-free kernels."""
    fused, _ = engines
    z = _z(B, T, 500 + T)
    outs = []
    for r in (304, 496, 240, 112, 176, 48):
        for kn in ({}, {"DCX_RP_W4": 1}, {"DCX_RP_OLD": 1}):
            with fused.knobs(DCX_H3_PAIRS=0, DCX_RP_R=r, **kn):
                outs.append(fused.generate(z))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    # conv_res_pair_h3 (the default): 624 / 240 / 112 rows at C = 32, 240 / 112 / 48 at C = 64
    h3 = [fused.generate(z)]
    for r in (624, 240, 112, 48):
        with fused.knobs(DCX_RP_R=r):
            h3.append(fused.generate(z))
    torch.cuda.synchronize()
    for o in h3[1:]:
        assert torch.equal(h3[0], o)


@pytest.mark.parametrize("B,T", [(1, 1), (2, 7), (3, 40), (8, 200), (1, 93)])
def test_ring_same_bits_as_per_wave_loads(engines, B, T):
    """conv_res_pair_h3's LDS weight ring (round 6, the default) against its per-wave weight loads
    (DCX_RP_RING=0): the same MFMAs in the same order on the same fragments, so the same bits, on
    every tile height (DCX_RP_R) and over many tiles per workgroup (B=8, T=200: the tap stream and its
    counters running on across tiles, and the issue cursor past the last tile); repeated runs of the
    ring agree (its slot handshake has no race)."""
    fused, _ = engines
    z = _z(B, T, 700 + T)
    with fused.knobs(DCX_RP_RING=0):
        a = fused.generate(z)
    outs = [fused.generate(z), fused.generate(z)]
    for r in (624, 240, 112, 48):
        with fused.knobs(DCX_RP_R=r):
            outs.append(fused.generate(z))
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    for b in outs:
        assert torch.equal(a, b)
