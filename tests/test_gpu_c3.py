"""C3 at full size (BASELINE.json configs[2]): encoder + GRFVQ token extraction of 256 x 10 s clips
in bf16 mode (the reference's enable_bfloat16).  At 239,872 VQ rows the search runs in the regime
where the prefilter addresses its input through per-tile buffer descriptors, so
exactness is checked there: the codes equal the fp64 argmin of the returned bf16-valued x_pjt_in
(the reference's search, vector_quantize_pytorch.py:41-45,496-506: first index of the minimum) on a
row sample that covers the first and last row panels, the last clip entirely, and a stride through
the rest.  Parity with the reference's bf16 autocast run is pinned separately on the fixture of the
reference's own modules under CUDA autocast's op lists (tests/test_gpu_bf16_autocast.py: every module,
the end-to-end features / codes / decode, and this search on the reference's own x_pjt_in)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_c3_full_size_codes_are_exact_argmin(cfg):
    from distilcodec_nabeel_amd import synth, weights
    from distilcodec_nabeel_amd.engine import NativeCodec

    B, n = 256, 240000
    state = {"encoder": weights.synthetic_encoder(cfg, 1234), "quantizer": weights.synthetic_quantizer(cfg, 1234)}
    eng = NativeCodec(cfg, state, "cuda:0", with_generator=False, gemm="bf16")
    audio = torch.zeros(B, n + 1)
    for i, c in enumerate(synth.clips(B, n, seed=0, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    feat = eng.encode(eng.mel(audio))
    codes, pin, _, _ = eng.vq_encode(feat, want_fup=False, want_quantized=False)
    T = codes.shape[1]
    assert codes.shape == (B, 937) and pin.shape == (B, T, 3584)
    assert int(codes.min()) >= 0 and int(codes.max()) < 32768
    assert torch.equal(pin, pin.to(torch.bfloat16).float())  # bf16-valued, like autocast's Linear

    rows = B * T
    sample = np.unique(np.concatenate([np.arange(0, 512), np.arange(rows - 2 * T, rows), np.arange(512, rows, 61)]))
    P = pin.reshape(rows, -1)[torch.from_numpy(sample).cuda()].double()
    E = torch.from_numpy(state["quantizer"]["grvq.rvqs.0.layers.0._codebook.embed"][0]).cuda().double()
    e2 = (E ** 2).sum(1)
    want = []
    for s in range(0, P.shape[0], 1024):
        x = P[s: s + 1024]
        want.append(torch.argmin((x ** 2).sum(1)[:, None] + e2[None] - 2.0 * x @ E.T, dim=1))
    want = torch.cat(want).cpu().numpy()
    got = codes.reshape(-1).cpu().numpy()[sample]
    assert np.array_equal(got, want), f"{int((got != want).sum())} of {len(sample)} sampled rows differ"
    # codes-only call (the C3 fast path) returns the same codes
    c2 = eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)[0]
    assert torch.equal(c2, codes)
