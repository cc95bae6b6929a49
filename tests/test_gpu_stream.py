"""C5 streaming hop as a captured HIP graph: replay equals eager execution bit-for-bit, and one
hop matches the CPU oracle run on the same 1 s clip (codes exact on decisive frames, waveform SNR)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_graph_replay_equals_eager(cfg, state):
    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.engine import NativeCodec
    from distilcodec_nabeel_amd.streaming import GraphedHop

    eng = NativeCodec(cfg, state, "cuda:0")
    hop = GraphedHop(eng, 24000)
    assert hop.frames == 93 and hop.wav.shape[1] == 23808
    audio = np.concatenate(synth.clips(1, 24000 * 3, seed=9, kind="speech"))
    for i in range(3):
        chunk = torch.from_numpy(audio[i * 24000:(i + 1) * 24000].astype(np.float32)).cuda()[None]
        codes, wav = eng.encode_decode(torch.nn.functional.pad(chunk, (1, 0)))
        gc, gw = hop(chunk)
        torch.cuda.synchronize()
        assert torch.equal(gc, codes)
        assert torch.equal(gw, wav)
    with pytest.raises(ValueError):
        hop(torch.zeros(1, 100, device="cuda"))


def test_hop_matches_oracle(cfg, state):
    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.engine import NativeCodec
    from distilcodec_nabeel_amd.streaming import GraphedHop
    from oracle import reference_cpu as R

    eng = NativeCodec(cfg, state, "cuda:0")
    hop = GraphedHop(eng, 24000)
    audio = np.concatenate(synth.clips(1, 24000, seed=21, kind="music")).astype(np.float32)
    gc, gw = hop(torch.from_numpy(audio).cuda()[None])
    gc, gw = gc.cpu().numpy(), gw.cpu().numpy()
    padded, _ = R.pad_batch([audio])
    ref = R.encode_decode(padded, state, cfg)
    rc = ref["codes"][0, :, :, 0].numpy()
    best, second, _ = R.top2_gap_fp64(ref["x_pjt_in"], R.codebook(state["quantizer"]))
    decisive = ((second - best) / best > 1e-4).numpy().reshape(rc.shape)
    assert np.array_equal(gc[decisive], rc[decisive])
    if np.array_equal(gc, rc):
        w = ref["wav"][0, 0].numpy().astype(np.float64)
        snr = 10 * np.log10((w ** 2).sum() / max(((gw[0] - w) ** 2).sum(), 1e-300))
        assert snr > 70
