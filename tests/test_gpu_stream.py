"""C5 streaming hop as a captured HIP graph: replay equals eager execution bit-for-bit, and one
hop matches the CPU oracle run on the same 1 s clip (codes exact on decisive frames, waveform SNR)."""
import numpy as np
import pytest
import torch
from _parity import check_codes, check_wave

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
    check_codes(gc, rc, decisive)
    check_wave(eng, gc, rc, torch.from_numpy(gw), ref["wav"][:, 0].numpy(), 80)


def test_graph_survives_workspace_growth(cfg, state):
    """The captured graph owns its workspace: a longer eager call on the same engine (which grows,
    i.e. reallocates, the engine's shared workspace) and a HaloStream push do not disturb later
    replays."""
    from distilcodec_nabeel_amd import synth
    from distilcodec_nabeel_amd.engine import NativeCodec
    from distilcodec_nabeel_amd.streaming import GraphedHop, HaloStream

    eng = NativeCodec(cfg, state, "cuda:0")
    hop = GraphedHop(eng, 24000)
    chunk = torch.from_numpy(synth.speech_like(24000, 31)).cuda()[None]
    c0, w0 = (t.clone() for t in hop(chunk))
    long = torch.nn.functional.pad(torch.from_numpy(synth.music_like(24000 * 6, 32)).cuda()[None], (1, 0))
    eng.encode_decode(long)  # needs a larger workspace than the hop
    hs = HaloStream(eng)
    hs.push(torch.from_numpy(synth.speech_like(24000 * 3, 33)))
    garbage = torch.full_like(long, 0.5)
    eng.encode_decode(garbage)  # reuse the grown shared workspace with other data
    c1, w1 = hop(chunk)
    torch.cuda.synchronize()
    assert torch.equal(c1, c0) and torch.equal(w1, w0)
    ce, we = eng.encode_decode(torch.nn.functional.pad(chunk, (1, 0)))
    assert torch.equal(c1, ce) and torch.equal(w1, we)
