"""Host-side logic of the drop-in surface (no GPU): token wire format, lengths, config checks,
weight-norm folding, WAV I/O, preprocessing layout."""
import os

import numpy as np
import pytest
import torch


def test_token_table_matches_reference_fixture(golden, cfg):
    from distilcodec_nabeel_amd import tokens

    table = tokens.construct_audio_code(1, 1, 32768, cfg["token_id_offset"])
    g = golden["e2e_batch"]
    hop = int(g["n_hop"][0])
    toks = tokens.audio_tokenize(table, g["codes"][0, :hop].tolist(), 1, 1)
    assert [t["absolute_token_id"] for t in toks] == g["tokens0"].tolist()
    t0 = toks[0]
    assert t0["content"] == f"<|g0r0_{t0['absolute_token_id']}|>" and t0["in_codebook_id"] == g["codes"][0, 0]
    sp = table["special_audio_tokens"]
    base = 152064 + 32768
    assert sp[str(base)]["content"] == "<|beginofaudio|>"
    # ids 5..7 carry the reference's +7/+8/+9 absolute ids (distil_codec.py:253-262)
    assert [sp[str(base + i)]["absolute_token_id"] for i in (5, 6, 7)] == [base + 7, base + 8, base + 9]
    assert table["g0r0"]["codebook_size"] == 32768


def test_lengths_match_reference_fixture(golden):
    from distilcodec_nabeel_amd.codec import DistilCodec

    g = golden["e2e_batch"]
    n = [24000, 17000]
    hop = [x // 256 for x in n]
    gen = [(x // 256) * 257 for x in n]
    assert hop == g["n_hop"].tolist() and gen == g["gen_len"].tolist()
    assert DistilCodec._lengths(type("S", (), {"hop_size": 256, "ds_factor": 1})(), 24000) == (93, 23901)


def test_pad_layout_matches_reference(golden):
    from distilcodec_nabeel_amd.sharding import pad_to_global

    g = golden["e2e_batch"]
    a = g["audio"]
    clips = [a[0, 1:24001], a[1, 1:17001]]
    assert np.array_equal(pad_to_global(clips, 24000), a)


def test_config_checks(cfg):
    import copy

    from distilcodec_nabeel_amd import config

    config.check_supported(cfg)
    ref = "/root/reference/configs/model_config.json"
    if os.path.exists(ref):
        config.check_supported(config.load_config(ref))
    bad = copy.deepcopy(cfg)
    bad["quantizer"]["n_groups"] = 2
    with pytest.raises(ValueError):
        config.check_supported(bad)
    bad = copy.deepcopy(cfg)
    bad["decoder"]["use_template"] = True
    with pytest.raises(ValueError):
        config.check_supported(bad)


def test_weight_norm_fold_matches_torch():
    from distilcodec_nabeel_amd import weights

    r = np.random.default_rng(0)
    v = r.standard_normal((8, 4, 5)).astype(np.float32)
    g = r.standard_normal((8, 1, 1)).astype(np.float32)
    w = weights.fold_weight_norm(g, v)
    wt = torch._weight_norm(torch.from_numpy(v), torch.from_numpy(g), 0).numpy()
    assert np.abs(w - wt).max() < 1e-6
    sd = {"a.parametrizations.weight.original0": g, "a.parametrizations.weight.original1": v, "b.weight_g": g, "b.weight_v": v}
    assert np.array_equal(weights.plain_weight(sd, "a"), weights.plain_weight(sd, "b"))
    with pytest.raises(KeyError):
        weights.plain_weight(sd, "c")


def test_wav_roundtrip(tmp_path):
    from distilcodec_nabeel_amd import audio_io

    x = (0.5 * np.sin(np.arange(4800) / 7.0)).astype(np.float32)
    p = str(tmp_path / "a.wav")
    audio_io.write_wav(p, x, 24000)
    y, sr = audio_io.load_wav(p, 24000)
    assert sr == 24000 and y.shape == x.shape and np.abs(y - x).max() < 1.0 / 32767 + 1e-6
    # another rate is resampled on the GPU (tests/test_gpu_resample.py); without one it fails loudly
    from distilcodec_nabeel_amd import _native

    x16, sr16 = audio_io.load_wav_mono(p)
    assert sr16 == 24000 and np.array_equal(x16, y)
    if not torch.cuda.is_available():
        with pytest.raises(_native.NativeUnavailable):
            audio_io.load_wav(p, 16000)


def test_reference_wav_is_readable():
    from distilcodec_nabeel_amd import audio_io

    p = "/root/reference/data/org_audios/0000.wav"
    if not os.path.exists(p):
        pytest.skip("reference data only exists in the build container")
    y, sr = audio_io.load_wav(p, 24000)
    assert sr == 24000 and y.ndim == 1 and y.shape[0] == 280968 and np.abs(y).max() <= 1.0


def test_synthetic_clips_deterministic():
    from distilcodec_nabeel_amd import synth

    a = synth.clips(3, 4000, seed=3, kind="mix")
    b = synth.clips(3, 4000, seed=3, kind="mix")
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert all(np.abs(x).max() < 1 for x in a)


def test_stream_receptive_field(cfg):
    # SURVEY.md §8(f) rank 4 quotes about +-60 encoder and +-21 decoder frames
    from distilcodec_nabeel_amd import streaming

    assert streaming.receptive_field(cfg) == (60, 22)
