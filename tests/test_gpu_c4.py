"""C4 (BASELINE.json configs[3]) at its own workload on one GPU: one rank's shard of the 1024-clip
universal-audio batch sharded over 8 GPUs, i.e. 128 ragged 9-10 s speech+music clips padded to the
GLOBAL maximum (distil_codec.py:133-136), run by the shipped `sharding.ShardedEncodeDecode` exactly
as bench.py does at N = 8 (rank 3 of 8 here; the gather is a no-op at world size 1).

Checked: two steps are bit-identical; clip i re-run alone at the global-max padding equals row i
(batch invariance: the other 127 clips do not change it); the shard's first and last clip against
the CPU oracle run on the same padded input (codes exact on decisive frames, waveform >= 80 dB)."""
import numpy as np
import pytest
import torch
from _parity import check_codes, check_wave

pytestmark = pytest.mark.gpu

WORLD, RANK, PER_GPU = 8, 3, 128


@pytest.fixture(scope="module")
def shard(cfg, state):
    from distilcodec_nabeel_amd import sharding, synth
    from distilcodec_nabeel_amd.engine import NativeCodec

    eng = NativeCodec(cfg, state, "cuda:0")
    n_total = PER_GPU * WORLD
    lengths = synth.ragged_lengths(n_total, 7, 240000, 216000)  # bench.py make_runner(seed=0)
    s, e = sharding.shard_bounds(n_total, RANK, WORLD)
    clips = synth.batch_clips(lengths, s, e, seed=0)
    runner = sharding.ShardedEncodeDecode(eng, clips, max(lengths), n_total, RANK, WORLD)
    return eng, runner, clips, max(lengths)


def test_c4_shard_deterministic_and_batch_invariant(shard):
    from distilcodec_nabeel_amd import sharding

    eng, runner, clips, gmax = shard
    assert runner.audio.shape == (PER_GPU, gmax + 1)
    assert len(set(runner.lengths)) > 1 and max(runner.lengths) <= gmax  # ragged, global padding
    c1, w1 = runner.step(gather=False)
    c1, w1 = c1.clone(), w1.clone()
    c2, w2 = runner.step(gather=False)
    torch.cuda.synchronize()
    assert c1.shape == (PER_GPU, eng.num_frames(gmax + 1))
    assert torch.equal(c1, c2) and torch.equal(w1, w2)
    assert int(c1.min()) >= 0 and int(c1.max()) < 32768 and bool(torch.isfinite(w1).all())
    for i in (0, 77, PER_GPU - 1):
        alone = torch.from_numpy(sharding.pad_to_global([clips[i]], gmax)).cuda()
        ci, wi = eng.encode_decode(alone)
        assert torch.equal(ci[0], c1[i]) and torch.equal(wi[0], w1[i]), i


@pytest.mark.parametrize("i", [0, PER_GPU - 1])
def test_c4_clip_against_oracle(shard, state, cfg, i):
    from oracle import reference_cpu as R

    eng, runner, clips, gmax = shard
    codes, wav = runner.step(gather=False)  # rank 3 of 8 without a process group: local rows
    torch.cuda.synchronize()
    audio = runner.audio[i: i + 1].cpu()
    torch.set_num_threads(16)
    ref = R.encode_decode(audio, state, cfg)
    rc = ref["codes"][0, :, :, 0].numpy()
    best, second, _ = R.top2_gap_fp64(ref["x_pjt_in"], R.codebook(state["quantizer"]))
    dec = (((second - best) / best) > 1e-4).numpy().reshape(rc.shape)
    match = check_codes(codes[i: i + 1], rc, dec)
    snr = check_wave(eng, codes[i: i + 1], rc, wav[i: i + 1], ref["wav"][:, 0].numpy(), 80)
    print(f"C4 clip {i} ({len(clips[i])} samples, padded to {gmax}): codes match {match:.4f}, SNR {snr:.1f} dB")
