"""Multi-process clip sharding (world_size 2, gloo, CPU) with the reference's algorithm: each rank
runs the CPU oracle (mel -> encoder -> GRFVQ search, oracle/reference_cpu.py) on its shard padded to
the GLOBAL maximum, and the gathered codes equal a single-process run of the whole batch
(pad-to-batch-max, distil_codec.py:133-136).  The same harness shows why every
rank pads globally: padding a shard to its own maximum changes the codes of its longest clip.
The GPU engine version of this test is tests/test_gpu_sharding.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distilcodec_nabeel_amd import sharding

LENGTHS = [9000, 4000, 6500, 3001, 7777]


def _state(cfg):
    from distilcodec_nabeel_amd import weights

    return {"encoder": weights.synthetic_encoder(cfg, 1234), "quantizer": weights.synthetic_quantizer(cfg, 1234)}


def _oracle_codes(padded: np.ndarray, state, cfg) -> torch.Tensor:
    """Codes of each padded clip, one clip at a time (the CPU library's result then depends on the
    clip and its padding only, not on how clips are grouped)."""
    from oracle import reference_cpu as R

    out = []
    with torch.no_grad():
        for row in padded:
            mel = R.log_mel(torch.from_numpy(row)[None])
            feat = R.encoder(mel, state["encoder"], tuple(cfg["encoder"]["depths"]))
            out.append(R.vq_forward(feat, state["quantizer"])["codes"][0, 0, :, 0])
    return torch.stack(out).to(torch.int32) if out else torch.empty(0, 0, dtype=torch.int32)


def _clips():
    from distilcodec_nabeel_amd import synth

    return synth.batch_clips(LENGTHS, 0, len(LENGTHS), seed=11)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, clips, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from distilcodec_nabeel_amd import config

    cfg = config.default_config()
    state = _state(cfg)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = sharding.encode_sharded(lambda p: _oracle_codes(p, state, cfg), clips, rank, world, gather=True)
        q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def expect(cfg):
    torch.set_num_threads(4)
    clips = _clips()
    state = _state(cfg)
    full = _oracle_codes(sharding.pad_to_global(clips, max(LENGTHS)), state, cfg).numpy()
    # rank 1's shard (clips 3, 4) padded to its own maximum instead of the global one
    s, e = sharding.shard_bounds(len(clips), 1, 2)
    own = _oracle_codes(sharding.pad_to_global(clips[s:e], max(LENGTHS[s:e])), state, cfg).numpy()
    return full, own, (s, e)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_oracle_matches_single_process(expect, world):
    """world 2 (shards 3 + 2 clips) and world 4 (2 + 1 + 1 + 1: uneven, single-clip shards)."""
    full, _, _ = expect
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, world, port, _clips(), q)) for rk in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rk in range(world):
        assert res[rk].shape == full.shape
        assert np.array_equal(res[rk], full)


def test_global_padding_is_what_matters(expect):
    """Clip 4 (7777 samples) is the longest of rank 1's shard: with the shard padded to its own
    maximum, its last frames see the STFT's reflect padding instead of the zeros the whole batch
    gives it, and its codes near the end change (the encoder's receptive field spreads the
    difference over ~60 frames, streaming.receptive_field)."""
    full, own, (s, e) = expect
    n = own.shape[1]
    j = int(np.argmax(LENGTHS[s:e]))
    assert not np.array_equal(full[s + j, :n], own[j])


@pytest.mark.parametrize("world,rows", [(3, 7), (8, 5)])
def test_gather_rows_uneven_shards(world, rows):
    """gather_rows reassembles unequal shards in rank order (gloo): world 3 over 7 rows, and world 8
    over 5 rows, where three ranks hold empty shards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(rk, world, port, rows, q)) for rk in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rk in range(world):
        assert np.array_equal(res[rk], np.arange(rows * 2).reshape(rows, 2))


def _gather_worker(rank, world, port, rows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = sharding.shard_bounds(rows, rank, world)
        local = torch.arange(s * 2, e * 2).reshape(e - s, 2)
        q.put((rank, sharding.gather_rows(local, rows, world).numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_everything():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            spans = [sharding.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_ragged_batch_is_deterministic_and_shardable():
    from distilcodec_nabeel_amd import synth

    lens = synth.ragged_lengths(16, 7, 240000, 216000)
    assert lens[0] == 240000 and min(lens) >= 216000 and lens == synth.ragged_lengths(16, 7, 240000, 216000)
    parts = [synth.batch_clips([1000] * 6, *sharding.shard_bounds(6, r, 3), seed=2) for r in range(3)]
    whole = synth.batch_clips([1000] * 6, 0, 6, seed=2)
    assert all(np.array_equal(a, b) for a, b in zip(sum(parts, []), whole))
    assert all(np.array_equal(a, b) for a, b in zip(whole, synth.clips(6, 1000, seed=2, kind="mix")))
