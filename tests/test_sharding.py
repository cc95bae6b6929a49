"""Multi-process clip sharding (world_size 2, gloo, CPU): every rank pads to the GLOBAL max length
and the gathered codes equal a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distilcodec_nabeel_amd import sharding


def _fake_codes(padded: np.ndarray) -> torch.Tensor:
    """Stand-in for the device path with the same batch dependence: frame energy depends on the
    padded length, so a wrong global max changes the result."""
    n = padded.shape[1]
    T = (n + 768 - 1024) // 256 + 1
    x = np.pad(padded, ((0, 0), (384, 384)), mode="reflect")
    e = np.stack([np.abs(x[:, t * 256: t * 256 + 1024]).sum(1) for t in range(T)], 1)
    return torch.from_numpy((e * 1e4).astype(np.int64) % 32768).to(torch.int32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, clips, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = sharding.encode_sharded(_fake_codes, clips, rank, world, gather=True)
        q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_clips", [5, 2])
def test_gloo_world2_matches_single_process(n_clips):
    r = np.random.default_rng(1)
    clips = [r.standard_normal(int(r.integers(3000, 9000))).astype(np.float32) * 0.1 for _ in range(n_clips)]
    expect = _fake_codes(sharding.pad_to_global(clips, max(len(c) for c in clips))).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, 2, port, clips, q)) for rk in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rk in range(2):
        assert np.array_equal(res[rk], expect)


def test_shard_bounds_cover_everything():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            spans = [sharding.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
