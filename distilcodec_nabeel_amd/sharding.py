"""Clip sharding across the GPUs of a node (BASELINE configs[3] "C4").

Clips are independent, so a batch of B clips is cut into contiguous per-rank shards and every
rank runs the whole path on its shard: no collective on the hot path.  One subtlety keeps the
result identical to a single-device run of the reference: `preprocess_*_batch` right-pads every
clip to the BATCH maximum (distil_codec.py:133-136) and the last ~3 codes of a shorter clip depend
on that padding.  The host knows every clip length, so each rank pads to the GLOBAL maximum
without exchanging anything.  The only collective is the result gather (codes are B x T int32,
3.8 MB at B = 1024), done once per batch after the data path: RCCL over xGMI with the "nccl"
backend, or gloo (CPU tensors) in the multi-process tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [start, end) of rank's share (sizes differ by at most one)."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pad_to_global(clips: list, global_max: int) -> np.ndarray:
    """Reference layout for a shard: 1 leading zero, right zero-pad to the global maximum."""
    out = np.zeros((len(clips), global_max + 1), dtype=np.float32)
    for i, c in enumerate(clips):
        if len(c) > global_max:
            raise ValueError(f"clip of {len(c)} samples is longer than the global maximum {global_max}")
        out[i, 1: 1 + len(c)] = c
    return out


def _gather_device(t: torch.Tensor, group) -> torch.device:
    """gloo gathers CPU tensors; nccl (RCCL) gathers device tensors in place."""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else t.device


def gather_rows(local: torch.Tensor, n_total: int, world: int, group=None) -> torch.Tensor:
    """all_gather of per-rank row blocks of unequal size (shard_bounds layout) -> (n_total, ...),
    on the device `local` lives on."""
    counts = [shard_bounds(n_total, r, world)[1] - shard_bounds(n_total, r, world)[0] for r in range(world)]
    if local.shape[0] != counts[dist.get_rank(group)]:
        raise ValueError(f"rank {dist.get_rank(group)} holds {local.shape[0]} rows, its shard is {counts[dist.get_rank(group)]}")
    dev = _gather_device(local, group)
    width = max(counts)
    padded = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    padded[: local.shape[0]] = local.to(dev)
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0).to(local.device)


def encode_sharded(run_shard, clips: list, rank: int, world: int, gather: bool = True, group=None):
    """Run `run_shard(padded_audio (b, N+1) np.float32) -> codes (b, T) tensor` on this rank's
    clips, padding to the global maximum; optionally gather all codes to every rank."""
    global_max = max(len(c) for c in clips)
    s, e = shard_bounds(len(clips), rank, world)
    codes = run_shard(pad_to_global(clips[s:e], global_max))
    if not gather or world == 1:
        return codes
    return gather_rows(codes, len(clips), world, group)


class ShardedEncodeDecode:
    """One rank's share of a clip-sharded encode -> decode (the C4 path).

    `local_clips` are this rank's clips (shard_bounds(n_total, rank, world) of the global list) and
    `global_max` the longest clip of the whole batch.  The padded shard is uploaded once and stays
    resident in HBM; `step()` runs `dcx_encode_decode` on it and gathers the codes of all ranks.
    Results equal a single-device run of the whole batch: each clip sees the same padding, and the
    kernels' tiling depends on the clip length only, never on the batch."""

    def __init__(self, engine, local_clips: list, global_max: int, n_total: int, rank: int = 0, world: int = 1,
                 group=None):
        s, e = shard_bounds(n_total, rank, world)
        if e - s != len(local_clips):
            raise ValueError(f"rank {rank} of {world} should hold {e - s} of {n_total} clips, got {len(local_clips)}")
        self.engine, self.n_total, self.rank, self.world, self.group = engine, n_total, rank, world, group
        self.lengths = [len(c) for c in local_clips]
        self.audio = torch.from_numpy(pad_to_global(local_clips, global_max)).to(engine.device)
        T = engine.num_frames(global_max + 1)
        self.frames = T
        self.codes = torch.empty(len(local_clips), T, dtype=torch.int32, device=engine.device)
        self.wav = torch.empty(len(local_clips), engine.hop * T, device=engine.device)

    def step(self, gather: bool = True):
        """encode -> decode of the shard; returns (all codes (n_total, T) or the local ones, local wav)."""
        if self.audio.shape[0]:
            self.engine.encode_decode(self.audio, self.codes, self.wav)
        if not gather or self.world == 1:
            return self.codes, self.wav
        return gather_rows(self.codes, self.n_total, self.world, self.group), self.wav

    def gather_wav(self) -> torch.Tensor:
        """All ranks' waveforms (n_total, 256 T): large (0.98 GB at C4), for tests and callers that
        want them in one place; the bench leaves them on their GPUs."""
        if self.world == 1:
            return self.wav
        return gather_rows(self.wav, self.n_total, self.world, self.group)
