"""Clip sharding across the GPUs of a node.

Clips are independent, so a batch of B clips is cut into contiguous per-rank shards and every
rank runs the whole path on its shard: no collective on the hot path.  One subtlety keeps the
result identical to a single-device run of the reference: `preprocess_*_batch` right-pads every
clip to the BATCH maximum (distil_codec.py:133-136) and the last ~3 codes of a shorter clip depend
on that padding.  The host knows every clip length, so each rank pads to the GLOBAL maximum
without exchanging anything.  The only collective is the optional result gather (codes are
B x T int32, a few MB even at B = 1024), done once after the data path.
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
        out[i, 1: 1 + len(c)] = c
    return out


def gather_rows(local: torch.Tensor, n_total: int, world: int, group=None) -> torch.Tensor:
    """all_gather of per-rank row blocks of unequal size (shard_bounds layout) -> (n_total, ...)."""
    counts = [shard_bounds(n_total, r, world)[1] - shard_bounds(n_total, r, world)[0] for r in range(world)]
    width = max(counts)
    padded = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)


def encode_sharded(run_shard, clips: list, rank: int, world: int, gather: bool = True, group=None):
    """Run `run_shard(padded_audio (b, N+1) np.float32) -> codes (b, T) tensor` on this rank's
    clips, padding to the global maximum; optionally gather all codes to every rank."""
    global_max = max(len(c) for c in clips)
    s, e = shard_bounds(len(clips), rank, world)
    codes = run_shard(pad_to_global(clips[s:e], global_max))
    if not gather or world == 1:
        return codes
    return gather_rows(codes, len(clips), world, group)
