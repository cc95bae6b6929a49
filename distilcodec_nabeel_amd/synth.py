"""Synthetic 24 kHz clips for tests and benchmarks.

Deterministic numpy PCG64; seed per clip = base_seed + clip_id.  `speech_like` is a sum of
amplitude-modulated harmonic stacks with a wandering pitch plus pink noise; `music_like` adds
sustained chords; `white` is 0.1 * N(0, 1).
"""
from __future__ import annotations

import numpy as np

SR = 24000


def _pink(r, n):
    white = r.standard_normal(n)
    spec = np.fft.rfft(white)
    f = np.arange(spec.shape[0], dtype=np.float64)
    f[0] = 1.0
    spec /= np.sqrt(f)
    x = np.fft.irfft(spec, n)
    return x / (np.std(x) + 1e-12)


def speech_like(n: int, seed: int) -> np.ndarray:
    r = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n) / SR
    f0 = 110 + 60 * r.random() + 25 * np.sin(2 * np.pi * (0.5 + r.random()) * t + r.random() * 6)
    phase = 2 * np.pi * np.cumsum(f0) / SR
    syll = 0.5 * (1 + np.sin(2 * np.pi * (3 + 2 * r.random()) * t + r.random() * 6))
    x = np.zeros(n)
    for h in range(1, 16):
        formant = np.exp(-((h * f0 - 700 - 400 * r.random()) / 900.0) ** 2) + 0.3 / h
        x += formant * np.sin(h * phase + r.random() * 6)
    x = x * syll ** 2
    x = x / (np.std(x) + 1e-12) * 0.15 + 0.01 * _pink(r, n)
    return np.clip(x, -0.99, 0.99).astype(np.float32)


def music_like(n: int, seed: int) -> np.ndarray:
    r = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n) / SR
    x = np.zeros(n)
    for _ in range(4):
        f = 110 * 2 ** (r.integers(0, 36) / 12)
        env = np.exp(-((t % (0.5 + r.random())) * (2 + 3 * r.random())))
        x += env * (np.sin(2 * np.pi * f * t) + 0.4 * np.sin(4 * np.pi * f * t + r.random()))
    x = x / (np.std(x) + 1e-12) * 0.12 + 0.02 * _pink(r, n)
    return np.clip(x, -0.99, 0.99).astype(np.float32)


def white(n: int, seed: int) -> np.ndarray:
    r = np.random.Generator(np.random.PCG64(seed))
    return (0.1 * r.standard_normal(n)).astype(np.float32)


def clips(batch: int, n: int, seed: int = 0, kind: str = "speech") -> list[np.ndarray]:
    fn = {"speech": speech_like, "music": music_like, "white": white}
    if kind == "mix":
        return [(speech_like if i % 2 == 0 else music_like)(n, seed + i) for i in range(batch)]
    return [fn[kind](n, seed + i) for i in range(batch)]


def ragged_lengths(n_clips: int, seed: int, max_len: int, min_len: int) -> list[int]:
    """Deterministic clip lengths in [min_len, max_len] for a ragged batch; clip 0 has max_len, so
    the batch maximum is known without drawing every length (C4's global padding)."""
    r = np.random.Generator(np.random.PCG64(seed))
    lens = r.integers(min_len, max_len + 1, size=n_clips).tolist()
    if n_clips:
        lens[0] = max_len
    return [int(x) for x in lens]


def batch_clips(lengths: list[int], start: int, end: int, seed: int = 0) -> list[np.ndarray]:
    """Clips [start, end) of a universal-audio batch (speech-like on even global indices,
    music-like on odd ones; seed per clip = seed + global index), so each rank synthesises only
    its own shard of the global list."""
    return [(speech_like if i % 2 == 0 else music_like)(lengths[i], seed + i) for i in range(start, end)]
