"""Streaming encode -> decode in fixed hops with the whole hop captured in one HIP graph (C5).

BASELINE.json configs[4] / SURVEY.md §8(d) C5: 1 s hops (24,000 samples -> 93 frames -> 23,808
output samples), B = 1, one hipGraph-captured step, p50/p99 latency. Each hop is encoded and
decoded on its own, exactly as the reference does for a 1 s clip
(`DistilCodec.encode` + `decode_from_codes`, distil_codec.py:545-594). The halo-overlapped
streaming that would make chunked output equal full-clip output is SURVEY §8(f) rank 4 and is not
done here.

The C-ABI stage calls allocate nothing and never synchronise (include/distilcodec_amd.h), so a
whole `dcx_encode_decode` call is captured by `torch.cuda.graph` as it is launched: every kernel
on the capture stream, and the workspace and outputs fixed before capture.
"""
from __future__ import annotations

import torch

from .engine import NativeCodec


class GraphedHop:
    """One captured encode->decode step for `batch` hops of `hop_samples` samples each.

    Each hop is preprocessed like a clip of that length (`preprocess_raw_audio_batch`,
    distil_codec.py:133-136): one zero sample in front, so the static input holds
    hop_samples + 1 samples. `__call__(chunk)` copies the chunk in after the pad, replays the graph
    on the current stream and returns the static (codes, wav) outputs. The next call overwrites
    them, so clone them to keep them.
    """

    def __init__(self, engine: NativeCodec, hop_samples: int = 24000, batch: int = 1):
        self.engine = engine
        self.device = engine.device
        self.hop_samples = hop_samples
        self.batch = batch
        self.frames = engine.num_frames(hop_samples + 1)
        self.audio = torch.zeros(batch, hop_samples + 1, device=self.device)  # [:, 0] stays 0
        self.codes = torch.empty(batch, self.frames, dtype=torch.int32, device=self.device)
        self.wav = torch.empty(batch, engine.hop * self.frames, device=self.device)
        engine.workspace(batch, self.frames)  # allocate before capture
        with torch.cuda.device(self.device):
            # one eager run (module loading, first-launch work) on a side stream, then capture
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                engine.encode_decode(self.audio, self.codes, self.wav)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                engine.encode_decode(self.audio, self.codes, self.wav)

    def __call__(self, chunk: torch.Tensor):
        if tuple(chunk.shape) != (self.batch, self.hop_samples):
            raise ValueError(f"expected a chunk of shape {(self.batch, self.hop_samples)}, got {tuple(chunk.shape)}")
        self.audio[:, 1:].copy_(chunk, non_blocking=True)
        self.graph.replay()
        return self.codes, self.wav
