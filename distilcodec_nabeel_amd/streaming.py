"""Streaming encode -> decode in fixed hops with the whole hop captured in one HIP graph (C5).

BASELINE.json configs[4] / SURVEY.md §8(d) C5: 1 s hops (24,000 samples -> 93 frames -> 23,808
output samples), B = 1, one hipGraph-captured step, p50/p99 latency. Each hop is encoded and
decoded on its own, exactly as the reference does for a 1 s clip
(`DistilCodec.encode` + `decode_from_codes`, distil_codec.py:545-594). `HaloStream` below is the
halo-overlapped variant whose chunked output equals the full-clip output.

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
        # The graph records raw pointers, so it owns its workspace: the engine's shared buffer is
        # reallocated whenever a later call on the same engine needs more (a longer clip, a
        # HaloStream window), which would leave replays writing into freed memory.
        self.ws = torch.empty(engine.workspace_size(batch, self.frames), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            # one eager run (module loading, first-launch work) on a side stream, then capture
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                engine.encode_decode(self.audio, self.codes, self.wav, ws=self.ws)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                engine.encode_decode(self.audio, self.codes, self.wav, ws=self.ws)

    def __call__(self, chunk: torch.Tensor):
        if tuple(chunk.shape) != (self.batch, self.hop_samples):
            raise ValueError(f"expected a chunk of shape {(self.batch, self.hop_samples)}, got {tuple(chunk.shape)}")
        self.audio[:, 1:].copy_(chunk, non_blocking=True)
        self.graph.replay()
        return self.codes, self.wav


def receptive_field(cfg: dict) -> tuple[int, int]:
    """(encoder, decoder) half receptive fields in frames, rounded up, for the architecture in `cfg`
    (about ±60 and ±21).  Encoder: the stem conv plus one depthwise conv
    per ConvNeXt block (encoders.py:21-60) and the quantizer's down block (grfvq.py:105-132).
    Decoder: the quantizer's up block, conv_pre, each stage's ConvTranspose and ResBlocks
    (generators.py:29-147), conv_post, each converted to frames at its stage's rate."""
    import math

    enc, q, dec = cfg["encoder"], cfg["quantizer"], cfg["decoder"]
    dw = 3  # ConvNeXt depthwise k7
    e = enc.get("kernel_size", 7) // 2 + dw * sum(enc["depths"]) + dw  # + the down block
    hop = 1
    for r in dec["upsample_rates"]:
        hop *= r
    d = dw + dec.get("pre_conv_kernel_size", 13) // 2  # up block + conv_pre (frame rate)
    rate = 1
    for r, k in zip(dec["upsample_rates"], dec["upsample_kernel_sizes"]):
        d += math.ceil(k / r / 2) / rate  # ConvTranspose: its input samples, at `rate` per frame
        rate *= r
        res = max(sum(dd * (kk - 1) // 2 + (kk - 1) // 2 for dd in dils)
                  for kk, dils in zip(dec["resblock_kernel_sizes"], dec["resblock_dilation_sizes"]))
        d += res / rate
    d += dec.get("post_conv_kernel_size", 13) // 2 / hop
    return int(e), int(math.ceil(d))


class HaloStream:
    """Streaming encode -> decode whose output equals the full-clip result.

    `push(chunk)` appends samples and returns the waveform samples that became final; `flush()`
    ends the stream and returns the rest.  A frame's code is final once its encoder receptive field
    (`enc_halo` frames each side, plus the 2 / 3 mel frames a segment edge reflects) has arrived;
    a frame's audio is final once the codes `gen_halo` frames around it are.  Each step runs the
    stage kernels on a window: mel + encoder + VQ from `enc_halo + 2` frames before the first new
    code to the end of the received audio, and VQ decode + generator over the new frames plus
    `gen_halo` on each side.  Inside a window the clip edges are the true clip edges (the
    reference's leading zero sample, reflect padding at the end on `flush`), so every emitted
    frame sees the same inputs as in a full-clip run.  Latency: about enc_halo + gen_halo + 3
    frames of look-ahead.  Results equal the full clip up to fp32 summation order (window lengths
    pick other conv tilings).

    Fixed windows (`push_samples`): every push of at most `push_samples` samples runs on windows of
    one shape, the encoder window zero-padded past the received audio and the generator window
    padded with code 0 past the last code.  The padding only reaches frames that are not final
    yet (it sits beyond the receptive field of every emitted frame), so the output is the same
    function of the input.  `graph=True` captures the two window steps (mel -> encoder -> VQ
    search; VQ decode -> generator) in two HIP graphs and replays them, bit-equal to the eager
    fixed-window run; `flush` runs the variable-shape eager step (the clip end is reflected).
    """

    def __init__(self, engine: NativeCodec, enc_halo: int | None = None, gen_halo: int | None = None,
                 record_codes: bool = False, push_samples: int | None = None, graph: bool = False):
        self.engine = engine
        self.code_log = [] if record_codes else None  # every final code, in order (tests / token output)
        e, d = receptive_field(engine.cfg)
        self.enc_halo = e if enc_halo is None else enc_halo
        self.gen_halo = d if gen_halo is None else gen_halo
        self.hop = engine.hop
        # only the still-needed tails are kept: audio from sample a_off (a multiple of 256, in the
        # coordinates of the padded clip, whose sample 0 is the reference's leading zero), codes
        # from frame c_off
        self.audio = torch.zeros(1, device=engine.device)
        self.a_off = 0
        self.codes = torch.empty(0, dtype=torch.int32, device=engine.device)
        self.c_off = 0
        self.emitted = 0  # frames whose audio was returned
        self.done = False
        self.push_samples = push_samples
        self.graphs = None
        if graph and not push_samples:
            raise ValueError("graph=True needs fixed windows: pass push_samples")
        if push_samples:
            self._init_windows(push_samples, graph)

    # ------------------------------------------------------------------ fixed windows
    def _init_windows(self, push: int, graph: bool):
        eng, hop = self.engine, self.hop
        # encoder window: received audio from frame a = (codes done) - enc_halo - 2; with codes done
        # = (mel frames of the previous audio) - enc_halo, it spans at most push + 639 + hop (2 e + 2)
        # samples (the first pushes, a = 0, span less)
        self.n_enc = push + 640 + hop * (2 * self.enc_halo + 2)
        # generator window: the frames that became final (at most ceil(push / hop) + 1) and gen_halo
        # on each side
        self.t_gen = -(-push // hop) + 1 + 2 * self.gen_halo
        dev = eng.device
        self.a_win = torch.zeros(1, self.n_enc, device=dev)
        self.c_win = torch.zeros(1, self.t_gen, dtype=torch.int32, device=dev)
        t_enc = eng.num_frames(self.n_enc)
        self.ws = torch.empty(max(eng.workspace_size(1, t_enc), eng.workspace_size(1, self.t_gen)),
                              dtype=torch.uint8, device=dev)
        self.codes_win = self.wav_win = None
        if graph:
            with torch.cuda.device(dev):
                s = torch.cuda.Stream(dev)  # eager warm-up (first-launch work) off the capture
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s):
                    self._enc_body()
                    self._gen_body()
                torch.cuda.current_stream(dev).wait_stream(s)
                g_enc, g_gen = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_enc):
                    self.codes_win = self._enc_body()
                with torch.cuda.graph(g_gen):
                    self.wav_win = self._gen_body()
            self.graphs = (g_enc, g_gen)

    def _enc_body(self):
        eng = self.engine
        feat = eng.encode(eng.mel(self.a_win, ws=self.ws), ws=self.ws)
        return eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False, ws=self.ws)[0]

    def _gen_body(self):
        eng = self.engine
        return eng.generate(eng.vq_decode(self.c_win, ws=self.ws), ws=self.ws)

    def _encode_window(self, seg: torch.Tensor, final: bool) -> torch.Tensor:
        """Codes of the window whose audio is seg (from its first sample on)."""
        eng = self.engine
        if self.push_samples is None or final:
            return eng.vq_encode(eng.encode(eng.mel(seg.unsqueeze(0))), want_pjt_in=False, want_fup=False,
                                 want_quantized=False)[0][0]
        n = seg.numel()
        if n > self.n_enc:
            raise ValueError(f"push larger than the fixed window allows (push_samples={self.push_samples})")
        self.a_win[0, :n].copy_(seg)
        self.a_win[0, n:].zero_()
        if self.graphs:
            self.graphs[0].replay()
            return self.codes_win[0]
        return self._enc_body()[0]

    def _generate_window(self, codes: torch.Tensor, final: bool) -> torch.Tensor:
        eng = self.engine
        if self.push_samples is None or final:
            return eng.generate(eng.vq_decode(codes.unsqueeze(0)))[0]
        n = codes.numel()
        if n > self.t_gen:
            raise ValueError(f"push larger than the fixed window allows (push_samples={self.push_samples})")
        self.c_win[0, :n].copy_(codes)
        self.c_win[0, n:].zero_()
        if self.graphs:
            self.graphs[1].replay()
            return self.wav_win[0]
        return self._gen_body()[0]

    # ------------------------------------------------------------------ stream
    @property
    def n_codes(self) -> int:
        return self.c_off + self.codes.numel()

    def _final_codes(self, final: bool) -> int:
        n = self.a_off + self.audio.numel()
        if final:
            return self.engine.num_frames(n)
        avail = (n - 640) // 256 + 1 if n >= 640 else 0  # mel frames with no reflected sample
        return max(0, avail - self.enc_halo)

    def _advance(self, final: bool) -> torch.Tensor:
        eng = self.engine
        c_done, c_new = self.n_codes, self._final_codes(final)
        if c_new > c_done:
            a = max(0, c_done - self.enc_halo - 2)
            seg = self.audio[256 * a - self.a_off:]
            codes = self._encode_window(seg, final)
            new_codes = codes[c_done - a:c_new - a].clone()
            self.codes = torch.cat([self.codes, new_codes])
            if self.code_log is not None:
                self.code_log.append(new_codes)
            keep = 256 * max(0, c_new - self.enc_halo - 2)  # the next window's first sample
            self.audio = self.audio[keep - self.a_off:]
            self.a_off = keep
        T = self.n_codes
        f_new = T if final else max(self.emitted, T - self.gen_halo)
        if f_new <= self.emitted:
            return torch.empty(0, device=eng.device)
        g0, g1 = max(0, self.emitted - self.gen_halo), min(T, f_new + self.gen_halo)
        wav = self._generate_window(self.codes[g0 - self.c_off:g1 - self.c_off], final)
        out = wav[self.hop * (self.emitted - g0):self.hop * (f_new - g0)].clone()
        self.emitted = f_new
        drop = max(0, f_new - self.gen_halo) - self.c_off
        self.codes, self.c_off = self.codes[drop:], self.c_off + drop
        return out

    def push(self, chunk) -> torch.Tensor:
        if self.done:
            raise RuntimeError("push after flush")
        chunk = torch.as_tensor(chunk, dtype=torch.float32).to(self.engine.device).reshape(-1)
        if self.push_samples is not None and chunk.numel() > self.push_samples:
            raise ValueError(f"chunk of {chunk.numel()} samples exceeds push_samples={self.push_samples}")
        self.audio = torch.cat([self.audio, chunk])
        return self._advance(final=False)

    def flush(self) -> torch.Tensor:
        self.done = True
        return self._advance(final=True)
