"""Drop-in `DistilCodec` surface over the MI355X HIP path.

Mirrors `distilcodec.DistilCodec` (distilcodec/distil_codec.py:29-727) and `GRVQResult`
(distilcodec/vector_quantization/grfvq.py:13-24): same constructor / classmethod / method names,
argument meanings, return types and error behaviour, with every tensor op executed by libdcx.so
kernels on the GPU.  Differences from the reference are listed in DESIGN.md §6; the main ones:

* the module always computes in eval mode (the reference leaves modules in train mode after
  `from_pretrained`, where EMA would mutate the codebook; README calls `.eval()`);
* `enable_bfloat16=True` runs the convs / linears in bf16 like the reference's CUDA autocast
  (engine mode "bf16"), while the mel front end, LayerNorm, residual adds and the VQ distance search
  stay fp32-accurate (the search returns the exact nearest code of the bf16-valued x_pjt_in).  On the
  CPU, where the reference's `device_type="cuda"` autocast is inactive, the reference computes fp32;
* `decode_from_codes_batch` decodes every clip (the reference decodes only clip 0 because of its
  (B,1,L,1) layout -- SURVEY.md §3(C));
* the mel front end runs on the GPU (the reference forces it to the CPU, mel_spec.py:39).
"""
from __future__ import annotations

import contextlib
import json
import os
from dataclasses import dataclass, field
from functools import reduce

import numpy as np
import torch

from . import audio_io, resample, tokens, weights
from .config import check_supported
from .engine import NativeCodec


@dataclass
class GRVQResult:
    """grfvq.py:13-24."""
    quantized: torch.Tensor
    codes: torch.Tensor
    codes_list: list
    total_loss: torch.Tensor
    commitment_loss: torch.Tensor
    codebook_diversity_loss: torch.Tensor
    quantized_fup: torch.Tensor
    quantized_fup_list: list = field(default_factory=list)
    x_pjt_in: torch.Tensor = None
    x_pjt_in_list: list = field(default_factory=list)


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def _cf(x: torch.Tensor) -> torch.Tensor:
    """channels-last (B, T, C) storage -> the reference's (B, C, T) view."""
    return x.transpose(1, 2)


class _Part:
    def __init__(self, codec):
        self._codec = codec

    @property
    def _eng(self) -> NativeCodec:
        return self._codec._engine()


class SpecTransform(_Part):
    """LogMelSpectrogram.forward (mel_spec.py:109-122): (B, N) / (B, 1, N) audio -> (B, n_mels, T).

    `sample_rate` other than the model rate resamples first with torchaudio's default
    `F.resample` (sinc_interp_hann, lowpass width 6, rolloff 0.99; mel_spec.py:112-113), on the GPU
    (`resample.resample_sinc_hann`).  `return_linear=True` also returns the log-compressed linear
    spectrogram (B, n_fft/2 + 1, T) (mel_spec.py:119-120)."""

    def __call__(self, x: torch.Tensor, return_linear: bool = False, sample_rate: int = None):
        if sample_rate is not None and sample_rate != self._codec.spec_config.sampling_rate:
            x = resample.resample_sinc_hann(x, int(sample_rate), self._codec.spec_config.sampling_rate, self._eng.device)
        if x.ndim == 3:
            x = x.squeeze(1)
        if return_linear:
            mel, lin = self._eng.mel(x, linear=True)
            return _cf(mel), _cf(lin)
        return _cf(self._eng.mel(x))


class Encoder(_Part):
    """ConvNeXtEncoder.forward (encoders.py:68-76): (B, 128, T) -> (B, 1024, T)."""

    def __call__(self, mel: torch.Tensor) -> torch.Tensor:
        return _cf(self._eng.encode(_cf(mel)))


class Quantizer(_Part):
    """DownsampleGRVQ (grfvq.py:27-146) in eval mode."""

    def __call__(self, encoded_feature: torch.Tensor) -> GRVQResult:
        codes, pin, fup, q = self._eng.vq_encode(_cf(encoded_feature))
        zero = torch.zeros((), device=codes.device)
        return GRVQResult(quantized=_cf(q), codes=codes.long()[None, :, :, None], codes_list=[], total_loss=zero,
                          commitment_loss=zero.clone(), codebook_diversity_loss=zero.clone(), quantized_fup=fup,
                          quantized_fup_list=[], x_pjt_in=pin, x_pjt_in_list=[])

    forward = __call__

    def encode(self, encoded_feature: torch.Tensor) -> torch.Tensor:
        """grfvq.py:134-139: indices rearranged 'g b l r -> b (g r) l' -> (B, 1, T) int64."""
        codes, *_ = self._eng.vq_encode(_cf(encoded_feature), want_pjt_in=False, want_fup=False, want_quantized=False)
        return codes.long()[:, None, :]

    def decode(self, indices: torch.Tensor) -> torch.Tensor:
        """grfvq.py:141-146 with indices (G=1, B, T, R=1) -> (B, 1024, T).  Like the reference, a
        (B, 1, T, 1) tensor is read with dim 0 as the group axis (get_output_from_indices zips
        groups over dim 0, residual_vq.py:301-303), i.e. only clip 0 of it is decoded."""
        idx = torch.as_tensor(indices)
        if idx.ndim != 4 or idx.shape[-1] != 1:
            raise ValueError("indices must be laid out (groups=1, batch, frames, residuals=1)")
        codes = idx[0, :, :, 0]
        self._codec._check_codes(codes)
        return _cf(self._eng.vq_decode(codes))


class Generator(_Part):
    """HiFiGANGenerator.forward (generators.py:118-147): (B, 1024, T) -> (B, 1, 256 T)."""

    def __call__(self, x: torch.Tensor, template=None, is_debug: bool = False) -> torch.Tensor:
        if template is not None:
            raise NotImplementedError("use_template=false in the published config")
        return self._eng.generate(_cf(x))[:, None, :]


class DistilCodec:
    def __init__(self, configs: dict, is_debug: bool = False, only_quantizer: bool = False, seed: int = 1234):
        check_supported(configs)
        self.is_debug = is_debug
        self.device = None
        self.ckpt_step = 0
        self.codec_config = configs
        self.ngroups = configs["quantizer"]["n_groups"]
        self.nresiduals = configs["quantizer"]["n_codebooks"]
        self.g_ckpt_path = ""
        self.encoder_config = AttrDict(configs["encoder"])
        self.decoder_config = AttrDict(configs["decoder"])
        self.quantizer_config = AttrDict(configs["quantizer"])
        self.quantizer_config.pop("quantizer_type", None)
        self.spec_config = AttrDict(configs["spec_transform"])
        self.only_quantizer = only_quantizer
        self.hop_size = self.spec_config.hop_size
        self.ds_factor = reduce(lambda x, y: x * y, self.quantizer_config.downsample_factor)
        self.tokens_id_offset = configs.get("token_id_offset", 0)
        self.gr_audio_code2token = tokens.construct_audio_code(self.ngroups, self.nresiduals,
                                                               self.quantizer_config.codebook_size, self.tokens_id_offset)
        # The reference builds randomly initialised modules here; the native path uses
        # deterministic synthetic weights of the same architecture (weights.py) instead, built per
        # part on first use so that a checkpoint load never synthesises what it replaces.
        self._state = weights.LazyState(configs, seed=seed, parts=weights.PARTS if not only_quantizer else ("encoder", "quantizer"))
        self._eng = None
        self.spec_transform = SpecTransform(self)
        self.encoder = None if only_quantizer else Encoder(self)
        self.quantizer = Quantizer(self)
        self.generator = None if only_quantizer else Generator(self)

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_pretrained(cls, config_path, model_path, load_steps=-1, is_debug=False, use_generator=False, local_rank=0):
        """distil_codec.py:77-97.  The generator is only taken from the checkpoint when
        `use_generator` (as in the reference; otherwise it keeps its initial weights)."""
        with open(config_path) as f:
            model_config = json.loads(f.read())
        codec = cls(model_config)
        codec.device = torch.device(f"cuda:{local_rank:d}")
        codec.is_debug = is_debug
        codec.ckpt_step = -1
        codec.g_ckpt_path = -1
        state = cls.load_checkpoint(model_path, codec.device)
        if use_generator:
            codec._state["generator"] = weights.to_numpy_state(state["generator"])
        codec._state["encoder"] = weights.to_numpy_state(state["encoder"])
        codec._state["quantizer"] = weights.to_numpy_state(state["quantizer"])
        del state
        codec.move_to_cuda()
        return codec

    @staticmethod
    def load_checkpoint(filepath, device):
        """distil_codec.py:488-492; loads tensors only (weights_only=True, nothing executed)."""
        assert os.path.isfile(filepath)
        return torch.load(filepath, map_location=torch.device("cpu"), weights_only=True)

    def load_state_dict(self, state: dict) -> None:
        """Replace weights with a `{encoder, quantizer[, generator]}` reference-format dict."""
        for part in ("encoder", "quantizer", "generator"):
            if part in state:
                self._state[part] = weights.to_numpy_state(state[part])
        self._eng = None

    def move_to_cuda(self):
        if self.device is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._engine()

    def to(self, device):
        self.device = torch.device(device)
        self._eng = None
        return self

    def cuda(self, device=None):
        return self.to(torch.device("cuda", device if device is not None else torch.cuda.current_device()))

    def eval(self):
        return self

    def _dev(self) -> torch.device:
        if self.device is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        return self.device

    def _engine(self) -> NativeCodec:
        if self._eng is None:
            if self.device is None:
                self.device = torch.device("cuda", torch.cuda.current_device())
            self._eng = NativeCodec(self.codec_config, self._state, self.device, with_generator=not self.only_quantizer)
        return self._eng

    @contextlib.contextmanager
    def _precision(self, enable_bfloat16: bool):
        """torch.autocast(bf16, enabled=enable_bfloat16) of distil_codec.py:550 / 577 / 590 / 621."""
        eng = self._engine()
        if not enable_bfloat16 or eng.gemm == "bf16":
            yield eng
            return
        prev = eng.gemm
        eng.set_gemm("bf16")
        try:
            yield eng
        finally:
            eng.set_gemm(prev)

    # ---------------------------------------------------------------- preprocessing
    def _pad_stack(self, audio_list):
        max_length = max(a.shape[0] for a in audio_list)
        batch = np.zeros((len(audio_list), max_length + 1), dtype=np.float32)
        for i, a in enumerate(audio_list):
            batch[i, 1: 1 + a.shape[0]] = a  # pad (1, max - N), distil_codec.py:133-136
        return batch

    def _lengths(self, n):
        n_hop = n // (self.hop_size * self.ds_factor)
        gen_len = (n // self.hop_size) * (self.hop_size + 1)
        return n_hop, gen_len

    def _finish_preprocess(self, audio_list):
        n_hop_lengths, gen_lengths = zip(*[self._lengths(a.shape[0]) for a in audio_list])
        audios = torch.from_numpy(self._pad_stack(audio_list)).to(self._engine().device)[:, None, :]
        mel_specs = self.spec_transform(audios)
        if self.is_debug:
            print(f"Max lengths: {max(a.shape[0] for a in audio_list)}")
            print(f"Audios shape: {audios.shape}")
        return audios, mel_specs, list(gen_lengths), list(n_hop_lengths)

    def preprocess_raw_audio_batch(self, audio_data_info_list: list):
        """distil_codec.py:99-145: items are [audio (samples,) or (channels, samples), sr]."""
        audio_list = []
        sr_target = self.spec_config.sampling_rate
        for audio, sampling_rate in audio_data_info_list:
            a = np.asarray(audio, dtype=np.float32)
            if sampling_rate != sr_target:  # :108-110, librosa.resample along the last axis (resample.py)
                a = resample.resample(a, int(sampling_rate), sr_target, self._dev()).cpu().numpy()
            if a.ndim == 2:
                a = a.mean(axis=0) if a.shape[0] > 1 else a[0]
            audio_list.append(a)
        return self._finish_preprocess(audio_list)

    def _read_audio_files(self, audio_pathes: list) -> list:
        """The file-reading half of distil_codec.py:147-198: mono float32 per path at the model rate.
        Like the reference (:155-160), ANY failure to read a file (missing, not audio, corrupt)
        substitutes 1 s of N(0,1)*0.05 noise.  Resampling of another rate (librosa.load(sr=24000))
        runs on the GPU outside that fallback, so a missing GPU still fails loudly.  The
        reference's sample-rate ValueError (:161-163) cannot trigger after resampling; it is kept.
        One exception is not a read failure: a valid MP3 stream in a format the host decoder lacks
        (`mp3.Mp3Unsupported`: MPEG-2/2.5, Layer I/II, free format, intensity stereo) would decode in
        the reference's librosa, so it is raised instead of being replaced by noise."""
        from .mp3 import Mp3Unsupported

        audio_list = []
        sr_target = self.spec_config.sampling_rate
        for p in audio_pathes:
            try:
                audio, sampling_rate = audio_io.load_audio_mono(p)
            except Mp3Unsupported:
                raise
            except Exception:
                print(f"Error on audio: {p}")
                audio = (np.random.normal(size=(sr_target,)) * 0.05).astype(np.float32)
                sampling_rate = sr_target
            if sampling_rate != sr_target:
                audio = resample.resample(audio, sampling_rate, sr_target, self._dev()).cpu().numpy()
                sampling_rate = sr_target
            if sampling_rate != sr_target:
                raise ValueError("{} SR doesn't match target {} SR".format(sampling_rate, sr_target))
            audio_list.append(np.asarray(audio, np.float32))
        return audio_list

    def preprocess_audio_batch(self, audio_pathes: list):
        """distil_codec.py:147-198 (file paths -> padded batch, mel)."""
        return self._finish_preprocess(self._read_audio_files(audio_pathes))

    # ---------------------------------------------------------------- tokens
    def construct_audio_code(self, tokens_id_offset: int = 0):
        return tokens.construct_audio_code(self.ngroups, self.nresiduals, self.quantizer_config.codebook_size, tokens_id_offset)

    def audio_tokenize(self, codes: list, n_groups: int, n_residual: int):
        return tokens.audio_tokenize(self.gr_audio_code2token, codes, n_groups, n_residual)

    # ---------------------------------------------------------------- encode / decode
    def encode(self, audio_pathes: list, enable_bfloat16: bool = False, raw_audio: bool = False, codes_only: bool = False):
        """distil_codec.py:545-573 -> (GRVQResult, gen_time_lengths, n_hop_lengths).
        `codes_only=True` (opt-in, not in the reference) skips quantized / feature outputs."""
        if raw_audio:
            _, mel_specs, gen_time_lengths, n_hop_lengths = self.preprocess_raw_audio_batch(audio_pathes)
        else:
            _, mel_specs, gen_time_lengths, n_hop_lengths = self.preprocess_audio_batch(audio_pathes)
        want = not codes_only
        with self._precision(enable_bfloat16) as eng:
            feat = eng.encode(_cf(mel_specs))
            if self.is_debug:
                print(f"Mel spectrums: {mel_specs.shape}")
                print(f"Encoded Mel spectrums: {tuple(_cf(feat).shape)}")
            codes, pin, fup, q = eng.vq_encode(feat, want_pjt_in=want, want_fup=want, want_quantized=want)
        zero = torch.zeros((), device=codes.device)
        ret = GRVQResult(quantized=_cf(q) if q is not None else None, codes=codes.long()[None, :, :, None], codes_list=[],
                         total_loss=zero, commitment_loss=zero.clone(), codebook_diversity_loss=zero.clone(),
                         quantized_fup=fup, quantized_fup_list=[], x_pjt_in=pin, x_pjt_in_list=[])
        codes_host = codes.cpu()
        for b, hop_len in enumerate(n_hop_lengths):
            codes_t = codes_host[b, :hop_len].tolist()
            ret.codes_list.append(self.audio_tokenize(codes=codes_t, n_groups=self.ngroups, n_residual=self.nresiduals))
            if want:
                ret.x_pjt_in_list.append(pin[b, :hop_len].reshape(hop_len * 2, -1).cpu())
                ret.quantized_fup_list.append(fup[b, :hop_len].reshape(hop_len * 2, -1).cpu())
        return ret, gen_time_lengths, n_hop_lengths

    def _check_codes(self, codes: torch.Tensor) -> None:
        nc = self.quantizer_config.codebook_size
        if codes.numel() and (int(codes.max()) >= nc or int(codes.min()) < -nc):
            raise IndexError(f"audio code out of range for a codebook of {nc} entries")

    def decode_from_features(self, quantized_features: torch.Tensor, enable_bfloat16: bool = False) -> torch.Tensor:
        """distil_codec.py:575-579."""
        with self._precision(enable_bfloat16):
            return self.generator(quantized_features)

    def decode_from_codes(self, codes: list, minus_token_offset: bool = True, enable_bfloat16: bool = False) -> torch.Tensor:
        """distil_codec.py:581-594 -> (1, 1, 256 n)."""
        if minus_token_offset:
            for c in codes:
                if c - self.tokens_id_offset < 0:
                    print(f"c is :{c}", flush=True)
            codes = [c - self.tokens_id_offset for c in codes]
        t = torch.tensor(codes, dtype=torch.int64)[None, :]
        self._check_codes(t)
        with torch.no_grad(), self._precision(enable_bfloat16) as eng:
            z = eng.vq_decode(t)
            wav = eng.generate(z)
        return wav[:, None, :]

    def decode_from_codes_batch(self, codes_list: list, minus_token_offset: bool = True, enable_bfloat16: bool = False) -> list:
        """distil_codec.py:598-639: zero-pads to the longest list and returns one (1, 1, 256 L_max)
        tensor per clip.  Unlike the reference (which decodes only clip 0),
        every clip is decoded."""
        if not codes_list:
            return []
        if minus_token_offset:
            codes_list = [[c - self.tokens_id_offset for c in codes] for codes in codes_list]
        max_length = max(len(c) for c in codes_list)
        batched = torch.zeros(len(codes_list), max_length, dtype=torch.int64)
        for i, c in enumerate(codes_list):
            batched[i, : len(c)] = torch.tensor(c, dtype=torch.int64)
        self._check_codes(batched)
        with self._precision(enable_bfloat16) as eng:
            wav = eng.generate(eng.vq_decode(batched))
        return [wav[i: i + 1, None, :].detach() for i in range(len(codes_list))]

    def forward(self, audio_pathes: list):
        """distil_codec.py:518-530 (eval semantics)."""
        audios, mel_specs, gen_time_lengths, n_hop_lengths = self.preprocess_audio_batch(audio_pathes=audio_pathes)
        rvq = self.quantizer(self.encoder(mel_specs))
        return self.generator(rvq.quantized), audios, gen_time_lengths, n_hop_lengths

    __call__ = forward

    def save_wav(self, audio_gen_batch: torch.Tensor, nhop_lengths, audio_names=None, save_path="./log", name_tag="default"):
        """distil_codec.py:640-654 (PCM_16 WAV)."""
        use_org_name = audio_names is not None and len(audio_names) == len(nhop_lengths)
        paths = []
        for i in range(audio_gen_batch.shape[0]):
            a = audio_gen_batch[i, 0, : nhop_lengths[i]].float().cpu().numpy()
            name = f"{name_tag}.wav" if not use_org_name else f"{audio_names[i]}"
            p = os.path.join(save_path, name)
            paths.append(p)
            audio_io.write_wav(p, a, self.spec_config.sampling_rate)
        return paths


# -------------------------------------------------------------------- module-level helpers
def load_and_resample_audio(file_path, target_sr, mono=True, limited=None, device=None):
    """distil_codec.py:657-684 (WAV or MP3 input; every channel resampled on the GPU `device`, then
    the mean)."""
    y, orig_sr = audio_io.read_audio(file_path)
    y = y.T  # (channels, samples) like librosa.load(mono=False)
    audio_duration = y.shape[1] / orig_sr
    if limited is not None and audio_duration > limited and y.shape[1] - int(orig_sr * limited) > 1000:
        start = np.random.randint(0, y.shape[1] - int(orig_sr * limited))
        y = y[:, start: start + int(orig_sr * limited)]
    if orig_sr != target_sr:
        y = resample.resample(y, orig_sr, target_sr, device if device is not None else "cuda").cpu().numpy()
    if mono and y.shape[0] > 1:
        y = np.mean(y, axis=0, keepdims=True)
    return y.astype(np.float32), target_sr, audio_duration


def decode_audio(codec: DistilCodec, audio_tsr, target_sr=24000, plus_offset: bool = True):
    """distil_codec.py:687-708: encode one clip and return its UNTRIMMED code list."""
    with torch.no_grad():
        audio = np.asarray(audio_tsr)[0]
        ret = codec.encode([[audio, target_sr]], enable_bfloat16=True, raw_audio=True, codes_only=True)[0]
        codes = ret.codes.squeeze().cpu().tolist()
        if isinstance(codes, int):
            codes = [codes]
        return [c + codec.tokens_id_offset for c in codes] if plus_offset else codes


def demo_for_generate_audio_codes(codec: DistilCodec, audio_path, target_sr=24000, plus_llm_offset=True):
    """distil_codec.py:711-727."""
    audio_tsr, _, _ = load_and_resample_audio(file_path=audio_path, target_sr=target_sr, device=codec._dev())
    return decode_audio(codec, audio_tsr=audio_tsr, plus_offset=plus_llm_offset)
