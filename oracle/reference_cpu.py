"""ORACLE — test infrastructure only.  CPU restatement of the reference inference path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker / the timed CPU baseline.  The product path
(`distilcodec_nabeel_amd`) never imports it and fails loudly when its HIP library is missing.

Each function restates the reference's eval-mode arithmetic as functional torch-CPU ops (the
same library kernels the reference runs on CPU), from a reference-format state dict
(`{encoder, quantizer, generator}`; see `distilcodec_nabeel_amd/weights.py`).  Citations are
`path:line` under `/root/reference/`.

Parity pinning: `tests/golden/make_golden.py` imports the real reference in the build
container, loads the same synthetic weights into it, and records its outputs as fixtures;
`tests/test_oracle.py` checks this restatement against them.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------------
# mel front end — distilcodec/models/mel_spec.py
# ---------------------------------------------------------------------------------------------


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def melscale_fbanks_slaney(n_freqs=513, f_min=0.0, f_max=12000.0, n_mels=128, sample_rate=24000):
    """torchaudio.functional.melscale_fbanks(norm='slaney', mel_scale='slaney') (torchaudio 2.4.1,
    called at mel_spec.py:85-93).  Returns (n_freqs, n_mels) float32."""
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    m_pts = np.linspace(_hz_to_mel_slaney(f_min), _hz_to_mel_slaney(f_max), n_mels + 2)
    f_pts = _mel_to_hz_slaney(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    enorm = 2.0 / (f_pts[2: n_mels + 2] - f_pts[:n_mels])
    fb = fb * enorm[None, :]
    return fb.astype(np.float32)


def log_mel(audio: torch.Tensor, fb: torch.Tensor | None = None, n_fft=1024, hop=256, win=1024,
            return_linear: bool = False):
    """LogMelSpectrogram.forward (mel_spec.py:109-122) on (B, N) or (B, 1, N) audio -> (B, 128, T);
    with return_linear also compress(linear) (B, n_fft/2 + 1, T) (:119-120)."""
    if audio.ndim == 3:
        audio = audio.squeeze(1)
    # LinearSpectrogram.forward, mel_spec.py:26-57
    y = F.pad(audio.unsqueeze(1), ((win - hop) // 2, (win - hop + 1) // 2), mode="reflect").squeeze(1)
    window = torch.hann_window(win, dtype=audio.dtype)
    spec = torch.stft(y, n_fft, hop_length=hop, win_length=win, window=window, center=False,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    spec = torch.view_as_real(spec)
    spec = torch.sqrt(spec.pow(2).sum(-1) + 1e-6)
    if fb is None:
        fb = torch.from_numpy(melscale_fbanks_slaney()).to(audio.dtype)
    # apply_mel_scale (mel_spec.py:106-107) then compress (mel_spec.py:100-101)
    x = torch.matmul(spec.transpose(-1, -2), fb).transpose(-1, -2)
    x = torch.log(torch.clamp(x, min=1e-5))
    if return_linear:
        return x, torch.log(torch.clamp(spec, min=1e-5))
    return x


def pad_batch(clips: list[np.ndarray]) -> tuple[torch.Tensor, list[int]]:
    """preprocess_raw_audio_batch padding (distil_codec.py:133-137): 1 leading zero, right pad to max."""
    n_max = max(len(c) for c in clips)
    out = torch.zeros(len(clips), n_max + 1, dtype=torch.float32)
    for i, c in enumerate(clips):
        out[i, 1: 1 + len(c)] = torch.as_tensor(np.asarray(c, dtype=np.float32))
    return out, [len(c) for c in clips]


# ---------------------------------------------------------------------------------------------
# building blocks — distilcodec/models/convnext_utils.py
# ---------------------------------------------------------------------------------------------


def _t(sd, key, dtype):
    return torch.as_tensor(np.asarray(sd[key])).to(dtype)


def _w(sd, prefix, dtype):
    """Effective conv weight; folds weight_norm (`torch._weight_norm(v, g, dim=0)`)."""
    if f"{prefix}.weight" in sd:
        return _t(sd, f"{prefix}.weight", dtype)
    g = _t(sd, f"{prefix}.parametrizations.weight.original0", dtype)
    v = _t(sd, f"{prefix}.parametrizations.weight.original1", dtype)
    return torch._weight_norm(v, g, 0)


def layer_norm_cf(x, w, b, eps=1e-6):
    """LayerNorm channels_first (convnext_utils.py:208-213): biased variance over dim 1."""
    u = x.mean(1, keepdim=True)
    s = (x - u).pow(2).mean(1, keepdim=True)
    x = (x - u) / torch.sqrt(s + eps)
    return w[:, None] * x + b[:, None]


def convnext_block(x, sd, p, dtype):
    """ConvNeXtBlock.forward (convnext_utils.py:263-282), eval mode (DropPath identity)."""
    C = x.shape[1]
    h = F.conv1d(x, _t(sd, f"{p}.dwconv.weight", dtype), _t(sd, f"{p}.dwconv.bias", dtype), padding=3, groups=C)
    h = h.permute(0, 2, 1)
    h = F.layer_norm(h, (C,), _t(sd, f"{p}.norm.weight", dtype), _t(sd, f"{p}.norm.bias", dtype), 1e-6)
    h = F.linear(h, _t(sd, f"{p}.pwconv1.weight", dtype), _t(sd, f"{p}.pwconv1.bias", dtype))
    h = F.gelu(h)
    h = F.linear(h, _t(sd, f"{p}.pwconv2.weight", dtype), _t(sd, f"{p}.pwconv2.bias", dtype))
    h = _t(sd, f"{p}.gamma", dtype) * h
    return x + h.permute(0, 2, 1)


# ---------------------------------------------------------------------------------------------
# encoder — distilcodec/models/encoders.py:68-76 (structure :21-60)
# ---------------------------------------------------------------------------------------------


def encoder(mel, sd, depths=(3, 3, 9, 3), dtype=torch.float32):
    x = mel.to(dtype)
    for i in range(len(depths)):
        p = f"downsample_layers.{i}"
        if i == 0:
            x = F.conv1d(x, _t(sd, f"{p}.0.weight", dtype), _t(sd, f"{p}.0.bias", dtype), padding=3)
            x = layer_norm_cf(x, _t(sd, f"{p}.1.weight", dtype), _t(sd, f"{p}.1.bias", dtype))
        else:
            x = layer_norm_cf(x, _t(sd, f"{p}.0.weight", dtype), _t(sd, f"{p}.0.bias", dtype))
            x = F.conv1d(x, _t(sd, f"{p}.1.weight", dtype), _t(sd, f"{p}.1.bias", dtype))
        for j in range(depths[i]):
            x = convnext_block(x, sd, f"stages.{i}.{j}", dtype)
    return layer_norm_cf(x, _t(sd, "norm.weight", dtype), _t(sd, "norm.bias", dtype))


# ---------------------------------------------------------------------------------------------
# quantizer — grfvq.py:105-146, residual_vq.py:103-259, vector_quantize_pytorch.py:41-45,462-538
# ---------------------------------------------------------------------------------------------


def codebook(sd_q, dtype=torch.float32):
    return _t(sd_q, "grvq.rvqs.0.layers.0._codebook.embed", dtype)[0]


def vq_search(x_pjt_in: torch.Tensor, embed: torch.Tensor, chunk: int = 4096) -> torch.Tensor:
    """EuclideanCodebook.forward eval path: `dist = -cdist(x, embed)` (vector_quantize_pytorch.py:41-45,
    496) then `argmax` (gumbel_sample eval branch, :96) -> first index of the minimum distance.
    Computed in the dtype of the inputs (fp32 in the reference: autocast off + x.float(), :462,473).
    Chunked over rows so the (rows, 32768) matrix stays bounded; each row is independent."""
    flat = x_pjt_in.reshape(-1, x_pjt_in.shape[-1])
    y2 = (embed ** 2).sum(-1)
    out = []
    for s in range(0, flat.shape[0], chunk):
        x = flat[s: s + chunk]
        x2 = (x ** 2).sum(-1)
        xy = torch.einsum("i d, j d -> i j", x, embed) * -2
        dist = -((x2[:, None] + y2[None, :] + xy).clamp(min=0).sqrt())
        out.append(dist.argmax(dim=-1))
    return torch.cat(out).reshape(x_pjt_in.shape[:-1])


def vq_forward(feat, sd_q, dtype=torch.float32):
    """DownsampleGRVQ.forward (grfvq.py:105-132) eval mode, G=1, R=1, downsample factor 1.

    Returns dict: quantized (B,1024,T), codes (1,B,T,1) int64, x_pjt_in (B,T,3584),
    quantized_fup (B,T,3584)."""
    x = F.conv1d(feat.to(dtype), _t(sd_q, "downsample.0.0.weight", dtype), _t(sd_q, "downsample.0.0.bias", dtype))
    x = convnext_block(x, sd_q, "downsample.0.1", dtype)
    x = x.mT  # grvq(encoded_ds.mT), grfvq.py:116
    x_pjt_in = F.linear(x, _t(sd_q, "grvq.rvqs.0.project_in.weight", dtype), _t(sd_q, "grvq.rvqs.0.project_in.bias", dtype))
    embed = codebook(sd_q, dtype)
    idx = vq_search(x_pjt_in, embed)
    quantize = embed[idx]  # batched_embedding, vector_quantize_pytorch.py:243-247
    q_down = F.linear(quantize, _t(sd_q, "grvq.rvqs.0.project_out.weight", dtype), _t(sd_q, "grvq.rvqs.0.project_out.bias", dtype))
    quantized = _vq_upsample(q_down.mT, sd_q, dtype)
    return {"quantized": quantized, "codes": idx[None, :, :, None], "x_pjt_in": x_pjt_in, "quantized_fup": quantize}


def _vq_upsample(x, sd_q, dtype):
    x = F.conv_transpose1d(x, _t(sd_q, "upsample.0.0.weight", dtype), _t(sd_q, "upsample.0.0.bias", dtype))
    return convnext_block(x, sd_q, "upsample.0.1", dtype)


def vq_decode(codes_bt: torch.Tensor, sd_q, dtype=torch.float32):
    """DownsampleGRVQ.decode (grfvq.py:141-146) with indices laid out (G=1, B, T, R=1):
    gather (residual_vq.py:123) -> sum over q -> project_out (:138) -> upsample.  Code -1 is the
    masked code (residual_vq.py:120-127): fetched as code 0, then zeroed before project_out; other
    negative codes wrap like torch indexing."""
    embed = codebook(sd_q, dtype)
    mask = codes_bt == -1
    q = embed[codes_bt.masked_fill(mask, 0)].masked_fill(mask[..., None], 0.0)
    q_down = F.linear(q, _t(sd_q, "grvq.rvqs.0.project_out.weight", dtype), _t(sd_q, "grvq.rvqs.0.project_out.bias", dtype))
    return _vq_upsample(q_down.mT, sd_q, dtype)


# ---------------------------------------------------------------------------------------------
# generator — distilcodec/models/generators.py:118-147, convnext_utils.py:106-113,137-138
# ---------------------------------------------------------------------------------------------


def _resblock1(x, sd, p, k, dils, dtype):
    for c, d in enumerate(dils):
        xt = F.silu(x)
        xt = F.conv1d(xt, _w(sd, f"{p}.convs1.{c}", dtype), _t(sd, f"{p}.convs1.{c}.bias", dtype), dilation=d, padding=(k * d - d) // 2)
        xt = F.silu(xt)
        xt = F.conv1d(xt, _w(sd, f"{p}.convs2.{c}", dtype), _t(sd, f"{p}.convs2.{c}.bias", dtype), padding=(k - 1) // 2)
        x = xt + x
    return x


def parallel_block(x, sd, i, cfg_decoder, dtype=torch.float32):
    """ParralelBlock.forward (convnext_utils.py:137-138) of generator stage i: the mean of its
    ResBlock1s (convnext_utils.py:106-113), stacked in block order."""
    d = cfg_decoder
    outs = [_resblock1(x, sd, f"resblocks.{i}.blocks.{b}", rk, dl, dtype)
            for b, (rk, dl) in enumerate(zip(d["resblock_kernel_sizes"], d["resblock_dilation_sizes"]))]
    return torch.stack(outs, dim=0).mean(dim=0)


def generator(z, sd, cfg_decoder, dtype=torch.float32, stages=None):
    d = cfg_decoder
    x = F.conv1d(z.to(dtype), _w(sd, "conv_pre", dtype), _t(sd, "conv_pre.bias", dtype), padding=(d["pre_conv_kernel_size"] - 1) // 2)
    n = len(d["upsample_rates"]) if stages is None else stages
    for i in range(n):
        u, k = d["upsample_rates"][i], d["upsample_kernel_sizes"][i]
        x = F.silu(x)
        x = F.conv_transpose1d(x, _w(sd, f"ups.{i}", dtype), _t(sd, f"ups.{i}.bias", dtype), stride=u, padding=(k - u) // 2)
        x = parallel_block(x, sd, i, d, dtype)
    if stages is not None:
        return x
    x = F.silu(x)
    x = F.conv1d(x, _w(sd, "conv_post", dtype), _t(sd, "conv_post.bias", dtype), padding=(d["post_conv_kernel_size"] - 1) // 2)
    return torch.tanh(x)


# ---------------------------------------------------------------------------------------------
# whole path
# ---------------------------------------------------------------------------------------------


def encode_decode(audio_padded: torch.Tensor, state: dict, cfg: dict, dtype=torch.float32):
    """mel -> encoder -> quantizer.forward -> quantizer.decode(codes) -> generator, like
    `DistilCodec.encode` (distil_codec.py:545-573) followed by `decode_from_codes` (:581-594)
    with batch layout (G=1,B,T,R=1).  Returns a dict of every intermediate."""
    with torch.no_grad():
        mel = log_mel(audio_padded.to(dtype))
        feat = encoder(mel, state["encoder"], tuple(cfg["encoder"]["depths"]), dtype)
        vq = vq_forward(feat, state["quantizer"], dtype)
        z = vq_decode(vq["codes"][0, :, :, 0], state["quantizer"], dtype)
        wav = generator(z, state["generator"], cfg["decoder"], dtype)
    return {"mel": mel, "feat": feat, **vq, "z": z, "wav": wav}


def top2_gap_fp64(x_pjt_in: torch.Tensor, embed: torch.Tensor, chunk: int = 2048):
    """fp64 nearest/second-nearest distances per row: decides which frames are 'decisive'."""
    flat = x_pjt_in.reshape(-1, x_pjt_in.shape[-1]).double()
    e = embed.double()
    e2 = (e ** 2).sum(-1)
    best, second, arg = [], [], []
    for s in range(0, flat.shape[0], chunk):
        x = flat[s: s + chunk]
        d2 = (x ** 2).sum(-1)[:, None] + e2[None, :] - 2 * x @ e.T
        d = d2.clamp(min=0).sqrt()
        v, i = torch.topk(d, 2, dim=-1, largest=False)
        best.append(v[:, 0]); second.append(v[:, 1]); arg.append(i[:, 0])
    return torch.cat(best), torch.cat(second), torch.cat(arg)
