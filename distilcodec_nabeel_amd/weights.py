"""Checkpoint handling: reference-format state dicts, synthetic weights, weight-norm folding.

The reference checkpoint `g_00204000` is a dict `{generator, encoder, quantizer}` of module
state dicts (`distilcodec/distil_codec.py:480-492`).  Convolutions of the generator are
weight-norm parametrised (`torch.nn.utils.parametrizations.weight_norm`, dim=0), stored as
`<name>.parametrizations.weight.original0` (g) and `.original1` (v); the legacy
`<name>.weight_g` / `<name>.weight_v` spelling is accepted too.  For `ConvTranspose1d` the
weight is (C_in, C_out, k) so g is per INPUT channel (`ups.0...original0` is (1024, 1, 1)).

No trained checkpoint is available offline, so tests and benchmarks use
`synthetic_state_dict`: deterministic numpy PCG64 weights whose scales keep every layer's
activations O(1) (the reference's own inits are degenerate for testing: ConvNeXt γ = 1e-6,
HiFiGAN std 0.01, kaiming codebook |e| <= 2.3e-4 -- SURVEY.md §7.1).
"""
from __future__ import annotations

import zlib

import numpy as np

# Calibrated once against the oracle so that the codebook matches the scale of
# `x_pjt_in` features (per-dimension std of project_in outputs on speech-like input).
CODEBOOK_STD = 0.55


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def _normal(seed, key, shape, std, mean=0.0):
    r = _rng(seed, key)
    return (r.standard_normal(size=shape, dtype=np.float32) * np.float32(std) + np.float32(mean)).astype(np.float32)


def _convnext(sd, seed, prefix, dim, gamma_mean):
    sd[f"{prefix}.gamma"] = np.abs(_normal(seed, prefix + ".gamma", (dim,), 0.1, gamma_mean)).astype(np.float32)
    sd[f"{prefix}.dwconv.weight"] = _normal(seed, prefix + ".dwconv.weight", (dim, 1, 7), 1.0 / np.sqrt(7))
    sd[f"{prefix}.dwconv.bias"] = _normal(seed, prefix + ".dwconv.bias", (dim,), 0.05)
    sd[f"{prefix}.norm.weight"] = _normal(seed, prefix + ".norm.weight", (dim,), 0.1, 1.0)
    sd[f"{prefix}.norm.bias"] = _normal(seed, prefix + ".norm.bias", (dim,), 0.05)
    sd[f"{prefix}.pwconv1.weight"] = _normal(seed, prefix + ".pwconv1.weight", (4 * dim, dim), 1.0 / np.sqrt(dim))
    sd[f"{prefix}.pwconv1.bias"] = _normal(seed, prefix + ".pwconv1.bias", (4 * dim,), 0.05)
    sd[f"{prefix}.pwconv2.weight"] = _normal(seed, prefix + ".pwconv2.weight", (dim, 4 * dim), 1.0 / np.sqrt(4 * dim))
    sd[f"{prefix}.pwconv2.bias"] = _normal(seed, prefix + ".pwconv2.bias", (dim,), 0.05)


def _wn(sd, seed, prefix, shape, std, bias_std=0.02, bias=True):
    """Weight-norm parametrised conv: v ~ N(0,1); g chosen so the folded weight has `std`."""
    v = _normal(seed, prefix + ".v", shape, 1.0)
    n = int(np.prod(shape[1:]))
    g = (np.float32(std * np.sqrt(n)) * (1.0 + 0.1 * _normal(seed, prefix + ".g", (shape[0], 1, 1), 1.0))).astype(np.float32)
    sd[f"{prefix}.parametrizations.weight.original0"] = g
    sd[f"{prefix}.parametrizations.weight.original1"] = v
    if bias:
        out_ch = shape[1] if prefix.startswith("ups.") else shape[0]
        sd[f"{prefix}.bias"] = _normal(seed, prefix + ".bias", (out_ch,), bias_std)


PARTS = ("encoder", "quantizer", "generator")


def synthetic_state_dict(cfg: dict, seed: int = 1234, with_generator: bool = True) -> dict:
    """Deterministic reference-format checkpoint `{encoder, quantizer, generator}` (numpy fp32)."""
    return {"encoder": synthetic_encoder(cfg, seed), "quantizer": synthetic_quantizer(cfg, seed),
            "generator": synthetic_generator(cfg, seed) if with_generator else {}}


class LazyState(dict):
    """`{part: state dict}` that synthesises a part (the same tensors synthetic_state_dict gives)
    only when it is first read.  `DistilCodec.from_pretrained` assigns the checkpoint's parts before
    anything reads them, so it never builds the 1.2 GB it replaces (the generator stays synthetic,
    i.e. at its "initial weights", unless `use_generator`)."""

    def __init__(self, cfg: dict, seed: int = 1234, parts=PARTS):
        super().__init__()
        self._cfg, self._seed, self._parts = cfg, seed, tuple(parts)

    def __missing__(self, part):
        if part not in self._parts:
            raise KeyError(part)
        v = {"encoder": synthetic_encoder, "quantizer": synthetic_quantizer, "generator": synthetic_generator}[part](
            self._cfg, self._seed)
        self[part] = v
        return v

    def materialised(self) -> tuple:
        return tuple(k for k in PARTS if dict.__contains__(self, k))


def synthetic_encoder(cfg: dict, seed: int = 1234) -> dict:
    enc_cfg = cfg["encoder"]
    dims, depths, cin = enc_cfg["dims"], enc_cfg["depths"], enc_cfg["input_channels"]
    k = enc_cfg["kernel_size"]

    enc = {}
    enc["downsample_layers.0.0.weight"] = _normal(seed, "enc.stem.w", (dims[0], cin, k), 1.0 / np.sqrt(cin * k))
    enc["downsample_layers.0.0.bias"] = _normal(seed, "enc.stem.b", (dims[0],), 0.05)
    enc["downsample_layers.0.1.weight"] = _normal(seed, "enc.stem.lnw", (dims[0],), 0.1, 1.0)
    enc["downsample_layers.0.1.bias"] = _normal(seed, "enc.stem.lnb", (dims[0],), 0.05)
    for i in range(1, len(dims)):
        p = f"downsample_layers.{i}"
        enc[f"{p}.0.weight"] = _normal(seed, p + ".lnw", (dims[i - 1],), 0.1, 1.0)
        enc[f"{p}.0.bias"] = _normal(seed, p + ".lnb", (dims[i - 1],), 0.05)
        enc[f"{p}.1.weight"] = _normal(seed, p + ".w", (dims[i], dims[i - 1], 1), 1.0 / np.sqrt(dims[i - 1]))
        enc[f"{p}.1.bias"] = _normal(seed, p + ".b", (dims[i],), 0.05)
    for i, (dim, depth) in enumerate(zip(dims, depths)):
        for j in range(depth):
            _convnext(enc, seed, f"stages.{i}.{j}", dim, 0.3)
    enc["norm.weight"] = _normal(seed, "enc.norm.w", (dims[-1],), 0.1, 1.0)
    enc["norm.bias"] = _normal(seed, "enc.norm.b", (dims[-1],), 0.05)
    return enc


def synthetic_quantizer(cfg: dict, seed: int = 1234) -> dict:
    q_cfg = cfg["quantizer"]
    D, CD, NC = q_cfg["input_dim"], q_cfg["codebook_dim"], q_cfg["codebook_size"]
    qd = {}
    qd["downsample.0.0.weight"] = _normal(seed, "q.down.w", (D, D, 1), 1.0 / np.sqrt(D))
    qd["downsample.0.0.bias"] = _normal(seed, "q.down.b", (D,), 0.05)
    _convnext(qd, seed, "downsample.0.1", D, 0.3)
    qd["upsample.0.0.weight"] = _normal(seed, "q.up.w", (D, D, 1), 1.0 / np.sqrt(D))
    qd["upsample.0.0.bias"] = _normal(seed, "q.up.b", (D,), 0.05)
    _convnext(qd, seed, "upsample.0.1", D, 0.3)
    qd["grvq.rvqs.0.project_in.weight"] = _normal(seed, "q.pin.w", (CD, D), 1.0 / np.sqrt(D))
    qd["grvq.rvqs.0.project_in.bias"] = _normal(seed, "q.pin.b", (CD,), 0.05)
    qd["grvq.rvqs.0.project_out.weight"] = _normal(seed, "q.pout.w", (D, CD), 1.0 / np.sqrt(CD))
    qd["grvq.rvqs.0.project_out.bias"] = _normal(seed, "q.pout.b", (D,), 0.05)
    qd["grvq.rvqs.0.layers.0._codebook.embed"] = _normal(seed, "q.codebook", (1, NC, CD), CODEBOOK_STD)
    qd["grvq.rvqs.0.layers.0._codebook.initted"] = np.ones((1,), np.float32)
    return qd


def synthetic_generator(cfg: dict, seed: int = 1234) -> dict:
    d_cfg = cfg["decoder"]
    gen = {}
    ch = d_cfg["upsample_initial_channel"]
    pre_k, post_k = d_cfg["pre_conv_kernel_size"], d_cfg["post_conv_kernel_size"]
    _wn(gen, seed, "conv_pre", (ch, d_cfg["num_mels"], pre_k), 1.0 / np.sqrt(d_cfg["num_mels"] * pre_k))
    for i, (u, kk) in enumerate(zip(d_cfg["upsample_rates"], d_cfg["upsample_kernel_sizes"])):
        cin_i, cout_i = ch // (2 ** i), ch // (2 ** (i + 1))
        # each output sample of a stride-u ConvTranspose sees cin*k/u taps
        _wn(gen, seed, f"ups.{i}", (cin_i, cout_i, kk), 1.5 / np.sqrt(cin_i * kk / u))
        for b, (rk, dils) in enumerate(zip(d_cfg["resblock_kernel_sizes"], d_cfg["resblock_dilation_sizes"])):
            for c in range(len(dils)):
                _wn(gen, seed, f"resblocks.{i}.blocks.{b}.convs1.{c}", (cout_i, cout_i, rk), 1.5 / np.sqrt(cout_i * rk))
                _wn(gen, seed, f"resblocks.{i}.blocks.{b}.convs2.{c}", (cout_i, cout_i, rk), 0.5 / np.sqrt(cout_i * rk))
    _wn(gen, seed, "conv_post", (1, ch // (2 ** len(d_cfg["upsample_rates"])), post_k), 1.0 / np.sqrt(32 * post_k))
    return gen


def fold_weight_norm(g: np.ndarray, v: np.ndarray) -> np.ndarray:
    """w = g * v / ||v|| with the norm over every dim but 0 (`torch._weight_norm(v, g, 0)`)."""
    v64 = v.astype(np.float64)
    norm = np.sqrt((v64.reshape(v.shape[0], -1) ** 2).sum(axis=1)).reshape((-1,) + (1,) * (v.ndim - 1))
    return (g.astype(np.float64) * v64 / norm).astype(np.float32)


def plain_weight(sd: dict, prefix: str) -> np.ndarray:
    """The effective `<prefix>.weight`, folding weight norm in either key spelling."""
    if f"{prefix}.weight" in sd:
        return np.asarray(sd[f"{prefix}.weight"], dtype=np.float32)
    for gk, vk in ((".parametrizations.weight.original0", ".parametrizations.weight.original1"),
                   (".weight_g", ".weight_v")):
        if prefix + gk in sd:
            return fold_weight_norm(np.asarray(sd[prefix + gk], np.float32), np.asarray(sd[prefix + vk], np.float32))
    raise KeyError(f"checkpoint has no weight for '{prefix}'")


def to_numpy_state(sd) -> dict:
    """torch tensors / numpy arrays -> contiguous fp32 numpy (buffers like `initted` kept as-is)."""
    out = {}
    for k, v in sd.items():
        if hasattr(v, "detach"):
            v = v.detach().cpu().float().numpy()
        out[k] = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
    return out
