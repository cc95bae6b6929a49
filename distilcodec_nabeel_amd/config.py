"""Model configuration: the reference's JSON schema (`configs/model_config.json`).

`DistilCodec.__init__` in the reference (`distilcodec/distil_codec.py:30-70`) reads the keys
`spec_transform`, `encoder`, `decoder`, `quantizer` and `token_id_offset`; the other keys
(`summary`, `base_model`, `teacher_quantizer`, `descriminators`) are ignored at inference.
`load_config` accepts the reference's own file unchanged.
"""
from __future__ import annotations

import copy
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_CONFIG_PATH = os.path.join(_HERE, "configs", "distilcodec_24k.json")


def load_config(path: str | None = None) -> dict:
    with open(path or DEFAULT_CONFIG_PATH) as f:
        return json.load(f)


def default_config() -> dict:
    return copy.deepcopy(load_config(DEFAULT_CONFIG_PATH))


def check_supported(cfg: dict) -> None:
    """Raise ValueError for architecture variants the native path does not implement.

    The native path is specialised for the published DistilCodec geometry (single group,
    single residual codebook, downsample factor 1, no template noise branch).  Anything else
    is rejected loudly instead of silently computing something different.
    """
    q = cfg["quantizer"]
    d = cfg["decoder"]
    e = cfg["encoder"]
    s = cfg["spec_transform"]
    problems = []
    if q.get("quantizer_type", "grvq") != "grvq":
        problems.append("quantizer_type must be 'grvq'")
    if q["n_groups"] != 1 or q["n_codebooks"] != 1:
        problems.append("only n_groups=1, n_codebooks=1 is supported")
    if list(q["downsample_factor"]) != [1]:
        problems.append("only downsample_factor=[1] is supported")
    if d.get("use_template", False):
        problems.append("decoder.use_template=true is not supported")
    if s["n_fft"] != 1024 or s["hop_size"] != 256 or s["win_size"] != 1024:
        problems.append("spec_transform must be n_fft=win=1024, hop=256")
    if e["input_channels"] != s["num_mels"]:
        problems.append("encoder.input_channels must equal spec_transform.num_mels")
    if e["kernel_size"] != 7:
        problems.append("encoder.kernel_size must be 7")
    for c in list(e["dims"]) + [q["codebook_dim"], d["upsample_initial_channel"]]:
        if c % 32:
            problems.append(f"channel count {c} must be a multiple of 32")
    ch = d["upsample_initial_channel"]
    for u, k in zip(d["upsample_rates"], d["upsample_kernel_sizes"]):
        if k % u or (k - u) % 2:
            problems.append(f"ConvTranspose k={k} s={u} must have k%s==0 and even k-s")
        ch //= 2
    if ch % 16:
        problems.append("final generator channel count must be a multiple of 16")
    if problems:
        raise ValueError("unsupported DistilCodec configuration: " + "; ".join(problems))
