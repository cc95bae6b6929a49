"""Import the upstream reference (`/root/reference/distilcodec`) in THIS container only.

Test infrastructure: used by `make_golden.py` to produce the committed fixtures under
`tests/golden/`.  Nothing here runs on the GPU box (the reference does not exist there).

The reference imports third-party packages that are absent from this image.  Only the
arithmetic-free ones are replaced by inert placeholders; the two that carry arithmetic on
the inference path are restated from their published algorithms:

* `torchaudio.functional.melscale_fbanks(norm="slaney", mel_scale="slaney")` (torchaudio 2.4.1,
  `requirements.txt:17`, called at `distilcodec/models/mel_spec.py:85-93`) -> the independent
  implementation `transformers.audio_utils.mel_filter_bank(..., norm="slaney",
  mel_scale="slaney")` that ships in this image, transposed to torchaudio's (n_freqs, n_mels).
* `einx.get_at('q [c] d, b n q -> q b n d', codebooks, indices)` (einx 0.3.0,
  `requirements.txt:2`, called at `vector_quantization/utils/residual_vq.py:123`) -> plain
  advanced indexing `codebooks[q][indices[..., q]]` for the single pattern used.

Placeholders (never reached on the inference path): librosa, soundfile, wandb, loguru,
tensorboard SummaryWriter, torchaudio.transforms, pip `vector_quantize_pytorch` (grfsq only).
"""
from __future__ import annotations

import os
import sys
import types

REF_ROOT = "/root/reference"


def _mod(name: str) -> types.ModuleType:
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


def _install_stubs() -> None:
    import numpy as np
    import torch
    # imported before any placeholder module exists: transformers probes importlib specs
    from transformers.audio_utils import mel_filter_bank

    if "torchaudio" not in sys.modules:
        ta = _mod("torchaudio")
        taf = _mod("torchaudio.functional")
        tat = _mod("torchaudio.transforms")
        ta.functional, ta.transforms = taf, tat

        def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate, norm=None, mel_scale="htk"):
            fb = mel_filter_bank(
                num_frequency_bins=n_freqs, num_mel_filters=n_mels, min_frequency=f_min,
                max_frequency=f_max, sampling_rate=sample_rate, norm=norm, mel_scale=mel_scale,
            )
            return torch.from_numpy(np.asarray(fb, dtype=np.float64)).float()

        def resample(*a, **k):
            raise RuntimeError("torchaudio.functional.resample is not available in this image")

        taf.melscale_fbanks = melscale_fbanks
        taf.resample = resample

        class _Dummy(torch.nn.Module):
            def __init__(self, *a, **k):
                super().__init__()

        tat.MelScale = _Dummy
        tat.Spectrogram = _Dummy

    if "einx" not in sys.modules:
        ex = _mod("einx")

        def get_at(pattern, codebooks, indices):
            assert pattern == "q [c] d, b n q -> q b n d", pattern
            return torch.stack([codebooks[q][indices[..., q]] for q in range(codebooks.shape[0])])

        def where(*a, **k):
            raise RuntimeError("einx.where is only used on the masked path")

        ex.get_at = get_at
        ex.where = where

    for name in ("librosa", "soundfile", "wandb", "loguru"):
        if name not in sys.modules:
            m = _mod(name)
            if name == "wandb":
                m.UsageError = type("UsageError", (Exception,), {})
            if name == "loguru":
                m.logger = types.SimpleNamespace(info=print, warning=print, error=print)

    if "torch.utils.tensorboard" not in sys.modules:
        tb = _mod("torch.utils.tensorboard")
        tb.SummaryWriter = type("SummaryWriter", (), {"__init__": lambda self, *a, **k: None})

    if "vector_quantize_pytorch" not in sys.modules:
        vqp = _mod("vector_quantize_pytorch")
        vqp.GroupedResidualFSQ = object
        vqp.GroupedResidualVQ = object


def import_reference():
    """Return the reference `distilcodec.distil_codec` module, imported from /root/reference."""
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError("the reference checkout is only available in the build container")
    sys.dont_write_bytecode = True  # the reference tree is read-only
    _install_stubs()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import distilcodec.distil_codec as dc  # noqa: E402

    return dc
