"""Reference-format checkpoints for the ingestion tests (distil_codec.py:480-492): a dict
`{generator, encoder, quantizer}` of module state dicts, as torch tensors, including what a trained
checkpoint carries beyond the eval weights: the codebook's EMA statistics `embed_avg` and
`cluster_size` and its `initted` flag (vector_quantize_pytorch.py:243-262), and weight-norm
parameters in both spellings (`parametrizations.weight.original0/1` and the legacy
`weight_g/weight_v`)."""
from __future__ import annotations

import numpy as np
import torch

from distilcodec_nabeel_amd import weights

G_NEW, V_NEW = ".parametrizations.weight.original0", ".parametrizations.weight.original1"


def reference_checkpoint(cfg: dict, seed: int) -> dict:
    enc = weights.synthetic_encoder(cfg, seed)
    q = weights.synthetic_quantizer(cfg, seed)
    gen = weights.synthetic_generator(cfg, seed)
    cb = "grvq.rvqs.0.layers.0._codebook."
    rng = np.random.default_rng(seed)
    q[cb + "embed_avg"] = (q[cb + "embed"] * 0.5).astype(np.float32)
    q[cb + "cluster_size"] = rng.random((1, q[cb + "embed"].shape[1]), dtype=np.float32)
    legacy = {}
    prefixes = sorted(k[: -len(G_NEW)] for k in gen if k.endswith(G_NEW))
    for i, p in enumerate(prefixes):
        if i % 2 == 0:  # every other conv in the legacy weight_g / weight_v spelling
            legacy[p + ".weight_g"] = gen.pop(p + G_NEW)
            legacy[p + ".weight_v"] = gen.pop(p + V_NEW)
    gen.update(legacy)
    t = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in d.items()}  # noqa: E731
    return {"generator": t(gen), "encoder": t(enc), "quantizer": t(q)}
