"""Checkpoint ingestion end to end on the GPU: a reference-format
checkpoint (distil_codec.py:480-492; legacy weight_g/_v keys, codebook EMA statistics) saved with
torch.save and loaded by `from_pretrained` (:77-97) gives bit-for-bit the codec that
`DistilCodec(cfg)` + `load_state_dict` of the same tensors gives.  With `use_generator=False` the
generator keeps its initial weights, as in the reference."""
import json

import numpy as np
import pytest
import torch
from ckpt_util import reference_checkpoint

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def files(cfg, tmp_path_factory):
    d = tmp_path_factory.mktemp("ckpt")
    cfg_path, ck_path = d / "model_config.json", d / "g_00204000"
    cfg_path.write_text(json.dumps(cfg))
    ck = reference_checkpoint(cfg, seed=77)
    torch.save(ck, ck_path)
    return str(cfg_path), str(ck_path), ck


def _run(codec, audio):
    codes, wav = codec._engine().encode_decode(audio)
    torch.cuda.synchronize()
    return codes.cpu(), wav.cpu()


def test_from_pretrained_equals_load_state_dict(cfg, files):
    from distilcodec_nabeel_amd import DistilCodec, synth

    cfg_path, ck_path, ck = files
    audio = torch.zeros(2, 24001)
    for i, c in enumerate(synth.clips(2, 24000, seed=41, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()

    a = DistilCodec.from_pretrained(cfg_path, ck_path, use_generator=True)
    assert a._engine().device == torch.device("cuda:0")
    ca, wa = _run(a, audio)
    del a
    b = DistilCodec(cfg)
    b.load_state_dict({k: ck[k] for k in ("encoder", "quantizer", "generator")})
    cb, wb = _run(b, audio)
    del b
    assert torch.equal(ca, cb) and torch.equal(wa, wb)

    c = DistilCodec.from_pretrained(cfg_path, ck_path, use_generator=False)
    cc, wc = _run(c, audio)
    del c
    d = DistilCodec(cfg)  # initial generator weights (synthetic, seed 1234)
    d.load_state_dict({k: ck[k] for k in ("encoder", "quantizer")})
    cd, wd = _run(d, audio)
    del d
    assert torch.equal(cc, cd) and torch.equal(wc, wd)
    # encoder + quantizer came from the file in both loads: identical codes; the generators differ
    assert torch.equal(ca, cc)
    assert not torch.equal(wa, wc)
    assert float(wa.abs().max()) > 0 and bool(torch.isfinite(wa).all())
