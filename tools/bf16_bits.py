"""Print a digest of the bf16-mode encoder features, x_pjt_in and codes for a fixed synthetic batch,
so two builds (DCX_LIB=...) can be compared bit for bit.  Usage: python tools/bf16_bits.py [B] [secs]"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distilcodec_nabeel_amd import config, synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
cfg = config.default_config()
st = weights.synthetic_state_dict(cfg, seed=1234)
eng = NativeCodec(cfg, {"encoder": st["encoder"], "quantizer": st["quantizer"]}, "cuda:0", with_generator=False, gemm="bf16")
n = int(24000 * secs)
audio = torch.zeros(B, n + 1)
for i, c in enumerate(synth.clips(B, n, seed=3, kind="mix")):
    audio[i, 1:] = torch.from_numpy(c)
feat = eng.encode(eng.mel(audio.cuda()))
codes, pin, _, _ = eng.vq_encode(feat, want_fup=False, want_quantized=False)
torch.cuda.synchronize()
for name, t in (("feat", feat), ("x_pjt_in", pin), ("codes", codes)):
    print(name, hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:16])
