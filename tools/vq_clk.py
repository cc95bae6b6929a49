#!/usr/bin/env python3
"""In-loop clock and cycles per K32 step of the VQ prefilter (library built with -DDCX_CLOCK_DIAG;
select it with DCX_LIB=...).  Runs only the VQ encode stage on random features (32 x 937 frames)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native, config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

f = _native.lib().dcx_diag_clock
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
cfg = config.default_config()
eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0")
feat = torch.randn(32, 937, cfg["encoder"]["dims"][-1], device="cuda")
for _ in range(2):
    eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 3)()
f(out, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)
e1.record()
torch.cuda.synchronize()
f(out, 1)
mt, rt, steps = out[0], out[1], out[2]
cyc = mt / max(steps, 1)
print(f"vq_encode {e0.elapsed_time(e1) / 5:8.3f} ms  in-loop clock {mt / max(rt, 1) * 100.0:5.0f} MHz  "
      f"cycles/step {cyc:6.0f}  MFMA eff {1536 / cyc:.3f}  (includes the 1x1 convs' loops)")
