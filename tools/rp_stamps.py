"""Per-phase clock breakdown of conv_res_pair from a -DRP_DIAG_STAMPS build (DCX_LIB=...rp_stamps.so):
wave 0 of every workgroup, shader clocks summed per phase, reported per member-tile and per step."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, weights, _native  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

cfg = config.default_config()
eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0", gemm="x6")
z = (torch.randn(32, 937, 1024, generator=torch.Generator().manual_seed(0)) * 0.5).cuda()
L = _native.lib()
buf = (ctypes.c_ulonglong * 32)()
eng.generate(z)
torch.cuda.synchronize()
L.dcx_diag_rp(buf, 1)
for _ in range(2):
    eng.generate(z)
torch.cuda.synchronize()
L.dcx_diag_rp(buf, 1)
names = ["c1 steps", "T image", "c2 steps", "epilogue", "next S image"]
for ci, C in enumerate((32, 64)):
    v = list(buf)[ci * 16:(ci + 1) * 16]
    n, s1, s2 = v[5], v[6], v[7]
    tot = sum(v[:5])
    print(f"C = {C}: {n} member-tiles (wave 0 of each workgroup), {tot / n:.0f} cycles per member-tile")
    for i, nm in enumerate(names):
        extra = ""
        if i == 0:
            extra = f"  {v[0] / s1:.0f} per step (MFMA phase {v[8] / s1:.0f}, wait + barrier {v[9] / s1:.0f})"
        if i == 2:
            extra = f"  {v[2] / s2:.0f} per step"
        print(f"   {nm:14s} {v[i] / n:8.0f} cycles ({v[i] / tot:5.1%}){extra}")
