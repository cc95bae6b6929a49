#!/usr/bin/env python3
"""In-loop clock and cycles per K16 step of the conv GEMM main loop (needs a library built with
-DDCX_CLOCK_DIAG, which exports dcx_diag_clock; select it with DCX_LIB=...).

    DCX_LIB=$PWD/libdcx_clk.so python tools/clk_diag.py [--shapes res512_k11d5,...]

s_memtime / s_memrealtime (100 MHz) bracket each workgroup's main loop, so the ratio is the shader
clock while MFMAs run; cycles/step are per workgroup.  The ideal for conv_gemm_x6pp (and the 8-wave
x6w8) is 2 waves per SIMD x 24 MFMA x 32 cycles = 1536 cycles per step.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeConv  # noqa: E402

T = 937
SHAPES = {"res512_k3": (512, 512, 3, 1, 32, 8 * T), "res512_k11d5": (512, 512, 11, 5, 32, 8 * T),
          "res256_k7d3": (256, 256, 7, 3, 32, 32 * T), "pw_1024": (1024, 4096, 1, 1, 1, 32 * T),
          "res64_k7d3": (64, 64, 7, 3, 32, 128 * T), "res64_k3d1": (64, 64, 3, 1, 32, 128 * T),
          "res128_k11": (128, 128, 11, 1, 32, 64 * T), "res128_k3": (128, 128, 3, 1, 32, 64 * T),
          "res64_k11d5": (64, 64, 11, 5, 32, 128 * T), "res32_k3d1": (32, 32, 3, 1, 32, 256 * T),
          "res32_k11d5": (32, 32, 11, 5, 32, 256 * T)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--gemm", default="x6", choices=["x6", "bf16"])
    a = ap.parse_args()
    f = _native.lib().dcx_diag_clock
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    for name in a.shapes.split(","):
        cin, cout, k, d, B, Lr = SHAPES[name]
        r = np.random.default_rng(0)
        w = (r.standard_normal((cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
        conv = NativeConv(w, np.zeros(cout, np.float32), dilation=d)
        x = torch.randn(B, Lr, cin, device="cuda")
        for _ in range(5):
            conv(x, gemm=a.gemm)
        torch.cuda.synchronize()
        out = (ctypes.c_ulonglong * 3)()
        f(out, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            conv(x, gemm=a.gemm)
        e1.record()
        torch.cuda.synchronize()
        f(out, 1)
        ms = e0.elapsed_time(e1) / a.reps
        mt, rt, steps = out[0], out[1], out[2]
        cyc = mt / max(steps, 1)
        clk = mt / max(rt, 1) * 100e6
        # loop share: workgroup-cycles inside the main loop per CU over the kernel's wall cycles
        # (can exceed 1 when two workgroups share a CU)
        share = mt / 256 / max(ms * 1e-3 * a.reps * clk, 1)
        print(f"{name:14s} {ms:8.3f} ms  in-loop clock {clk / 1e6:5.0f} MHz  "
              f"cycles/step {cyc:6.0f}  MFMA eff {1536 / cyc:.3f}  loop share {share:.2f}", flush=True)


if __name__ == "__main__":
    main()
