#!/usr/bin/env python3
"""Per-segment cycle breakdown of conv_gemm_x6pp's ping-pong main loop (library built with
-DDCX_SEG_DIAG -DDCX_NO_DMA, exporting dcx_diag_seg; select it with DCX_LIB=...).

    DCX_LIB=$PWD/libdcx_seg.so python tools/seg_diag.py [--shapes res512_k11d5,...]

Per K16 step and per wave (wave 0 of group 0, wave 4 of group 1): cycles to issue the MFMAs, the
fragment reads, the LDS stores (including their wait for the loads), the loads and loop control,
and the two barrier waits.
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
from tools.clk_diag import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    f = _native.lib().dcx_diag_seg
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    for name in a.shapes.split(","):
        cin, cout, k, d, B, Lr = SHAPES[name]
        r = np.random.default_rng(0)
        w = (r.standard_normal((cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
        conv = NativeConv(w, np.zeros(cout, np.float32), dilation=d)
        x = torch.randn(B, Lr, cin, device="cuda")
        conv(x)
        torch.cuda.synchronize()
        out = (ctypes.c_ulonglong * 13)()
        f(out, 1)
        for _ in range(5):
            conv(x)
        torch.cuda.synchronize()
        f(out, 1)
        st = max(out[12], 1)
        v = [out[i] / st for i in range(12)]
        lab = (["mfma", "wait", "mem", "wait", "-", "-"] if os.environ.get("DCX_SEG_DQ")
               else ["mfma", "wait", "reads", "stores", "loads", "wait"])
        for g in range(2):
            print(f"{name:14s} g{g}: " + "  ".join(f"{lab[i]} {v[6 * g + i]:5.0f}" for i in range(6))
                  + f"  | step {sum(v[6 * g:6 * g + 6]):6.0f}", flush=True)


if __name__ == "__main__":
    main()
