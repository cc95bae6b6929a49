#!/usr/bin/env python3
"""Per-segment cycle breakdown of vq_prefilter_b1's ping-pong main loop (library built with
-DDCX_SEG_DIAG, exporting dcx_diag_seg; select it with DCX_LIB=...).

    DCX_LIB=$PWD/distilcodec_nabeel_amd/seg.so python tools/seg_diag_vq.py [--rows 65536]

Runs the module "quantizer.search" (x6 mode: the same prefilter kernel as the bf16 mode's, on
compact x_pjt_in) on random rows, so no other kernel with segment stamps runs.  Per K32 step and per
wave (wave 0 of group 0, wave 4 of group 1, summed over workgroups and divided by steps x
workgroups): shader cycles of MFMA issue, the barrier after it, fragment reads + DMA issue, the DMA
wait, and the barrier after the memory segment.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native, config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234, with_generator=False), "cuda:0",
                      with_generator=False)
    f = _native.lib().dcx_diag_seg
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    cin = eng.module_io("quantizer.search")[0]
    x = torch.randn(1, a.rows, cin, device="cuda") * 0.05
    eng.module("quantizer.search", x)
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 13)()
    f(out, 1)
    for _ in range(a.reps):
        eng.module("quantizer.search", x)
    torch.cuda.synchronize()
    f(out, 1)
    st = max(out[12], 1)
    lab = ["mfma", "bar", "reads+dma", "dma_wait", "bar"]
    for g in range(2):
        v = [out[6 * g + i] / st for i in range(5)]
        print(f"vq_prefilter_b1 rows {a.rows} g{g}: " + "  ".join(f"{lab[i]} {v[i]:6.0f}" for i in range(5))
              + f"  | step {sum(v):6.0f} cycles (32 MFMAs x 16 = 512 per wave)", flush=True)


if __name__ == "__main__":
    main()
