#!/usr/bin/env python3
"""Per-segment cycle breakdown of conv_gemm_x3dq's ping-pong main loop (library built with
-DDCX_SEG_DIAG, exporting dcx_diag_seg; select it with DCX_LIB=...), on the ResBlock convs of the
wide generator stages in h3 arithmetic (DCX_H3=1).

    DCX_LIB=$PWD/distilcodec_nabeel_amd/libdcx_seg.so python tools/seg_diag_h3.py [--stages 0,1,2]

Per K32 step and per wave (group 0 / group 1): cycles issuing the MFMAs, waiting at the barrier
after them, in the memory segment (DMA issue, fragment reads, the counted DMA wait; the first two
also shown apart), and waiting at the barrier after it.  Averages over every tile of every conv of the stage's ParallelBlock.
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native, config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="0,1,2")
    ap.add_argument("--rows", type=int, default=19200, help="rows (B * L) of the stage input")
    ap.add_argument("--blocks", default="", help="encoder ConvNeXt blocks instead (conv_gemm_x3dm), e.g. 0.0,2.0")
    ap.add_argument("--no-diag", action="store_true", help="run the modules only (any library; PMC passes)")
    ap.add_argument("--per-wave", action="store_true", help="conv_gemm_x3dw: every wave's sums (dcx_diag_seg8)")
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1), "cuda:0", gemm="x6")
    eng.set_knob("DCX_H3", 1)
    f = None
    if not a.no_diag:
        f = _native.lib().dcx_diag_seg
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    jobs = []
    if a.blocks:
        for blk in a.blocks.split(","):
            C = cfg["encoder"]["dims"][int(blk.split(".")[0])]
            jobs.append((f"encoder.stages.{blk}", C))
    else:
        for st in [int(s) for s in a.stages.split(",")]:
            jobs.append((f"generator.resblocks.{st}", cfg["decoder"]["upsample_initial_channel"] >> (st + 1)))
    for mod, C in jobs:
        x = torch.randn(4, a.rows // 4, C, device="cuda")
        eng.module(mod, x)
        torch.cuda.synchronize()
        if f is None:
            for _ in range(3):
                eng.module(mod, x)
            torch.cuda.synchronize()
            print(f"{mod} (C = {C}) done", flush=True)
            continue
        out = (ctypes.c_ulonglong * 13)()
        f(out, 1)
        for _ in range(3):
            eng.module(mod, x)
        torch.cuda.synchronize()
        f(out, 1)
        if a.per_wave:
            g8 = _native.lib().dcx_diag_seg8
            g8.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
            o8 = (ctypes.c_ulonglong * 49)()
            g8(o8, 1)
            for _ in range(3):
                eng.module(mod, x)
            torch.cuda.synchronize()
            g8(o8, 1)
            n8 = max(o8[48], 1)
            for w in range(8):
                v = [o8[w * 6 + i] / n8 for i in range(6)]
                print(f"{mod} wave {w}: " + "  ".join(f"{v[i]:6.0f}" for i in range(6)), flush=True)
        n = max(out[12], 1)
        v = [out[i] / n for i in range(12)]
        lab = ["mfma", "wait", "mem", "wait", "(dma issue", "reads"]
        for g in range(2):
            print(f"{mod} (C = {C}) g{g}: " + "  ".join(f"{lab[i]} {v[6 * g + i]:6.0f}" for i in range(6))
                  + f")  | step {sum(v[6 * g:6 * g + 4]):6.0f}", flush=True)


if __name__ == "__main__":
    main()
