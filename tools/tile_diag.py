#!/usr/bin/env python3
"""Per-tile timeline of conv_gemm_x6dq launches (needs a library built with -DDCX_TILE_DIAG, which
exports dcx_diag_tiles; select it with DCX_LIB=...).

    DCX_LIB=$PWD/distilcodec_nabeel_amd/libdcx_tile.so python tools/tile_diag.py [--shapes ...]

Each workgroup stamps s_memrealtime (100 MHz) at entry, main-loop start, main-loop end and exit,
with its CU's HW_ID / XCC_ID.  Printed: median prologue / loop / epilogue times, the median gap
between consecutive tiles on one CU, and the share of CU time spent inside main loops.
"""
import argparse
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeConv  # noqa: E402

T = 937
SHAPES = {"res512_k3": (512, 512, 3, 1, 32, 8 * T), "res512_k11d5": (512, 512, 11, 5, 32, 8 * T),
          "res256_k7d3": (256, 256, 7, 3, 32, 32 * T), "res128_k3": (128, 128, 3, 1, 32, 64 * T),
          # one round on 120 / 240 of the 256 CUs: the epilogue without the other CUs' bursts
          "res512_k3_b2": (512, 512, 3, 1, 2, 8 * T), "res512_k3_b4": (512, 512, 3, 1, 4, 8 * T)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    f = _native.lib().dcx_diag_tiles
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    nmax = 16384
    buf = (ctypes.c_ulonglong * (6 * nmax))()
    for name in a.shapes.split(","):
        cin, cout, k, d, B, L = SHAPES[name]
        r = np.random.default_rng(0)
        w = (r.standard_normal((cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
        conv = NativeConv(w, np.zeros(cout, np.float32), dilation=d)
        x = torch.randn(B, L, cin, device="cuda")
        res = torch.randn(B, L, cout, device="cuda")
        for epi, label in ((0, "plain"), (3, "residual+silu")):
            kw = dict(epi=3, res=res, want_silu=True) if epi == 3 else {}
            for _ in range(3):
                conv(x, gemm="x6", **kw)
            torch.cuda.synchronize()
            f(buf, nmax, 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            conv(x, gemm="x6", **kw)
            e1.record()
            torch.cuda.synchronize()
            n = f(buf, nmax, 1)
            if n <= 0:
                print(f"{name} {label}: no tiles recorded (x6dq not used for this shape?)")
                continue
            t = np.ctypeslib.as_array(buf)[: 6 * n].reshape(n, 6).astype(np.int64)
            us = lambda v: v / 100.0  # noqa: E731  100 MHz ticks -> us
            pro, loop, epi_t = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
            span = t[:, 3].max() - t[:, 0].min()
            cus = defaultdict(list)
            for row in t:
                cus[(int(row[5]), (int(row[4]) >> 8) & 0xFF)].append(row)
            gaps = []
            for rows in cus.values():
                rows.sort(key=lambda z: z[0])
                gaps += [rows[i + 1][0] - rows[i][3] for i in range(len(rows) - 1)]
            share = loop.sum() / (len(cus) * span)
            print(f"{name:13s} {label:14s} {e0.elapsed_time(e1):7.3f} ms  tiles {n:5d} on {len(cus):3d} CUs  "
                  f"prologue {us(np.median(pro)):6.1f} us  loop {us(np.median(loop)):7.1f} us  "
                  f"epilogue {us(np.median(epi_t)):6.1f} us  gap {us(np.median(gaps)) if gaps else 0:5.1f} us  "
                  f"loop share {share:.3f}", flush=True)


if __name__ == "__main__":
    main()
