#!/usr/bin/env python3
"""Per-tile timeline of vq_prefilter_b1 from a -DDCX_TILE_DIAG build (select with DCX_LIB=...): the
module "quantizer.search" (x6 mode, the same prefilter kernel as the bf16 mode's) on random rows;
median prologue (launch to the first steps' DMA landed), main loop, epilogue per tile, the gap
between consecutive tiles on a CU, and the share of CU time inside main loops.

    DCX_LIB=$PWD/distilcodec_nabeel_amd/tile.so python tools/tile_diag_vq.py [--rows 65536]
"""
import argparse
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import _native, config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234, with_generator=False), "cuda:0",
                      with_generator=False)
    f = _native.lib().dcx_diag_tiles
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    nmax = 16384
    buf = (ctypes.c_ulonglong * (6 * nmax))()
    cin = eng.module_io("quantizer.search")[0]
    x = torch.randn(1, a.rows, cin, device="cuda") * 0.05
    for _ in range(2):
        eng.module("quantizer.search", x)
    torch.cuda.synchronize()
    f(buf, nmax, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.module("quantizer.search", x)
    e1.record()
    torch.cuda.synchronize()
    n = f(buf, nmax, 1)
    t = np.ctypeslib.as_array(buf)[: 6 * n].reshape(n, 6).astype(np.int64)
    s = t[(t[:, 5] >> 16) >= 32]  # the prefilter's tiles (K32 steps = dim / 32)
    us = lambda v: v / 100.0  # noqa: E731  (s_memrealtime: 100 MHz)
    pro, loop, epi = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
    span = s[:, 3].max() - s[:, 0].min()
    cus = defaultdict(list)
    for row in s:
        cus[(int(row[5]) & 0xFFFF, (int(row[4]) >> 8) & 0xFF)].append(row)
    gaps = []
    for rows in cus.values():
        rows.sort(key=lambda z: z[0])
        gaps += [rows[i + 1][0] - rows[i][3] for i in range(len(rows) - 1)]
    steps = int(np.median(s[:, 5] >> 16))
    print(f"search {a.rows} rows: {e0.elapsed_time(e1):.3f} ms, {n} tiles recorded, {len(s)} prefilter tiles on "
          f"{len(cus)} CUs, span {us(span):.1f} us; per tile: prologue {us(np.median(pro)):.2f} us, loop "
          f"{us(np.median(loop)):.1f} us ({us(np.median(loop)) / steps * 1e3:.1f} ns/step, {steps} steps), epilogue "
          f"{us(np.median(epi)):.2f} us, gap {us(np.median(gaps)) if gaps else 0:.2f} us; loop share "
          f"{loop.sum() / (len(cus) * span):.3f}", flush=True)


if __name__ == "__main__":
    main()
