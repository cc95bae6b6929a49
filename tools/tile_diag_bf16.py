#!/usr/bin/env python3
"""Per-tile timeline of the bf16-mode 1x1 convs (conv_gemm_bf16dm) inside one ConvNeXt block of the
C3 encoder (dcx_module_forward), from a -DDCX_TILE_DIAG build selected with DCX_LIB=...: median
prologue / main loop / epilogue per tile, the gap between consecutive tiles on a CU, the share of CU
time inside main loops, per launch (told apart by their K32 step counts)."""
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
    ap.add_argument("--stages", default="0,3")
    ap.add_argument("--batch", type=int, default=0, help="clips (0: 256 for stage 0, 64 for stage 3)")
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234, with_generator=False), "cuda:0",
                      with_generator=False, gemm="bf16")
    f = _native.lib().dcx_diag_tiles
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    nmax = 16384
    buf = (ctypes.c_ulonglong * (6 * nmax))()
    for st in map(int, a.stages.split(",")):
        C = cfg["encoder"]["dims"][st]
        B = a.batch or (256 if st == 0 else 64)
        x = torch.randn(B, 937, C, device="cuda") * 0.5
        for _ in range(2):
            eng.module(f"encoder.stages.{st}.0", x)
        torch.cuda.synchronize()
        f(buf, nmax, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.module(f"encoder.stages.{st}.0", x)
        e1.record()
        torch.cuda.synchronize()
        n = f(buf, nmax, 1)
        t = np.ctypeslib.as_array(buf)[: 6 * n].reshape(n, 6).astype(np.int64)
        print(f"stage {st} (C = {C}, {B} clips): block {e0.elapsed_time(e1):.3f} ms, {n} tiles recorded")
        for steps in sorted(set((t[:, 5] >> 16).tolist())):
            s = t[(t[:, 5] >> 16) == steps]
            us = lambda v: v / 100.0  # noqa: E731
            pro, loop, epi = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
            span = s[:, 3].max() - s[:, 0].min()
            cus = defaultdict(list)
            for row in s:
                cus[(int(row[5]) & 0xFFFF, (int(row[4]) >> 8) & 0xFF)].append(row)
            gaps = []
            for rows in cus.values():
                rows.sort(key=lambda z: z[0])
                gaps += [rows[i + 1][0] - rows[i][3] for i in range(len(rows) - 1)]
            print(f"  K32 steps {steps:4d}: {len(s):5d} tiles on {len(cus):3d} CUs, launch span {us(span):8.1f} us, "
                  f"prologue {us(np.median(pro)):5.1f} loop {us(np.median(loop)):6.1f} ({us(np.median(loop)) / steps:.3f}/step) "
                  f"epilogue {us(np.median(epi)):5.1f} gap {us(np.median(gaps)) if gaps else 0:4.1f} us, "
                  f"loop share {loop.sum() / (len(cus) * span):.3f}", flush=True)


if __name__ == "__main__":
    main()
