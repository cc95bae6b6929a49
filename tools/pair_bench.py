"""The small-C ParallelBlocks alone (generator.resblocks.3 / .4: the fused pair kernels at C = 64 / 32) on
C2-sized synthetic inputs (32 clips x 10 s), for PMC passes and kernel A/B.  Knobs from the environment
(read at dcx_create).  Usage: python tools/pair_bench.py [--reps N] [--stage 3|4|both]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stage", default="both")
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    from distilcodec_nabeel_amd import config, weights
    from distilcodec_nabeel_amd.engine import NativeCodec

    cfg = config.default_config()
    st = weights.synthetic_state_dict(cfg, seed=1234)
    e = NativeCodec(cfg, st, "cuda:0", gemm="x6")
    frames = 937
    out = {}
    stages = [3, 4] if args.stage == "both" else [int(args.stage)]
    for s in stages:
        C = 1024 >> (s + 1)
        L = frames * 256 * 32 // C  # rows of stage s at 24 kHz: 128 T (C = 64), 256 T (C = 32)
        g = torch.Generator().manual_seed(s)
        x = (torch.randn(args.batch, L, C, generator=g) * 0.5).cuda()
        name = f"generator.resblocks.{s}"
        e.module(name, x)
        torch.cuda.synchronize()
        t = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            e.module(name, x)
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e3)
        out[name] = {"C": C, "L": L, "ms": sorted(t)[len(t) // 2]}
        del x
    print(json.dumps(out))


if __name__ == "__main__":
    main()
