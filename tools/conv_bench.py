#!/usr/bin/env python3
"""Microbenchmark of the conv kernel family on the generator's shapes (C2 sizes, both modes)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd.engine import NativeConv  # noqa: E402

T = 937
SHAPES = {  # name: (cin, cout, k, dil, transposed, stride, B, L)
    "res512_k3": (512, 512, 3, 1, False, 1, 32, 8 * T),
    "res512_k11d5": (512, 512, 11, 5, False, 1, 32, 8 * T),
    "res256_k7d3": (256, 256, 7, 3, False, 1, 32, 32 * T),
    "res128_k11": (128, 128, 11, 1, False, 1, 32, 64 * T),
    "res128_k3": (128, 128, 3, 1, False, 1, 32, 64 * T),
    "res64_k7d3": (64, 64, 7, 3, False, 1, 32, 128 * T),
    "res32_k11d5": (32, 32, 11, 5, False, 1, 32, 256 * T),
    "res32_k7d3": (32, 32, 7, 3, False, 1, 32, 256 * T),
    "res32_k3d1": (32, 32, 3, 1, False, 1, 32, 256 * T),
    "res64_k3d1": (64, 64, 3, 1, False, 1, 32, 128 * T),
    "res64_k11d5": (64, 64, 11, 5, False, 1, 32, 128 * T),
    "ups0": (1024, 512, 16, 1, True, 8, 32, T),
    "pw1_1024": (1024, 4096, 1, 1, False, 1, 1, 32 * T),
    "pw2_1024": (4096, 1024, 1, 1, False, 1, 1, 32 * T),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--modes", default="x6,f32")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--data", default="randn", choices=["randn", "zero", "bf16"],
                    help="input values: randn, all zeros, or randn rounded to bf16 (mid/lo planes zero)")
    a = ap.parse_args()
    out = {}
    for name in a.shapes.split(","):
        cin, cout, k, d, tr, s, B, L = SHAPES[name]
        r = np.random.default_rng(0)
        w = (r.standard_normal((cin, cout, k) if tr else (cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
        conv = NativeConv(w, np.zeros(cout, np.float32), dilation=d, transposed=tr, stride=s)
        x = torch.randn(B, L, cin, device="cuda")
        if a.data == "zero":
            x.zero_()
        elif a.data == "bf16":
            x = x.bfloat16().float()
        flops = 2.0 * B * L * (s if tr else 1) * cout * cin * (k // s if tr else k)
        for mode in a.modes.split(","):
            y = conv(x, gemm=mode)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                conv(x, gemm=mode)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            out[f"{name}/{mode}"] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
            print(f"{name:14s} {mode:4s} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TF/s", flush=True)
            del y
    if os.environ.get("CONV_BENCH_JSON"):
        json.dump(out, open(os.environ["CONV_BENCH_JSON"], "w"), indent=1)


if __name__ == "__main__":
    main()
