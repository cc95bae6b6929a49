#!/usr/bin/env python3
"""Throughput of the GPU resampler (dcx_resample_poly) on C2-sized inputs: 32 clips x 10 s at
common rates -> 24 kHz.  HBM roofline: 4 * (n_in + n_out) bytes per clip (read once, written once).

    python tools/resample_bench.py [--rates 16000,44100,48000] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import resample  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="8000,16000,22050,44100,48000")
    ap.add_argument("--clips", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for sr in map(int, a.rates.split(",")):
        x = torch.randn(a.clips, int(sr * a.seconds), device="cuda") * 0.1
        for _ in range(3):
            y = resample.resample(x, sr, 24000)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            y = resample.resample(x, sr, 24000)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        up, down = resample.ratio(sr, 24000)
        h, _ = resample.design(up, down)
        nbytes = 4.0 * (x.numel() + y.numel())
        print(json.dumps({"sr_in": sr, "sr_out": 24000, "clips": a.clips, "seconds": a.seconds, "ms": round(ms, 4),
                          "in_samples_per_s": round(x.numel() / (ms * 1e-3)), "taps_per_output": round(len(h) / up, 1),
                          "hbm_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1),
                          "note": "wall time of resample.resample incl. its output allocation"}), flush=True)


if __name__ == "__main__":
    main()
