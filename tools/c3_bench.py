#!/usr/bin/env python3
"""C3 (BASELINE.json configs[2]): encoder + GRFVQ token extraction only, 256 x 10 s, bf16, 1 GPU.

    python tools/c3_bench.py [--batch 256] [--steps 3] [--warmup 1] [--gemm bf16,x6] [--kernels PREFIX]

Per GEMM mode, one JSON line: samples/s of mel -> encoder -> VQ codes (x_pjt_in and the other
feature outputs not returned), inputs resident in HBM, HIP events around the timed steps, plus
the per-kernel device time. Algorithmic work: 415.36 MFLOP per frame. bf16 mode
is the reference's enable_bfloat16; its VQ search still returns the exact nearest code of the
bf16-valued x_pjt_in (prefilter + fp64 rescore). Synthetic clips, seeded synthetic weights.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

ENC_MFLOP_PER_FRAME = 415.36


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gemm", default="bf16,x6")
    ap.add_argument("--kernels", default=None, help="write per-kernel tables to PREFIX_<mode>.json")
    a = ap.parse_args()
    cfg = config.default_config()
    state = weights.synthetic_state_dict(cfg, seed=1234, with_generator=False)
    n = int(a.seconds * 24000)
    audio = torch.zeros(a.batch, n + 1)
    for i, c in enumerate(synth.clips(a.batch, n, seed=0, kind="mix")):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    eng = NativeCodec(cfg, state, "cuda:0", with_generator=False)
    T = eng.num_frames(n + 1)
    codes_ref = None
    for mode in a.gemm.split(","):
        eng.set_gemm(mode)

        def step():
            feat = eng.encode(eng.mel(audio))
            return eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)[0]

        for _ in range(a.warmup):
            codes = step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            codes = step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        # per-kernel HIP-event timing of one more step: the dominant kernel against its MFMA ceiling
        # (products per fp32-equivalent FLOP: 1 for bf16 GEMMs and vq_prefilter_b1, 2 for vq_prefilter_bq, 6 in x6,
        # 3 for the h3 kernels conv_gemm_x3*, fp16 products at the bf16 MFMA rate)
        with eng.knobs(DCX_ENC_STREAMS=0):  # launches in isolation (the timed steps overlap two half-batches)
            eng.profile(True)
            eng.profile_reset()
            step()
            kern = eng.profile_read()
            eng.profile(False)
        if a.kernels:
            json.dump({"steps": 1, "kernels": kern}, open(f"{a.kernels}_{mode}.json", "w"), indent=1)
        name, rec = max(kern.items(), key=lambda kv: kv[1]["ms"])
        prods = (1 if "prefilter_b1" in name else 2 if "prefilter_bk" in name or "prefilter_bq" in name or "_x2" in name
                 else 3 if "prefilter" in name or "_x3" in name else 1 if "bf16" in name else 6)
        ach = rec["flops"] / (rec["ms"] * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": name, "achieved": round(ach, 1), "peak": round(2500.0 / prods, 1),
                "unit": "TFLOP/s (fp32-equivalent)", "frac": round(ach * prods / 2500.0, 4),
                "peak_basis": f"dense bf16 / fp16 MFMA 2500 TF / {prods} product(s) per fp32-equivalent product",
                "share_of_device_time": round(rec["ms"] / sum(v["ms"] for v in kern.values()), 4)}
        agree = None
        if codes_ref is None:
            codes_ref = codes.clone()
        else:
            agree = round(float((codes == codes_ref).double().mean()), 5)
        flops = ENC_MFLOP_PER_FRAME * 1e6 * a.batch * T
        print(json.dumps({
            "config": "C3: encoder + GRFVQ token extraction, %d x %g s" % (a.batch, a.seconds), "gemm": mode,
            "value": round(a.batch * n / (ms * 1e-3), 1), "unit": "samples/s", "ms_per_step": round(ms, 3),
            "tflops_algorithmic": round(flops / (ms * 1e-3) / 1e12, 1), "frames": a.batch * T,
            "codes_agree_with_first_mode": agree, "roofline": roof,
            "data": "synthetic speech/music-like clips, seeded synthetic weights"}), flush=True)
        del codes
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
