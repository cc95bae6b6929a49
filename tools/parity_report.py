#!/usr/bin/env python3
"""Print measured parity margins of the GPU path vs the reference fixtures, per GEMM mode.

    python tools/parity_report.py [--modes x6,f32] > profiles/rNN_parity.md      (needs a GPU)
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from distilcodec_nabeel_amd import config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def snr(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return float(10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="x6,f32")
    a = ap.parse_args()
    cfg = config.default_config()
    state = weights.synthetic_state_dict(cfg, seed=1234)
    gd = os.path.join(HERE, "tests", "golden")
    golden = {n: dict(np.load(os.path.join(gd, f"{n}.npz"))) for n in ("e2e_batch", "e2e_3s", "e2e_real")}
    print("| mode | fixture | mel max/mean abs | encoder rel | x_pjt_in rel | codes exact (e2e) | quantized rel | wav SNR dB (decode of ref codes) | wav SNR dB (e2e) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for mode in a.modes.split(","):
        eng = NativeCodec(cfg, state, "cuda:0", gemm=mode)
        for name, g in golden.items():
            mel = eng.mel(torch.from_numpy(g["audio"])).transpose(1, 2).cpu().numpy()
            d = np.abs(mel.astype(np.float64) - g["mel"])
            enc = pin = "-"
            if "feat" in g:
                feat = eng.encode(torch.from_numpy(g["mel"]).transpose(1, 2))
                enc = f"{rel(feat.transpose(1, 2).cpu(), g['feat']):.2e}"
                _, p, _, _ = eng.vq_encode(torch.from_numpy(g["feat"]).transpose(1, 2))
                pin = f"{rel(p[:1].cpu(), g['x_pjt_in']):.2e}"
            z = eng.vq_decode(torch.from_numpy(g["codes"]))
            qrel = rel(z.transpose(1, 2).cpu(), g["quantized"])
            wav = eng.generate(torch.from_numpy(g["quantized"]).transpose(1, 2)).cpu()
            codes, w2 = eng.encode_decode(torch.from_numpy(g["audio"]))
            match = float((codes.cpu().numpy() == g["codes"]).mean())
            e2e = f"{snr(w2.cpu(), g['wav']):.1f}" if match == 1.0 else "codes differ"
            print(f"| {mode} | {name} | {d.max():.2e} / {d.mean():.2e} | {enc} | {pin} | {match:.4f} | {qrel:.2e} | "
                  f"{snr(wav, g['wav']):.1f} | {e2e} |")
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
