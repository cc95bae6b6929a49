#!/usr/bin/env python3
"""Measured accuracy of the bf16 GEMM mode (the reference's enable_bfloat16) vs the fp32 reference
fixtures: conv primitive error vs a bf16-operand fp64 reference, code agreement, decode SNR.

    python tools/bf16_report.py            (needs a GPU)
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from distilcodec_nabeel_amd import config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec, NativeConv  # noqa: E402


def bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def snr(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return float(10 * np.log10((ref ** 2).sum() / max(((x - ref) ** 2).sum(), 1e-300)))


def main():
    r = np.random.default_rng(0)
    for cin, cout, k, d, L in [(512, 512, 11, 5, 300), (1024, 4096, 1, 1, 190), (64, 64, 7, 3, 700), (32, 32, 3, 1, 500)]:
        w = (r.standard_normal((cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
        b = (0.1 * r.standard_normal(cout)).astype(np.float32)
        x = r.standard_normal((2, L, cin)).astype(np.float32)
        conv = NativeConv(w, b, dilation=d)
        y = conv(torch.from_numpy(x).cuda(), gemm="bf16")
        ref = F.conv1d(bf(torch.from_numpy(x).double()).transpose(1, 2), bf(torch.from_numpy(w).double()),
                       torch.from_numpy(b).double(), dilation=d, padding=d * (k - 1) // 2).transpose(1, 2)
        refb = bf(ref.float()).double()
        e = (y.cpu().double() - refb).abs()
        print(f"conv {cin}->{cout} k{k} d{d}: max|y-bf16(ref)|/max|ref| {float(e.max() / ref.abs().max()):.2e}, "
              f"frac elements != bf16(ref) {float((e > 0).double().mean()):.4f}")
    cfg = config.default_config()
    state = weights.synthetic_state_dict(cfg, seed=1234)
    eng = NativeCodec(cfg, state, "cuda:0", gemm="bf16")
    for name in ("e2e_batch", "e2e_3s", "e2e_real"):
        g = dict(np.load(os.path.join(HERE, "tests", "golden", f"{name}.npz")))
        mel = eng.mel(torch.from_numpy(g["audio"]))
        feat = eng.encode(mel)
        codes, pin, _, _ = eng.vq_encode(feat)
        match = float((codes.cpu().numpy() == g["codes"]).mean())
        wav = eng.generate(eng.vq_decode(torch.from_numpy(g["codes"]))).cpu().numpy()
        print(f"{name}: codes == fp32 reference {match:.4f} ({codes.numel()} frames); "
              f"decode of reference codes SNR vs fp32 reference {snr(wav, g['wav']):.1f} dB")


if __name__ == "__main__":
    main()
