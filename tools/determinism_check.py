#!/usr/bin/env python3
"""Run-to-run determinism of encode -> decode at the C2 shape under several kernel switches:
for each knob set, one reference run and N more, counting waveforms / codes that differ bit-wise
(a race shows up as an occasional difference).  python tools/determinism_check.py [--runs 6]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

CONFIGS = [
    {},
    {"DCX_H3_SPLIT": 0},
    {"DCX_H3_PAIRS": 0},
    {"DCX_H3_SPLIT": 0, "DCX_H3_PAIRS": 0},
    {"DCX_H3": 0, "DCX_H3_1X1": 0, "DCX_H3_PAIRS": 0},
    {"DCX_ENC_STREAMS": 0},  # the half-batch streams (round 6): one stream, and the generator per half too
    {"DCX_ENC_STREAMS": 3},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--clips", type=int, default=32)
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0", gemm="x6")
    clips = synth.clips(a.clips, 240000, seed=0, kind="mix")
    audio = torch.zeros(a.clips, 240001)
    for i, c in enumerate(clips):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.cuda()
    for kn in CONFIGS:
        with eng.knobs(**kn):
            c0, w0 = eng.encode_decode(audio)
            bad_w = bad_c = 0
            worst = []
            for _ in range(a.runs):
                c, w = eng.encode_decode(audio)
                if not torch.equal(c, c0):
                    bad_c += 1
                if not torch.equal(w, w0):
                    bad_w += 1
                    d = (w - w0).abs().reshape(a.clips, -1).amax(1)
                    worst.append(int(torch.argmax(d)))
        print(f"{kn}: {bad_w} / {a.runs} waveforms and {bad_c} / {a.runs} code sets differ from the first run"
              + (f"; clips {worst}" if worst else ""), flush=True)


if __name__ == "__main__":
    main()
