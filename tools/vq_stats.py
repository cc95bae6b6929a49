#!/usr/bin/env python3
"""VQ search diagnostics on the C2 (x6) or C3 (bf16) workload: rows rescored, codes rescored and the
per-kernel time of the search (prefilter, certify, pair eval, reduce).  Environment knobs
(DCX_VQ_PAIRS_PER_ROW ...) apply as at dcx_create.  Usage: python tools/vq_stats.py [--gemm x6|bf16]
[--batch 32]"""
import argparse
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from distilcodec_nabeel_amd import config, synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gemm", default="x6")
ap.add_argument("--batch", type=int, default=32)
a = ap.parse_args()
cfg = config.default_config()
state = weights.synthetic_state_dict(cfg, seed=1234)
n = 240000
audio = torch.zeros(a.batch, n + 1)
for i, c in enumerate(synth.clips(a.batch, n, seed=0, kind="mix")):
    audio[i, 1:] = torch.from_numpy(c)
audio = audio.cuda()
eng = NativeCodec(cfg, {"encoder": state["encoder"], "quantizer": state["quantizer"]}, "cuda:0",
                  with_generator=False, gemm=a.gemm)
feat = eng.encode(eng.mel(audio))
eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)
torch.cuda.synchronize()
eng.vq_rescore_stats(reset=True)
eng.profile(True)
eng.profile_reset()
codes = eng.vq_encode(feat, want_pjt_in=False, want_fup=False, want_quantized=False)[0]
torch.cuda.synchronize()
kern = eng.profile_read()
eng.profile(False)
rows, nc = eng.vq_rescore_stats()
M = codes.numel()
out = {"gemm": a.gemm, "rows": M, "rows_rescored": rows, "frac_rescored": round(rows / M, 4),
       "codes_rescored": nc, "codes_per_rescored_row": round(nc / max(rows, 1), 2),
       "pairs_per_row_env": os.environ.get("DCX_VQ_PAIRS_PER_ROW"),
       "ms": {k: round(v["ms"], 3) for k, v in kern.items() if k.startswith("vq") or k == "row_sqnorm"}}
print(json.dumps(out))
