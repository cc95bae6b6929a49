"""Generator-only timing loop (dcx_generate at C2 shape by default) for rocprofv3 passes.

    python tools/gen_bench.py --batch 32 --frames 937 --reps 3
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--frames", type=int, default=937)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--kernels", action="store_true", help="per-kernel device times (HIP events)")
a = ap.parse_args()
cfg = config.default_config()
eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0", gemm="x6")
z = (torch.randn(a.batch, a.frames, cfg["decoder"]["upsample_initial_channel"], generator=torch.Generator().manual_seed(0)) * 0.5).cuda()
eng.generate(z)
torch.cuda.synchronize()
t0 = time.time()
for _ in range(a.reps):
    eng.generate(z)
torch.cuda.synchronize()
print(f"generate {a.batch} x {a.frames} frames: {(time.time() - t0) / a.reps * 1e3:.2f} ms")
if a.kernels:
    eng.profile(True)
    eng.profile_reset()
    for _ in range(a.reps):
        eng.generate(z)
    k = eng.profile_read()
    for name, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"])[:12]:
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
        print(f"  {name:42s} {v['ms'] / a.reps:8.2f} ms  {v['launches'] // a.reps:4d} launches  {tf:6.1f} TF")
