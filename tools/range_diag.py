"""Round-6 diagnostic: the generator on decoded features scaled by 2^sc in x6, h3 (all), h3 without
the pair kernels, against the fp64 oracle (SNR in dB)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, weights
from distilcodec_nabeel_amd.engine import NativeCodec
from oracle import reference_cpu as R


def snr(x, r):
    x = np.asarray(x, np.float64); r = np.asarray(r, np.float64)
    return 10 * np.log10((r ** 2).sum() / max(((x - r) ** 2).sum(), 1e-300))


cfg = config.default_config()
state = weights.synthetic_state_dict(cfg, seed=1234)
eng = NativeCodec(cfg, state, "cuda:0", gemm="x6")
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "e2e_batch.npz"))
z0 = torch.from_numpy(g["quantized"])  # (B, 1024, T)
for sc in [0, 4, 8]:
    z = z0 * 2.0 ** sc
    ref = R.generator(z.double(), state["generator"], cfg["decoder"], torch.float64)[:, 0].numpy()
    zc = z.transpose(1, 2)
    out = {}
    for name, kn in [("x6", dict(DCX_H3=0, DCX_H3_PAIRS=0)), ("h3", {}), ("h3 wide only", dict(DCX_H3_PAIRS=0)),
                     ("h3 pairs only", dict(DCX_H3=0))]:
        with eng.knobs(**kn):
            out[name] = eng.generate(zc).cpu().double().numpy().reshape(ref.shape)
    line = "  ".join(f"{k}: {snr(v, ref):.1f}" for k, v in out.items())
    print(f"2^{sc}: vs fp64 oracle  {line}   h3 vs x6 {snr(out['h3'], out['x6']):.1f}  flags {eng.range_flags()}", flush=True)
    # per-stage: the generator's intermediate after stage i
    for st in [1, 3, 5]:
        refs = R.generator(z.double(), state["generator"], cfg["decoder"], torch.float64, stages=st)
        print(f"   (oracle stage {st} max |x| {refs.abs().max().item():.3g})", flush=True)
