"""GPU diagnostic: how the conv kernels' fp32 accumulation of exact bf16 products errs, against fp64.

A 1x1 conv (K = Cin) on bf16-exact inputs and weights in x6 mode (mid / lo planes zero, so only the hi
products contribute and nothing is rounded to bf16): the signed error (ours - fp64) per output, in
units of 2^-24 |sum of |terms||.  Round-to-nearest accumulation gives mean ~0 and spread ~sqrt(K);
a truncating adder gives a mean biased toward zero growing ~K.  Prints one JSON line per K."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from distilcodec_nabeel_amd.engine import NativeConv  # noqa: E402


def bf(a):
    return torch.from_numpy(a).bfloat16().float().numpy()


def main():
    g = np.random.default_rng(0)
    for K in (128, 512, 2048, 4096):
        x = bf(g.standard_normal((1, 4096, K)).astype(np.float32))
        w = bf((g.standard_normal((256, K, 1)) / np.sqrt(K)).astype(np.float32))
        conv = NativeConv(w)
        y = conv(torch.from_numpy(x).cuda(), gemm="x6").cpu().numpy().astype(np.float64)[0]
        ex = x[0].astype(np.float64) @ w[:, :, 0].T.astype(np.float64)
        scale = np.abs(x[0]).astype(np.float64) @ np.abs(w[:, :, 0]).T.astype(np.float64)
        e = (y - ex) / (scale * 2.0 ** -24)
        toward_zero = float(np.mean(np.sign(y - ex) == -np.sign(ex)))
        ef = (x[0].astype(np.float32) @ w[:, :, 0].T.astype(np.float32)).astype(np.float64)
        e32 = (ef - ex) / (scale * 2.0 ** -24)
        print(json.dumps({"K": K, "mean_err_units": float(e.mean()), "rms_err_units": float(np.sqrt((e ** 2).mean())),
                          "frac_toward_zero": toward_zero, "numpy_fp32_rms_units": float(np.sqrt((e32 ** 2).mean()))}))


if __name__ == "__main__":
    main()
