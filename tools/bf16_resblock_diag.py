"""GPU diagnostic: ResBlock1 of a small-C generator stage in bf16 mode, three ways, on the bf16
fixture's captured input: (a) the module path (dcx_module_forward: fp32-input conv kernels with
SiLU on load), (b) the same convs through the conv primitive (planes input) with torch doing the
bf16 SiLU / residual roundings between them, (c) the reference's output from the fixture.  Prints
relative distances, to localise a discrepancy."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec, NativeConv  # noqa: E402


def bfv(t):
    return t.to(torch.bfloat16).float()


def get(fx, k):
    if k in fx:
        return fx[k].astype(np.float32)
    return (fx[k + "_bf16"].astype(np.uint32) << 16).view(np.float32)


def fold(sd, p):
    g = torch.from_numpy(np.asarray(sd[f"{p}.parametrizations.weight.original0"], np.float64))
    v = torch.from_numpy(np.asarray(sd[f"{p}.parametrizations.weight.original1"], np.float64))
    return torch._weight_norm(v, g, 0).float().numpy()


def main():
    cfg = config.default_config()
    state = weights.synthetic_state_dict(cfg, seed=1234)
    eng = NativeCodec(cfg, state, "cuda:0", gemm="bf16")
    fx = dict(np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/bf16.npz")))
    d = cfg["decoder"]
    for stage, blk in ((4, 0), (4, 1), (4, 2), (3, 2)):
        name = f"generator.resblocks.{stage}.blocks.{blk}"
        x = torch.from_numpy(get(fx, f"m:{name}:in"))  # (1, C, L)
        ref = torch.from_numpy(get(fx, f"m:{name}:out"))
        ya = eng.module(name, x.transpose(1, 2).contiguous().cuda()).transpose(1, 2).cpu()
        sd = state["generator"]
        k = d["resblock_kernel_sizes"][blk]
        xs = x.clone()
        for c, dil in enumerate(d["resblock_dilation_sizes"][blk]):
            p1, p2 = f"resblocks.{stage}.blocks.{blk}.convs1.{c}", f"resblocks.{stage}.blocks.{blk}.convs2.{c}"
            c1 = NativeConv(fold(sd, p1), np.asarray(sd[p1 + ".bias"], np.float32), dilation=dil)
            c2 = NativeConv(fold(sd, p2), np.asarray(sd[p2 + ".bias"], np.float32), dilation=1)
            t = bfv(F.silu(xs))
            t = c1(t.transpose(1, 2).contiguous().cuda(), gemm="bf16").cpu().transpose(1, 2)
            t = bfv(F.silu(t))
            t = c2(t.transpose(1, 2).contiguous().cuda(), gemm="bf16").cpu().transpose(1, 2)
            xs = bfv(t + xs)
        rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())  # noqa: E731
        print(f"{name} k={k}: module-vs-ref {rel(ya, ref):.3e}  prim-vs-ref {rel(xs, ref):.3e}  module-vs-prim {rel(ya, xs):.3e}"
              f"  exact_spread {float(fx[f'm:{name}:exact_spread']):.3e}")


if __name__ == "__main__":
    main()
