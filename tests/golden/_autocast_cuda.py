"""CUDA autocast's bf16 op policy applied to CPU tensors (fixture generation only).

The reference's `enable_bfloat16=True` wraps encode / decode in
`torch.autocast(device_type="cuda", dtype=torch.bfloat16)` (`distilcodec/distil_codec.py:550,576,590,
629`).  On a machine without CUDA that context disables itself, and `torch.autocast("cpu")` is a
different policy (CPU autocast keeps `pow` and `layer_norm` in the input dtype, and the codebook's
`torch.cuda.amp.autocast(enabled=False)` at `vector_quantize_pytorch.py:10,462` does not switch it
off).  This module restates CUDA's policy (torch 2.x `autocast_mode.cpp`, CUDA op lists) as a
`TorchFunctionMode` so the reference's own modules can be run with CUDA's dtypes on the CPU:

* lower-precision list (conv1d, conv_transpose1d, linear, matmul, mm, bmm, addmm, ...): floating
  tensor arguments are cast to bf16, so outputs are bf16 (fp32 accumulation inside the CPU kernel);
* fp32 list (pow, layer_norm, cdist, sum, softmax, log, exp, rsqrt, norm, ...): floating tensor
  arguments are cast to fp32;
* promote list (cat, stack, addcmul, addcdiv, ...): arguments are cast to the widest floating dtype;
* every other op runs in its inputs' dtypes (bf16 elementwise ops such as silu, gelu, tanh, mean and
  the residual `+` stay bf16 when their inputs are bf16, as on the GPU).

The policy is active while the CUDA autocast flag is set (`torch.set_autocast_enabled("cuda", ...)`,
which works without a GPU), so the reference's own `autocast(enabled=False)` regions (the codebook
search) run in fp32 exactly as they do on a GPU.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

_LOWER = {
    "conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
    "conv_tbc", "linear", "matmul", "__matmul__", "mm", "mv", "bmm", "baddbmm", "addmm", "addmv",
    "addr", "addbmm", "chain_matmul", "multi_dot", "prelu", "einsum",
}
_FP32 = {
    "pow", "__pow__", "__rpow__", "__rdiv__", "__rtruediv__", "layer_norm", "group_norm", "cdist",
    "sum", "prod", "cumsum", "cumprod", "softmax", "log_softmax", "softmin", "log", "log10", "log2",
    "log1p", "exp", "expm1", "rsqrt", "reciprocal", "norm", "normalize", "acos", "asin", "cosh",
    "sinh", "tan", "erfinv", "softplus", "dist", "pdist", "renorm", "cosine_similarity",
    "mse_loss", "l1_loss", "smooth_l1_loss", "kl_div", "nll_loss", "cross_entropy",
}
_PROMOTE = {"cat", "stack", "addcmul", "addcdiv", "atan2", "cross", "dot", "tensordot", "index_put",
            "scatter_add", "bilinear"}


def _name(func) -> str:
    return getattr(func, "__name__", "")


def _cast(obj, dtype):
    if isinstance(obj, torch.Tensor) and obj.is_floating_point() and obj.dtype != dtype:
        return obj.to(dtype)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cast(o, dtype) for o in obj)
    return obj


def _widest(objs):
    best = None
    for o in objs:
        if isinstance(o, (list, tuple)):
            w = _widest(o)
            o = torch.empty(0, dtype=w) if w is not None else None
        if isinstance(o, torch.Tensor) and o.is_floating_point():
            if best is None or torch.finfo(o.dtype).bits > torch.finfo(best).bits:
                best = o.dtype
    return best


class CudaAutocastPolicy(TorchFunctionMode):
    """Applies CUDA autocast's bf16 policy while `torch.is_autocast_enabled("cuda")`.

    exact=True: the lower-precision ops take the same bf16 operands but accumulate in fp64 and round
    once to bf16 (an idealised kernel).  Its distance to the fp32-accumulating CPU kernels measures how
    much a module's bf16 output moves with accumulation order alone (the tests' noise scale).
    wn64=True: weight-normed convs fold torch._weight_norm(v, g) in fp64 and round the result to fp32,
    as the library does once at load, instead of the reference's fp32 fold.  In bf16
    the two folds round a few weights to different bf16 values (where the fp32 folds straddle a bf16
    rounding boundary), which moves a chained module's output by more than accumulation order does."""

    def __init__(self, exact: bool = False, wn64: bool = False):
        super().__init__()
        self.exact = exact
        self.wn64 = wn64

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.wn64 and _name(func) == "_weight_norm":  # torch._weight_norm(v, g, dim) folded in fp64
            v, g = args[0], args[1]
            return func(v.double(), g.double(), *args[2:], **kwargs).to(v.dtype)
        if torch.is_autocast_enabled("cuda"):
            n = _name(func)
            if n in _LOWER and self.exact:
                args = _cast(_cast(args, torch.bfloat16), torch.float64)
                kwargs = {k: _cast(_cast(v, torch.bfloat16), torch.float64) for k, v in kwargs.items()}
                return func(*args, **kwargs).to(torch.bfloat16)
            if n in _LOWER:
                args, kwargs = _cast(args, torch.bfloat16), {k: _cast(v, torch.bfloat16) for k, v in kwargs.items()}
            elif n in _FP32:
                args, kwargs = _cast(args, torch.float32), {k: _cast(v, torch.float32) for k, v in kwargs.items()}
            elif n in _PROMOTE:
                w = _widest(list(args) + list(kwargs.values()))
                if w is not None:
                    args, kwargs = _cast(args, w), {k: _cast(v, w) for k, v in kwargs.items()}
        return func(*args, **kwargs)


@contextlib.contextmanager
def cuda_autocast_bf16(exact: bool = False, wn64: bool = False):
    """`with torch.autocast("cuda", torch.bfloat16)` as the reference's GPU run sees it, on CPU tensors
    (exact: fp64 accumulation inside the bf16 ops; wn64: weight norm folded in fp64; see
    CudaAutocastPolicy)."""
    prev = torch.is_autocast_enabled("cuda")
    torch.set_autocast_enabled("cuda", True)
    try:
        with CudaAutocastPolicy(exact, wn64):
            yield
    finally:
        torch.set_autocast_enabled("cuda", prev)


__all__ = ["cuda_autocast_bf16", "CudaAutocastPolicy"]
