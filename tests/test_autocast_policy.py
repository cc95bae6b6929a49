"""The CUDA-autocast policy restatement used to make tests/golden/bf16.npz (`_autocast_cuda.py`):
op-level dtypes as torch's CUDA autocast gives them (lower-precision list -> bf16, fp32 list -> fp32,
other ops in their inputs' dtype), and the reference's `autocast(enabled=False)` regions honoured."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

from _autocast_cuda import cuda_autocast_bf16  # noqa: E402


def test_policy_dtypes():
    x = torch.randn(2, 8, 16)
    conv = torch.nn.Conv1d(8, 8, 3, padding=1)
    lin = torch.nn.Linear(8, 8)
    with torch.no_grad(), cuda_autocast_bf16():
        y = conv(x)
        assert y.dtype == torch.bfloat16                      # conv1d: lower-precision list
        assert y.mean(1).dtype == torch.bfloat16              # mean: no list, input dtype
        assert (y - y.mean(1, keepdim=True)).pow(2).dtype == torch.float32  # pow: fp32 list
        z = F.layer_norm(y.transpose(1, 2), (8,))
        assert z.dtype == torch.float32                       # layer_norm: fp32 list
        h = lin(z)
        assert h.dtype == torch.bfloat16 and F.gelu(h).dtype == torch.bfloat16
        assert (torch.ones(8) * h).dtype == torch.float32     # fp32 param * bf16 -> promotion
        assert torch.stack([h, h.float()]).dtype == torch.float32  # promote list
        with torch.cuda.amp.autocast(enabled=False):          # vector_quantize_pytorch.py:462
            assert lin(z).dtype == torch.float32
        assert lin(z).dtype == torch.bfloat16
    assert not torch.is_autocast_enabled("cuda")
    assert conv(x).dtype == torch.float32


def test_policy_single_rounding():
    """bf16 conv / linear on the CPU: fp32 accumulation and one rounding of the exact result (what
    the bf16 fixture assumes of the reference's GPU kernels)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(300, 256, generator=g)
    w = torch.randn(512, 256, generator=g) * 0.05
    b = torch.randn(512, generator=g) * 0.1
    with torch.no_grad(), cuda_autocast_bf16():
        y = F.linear(x, w, b)
    exact = F.linear(x.bfloat16().double(), w.bfloat16().double(), b.bfloat16().double()).bfloat16()
    assert (y == exact).double().mean() > 0.999
