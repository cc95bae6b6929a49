"""The conv kernel family in isolation (both GEMM modes) vs an fp64 CPU reference of
F.conv1d / F.conv_transpose1d, across the shapes the path uses: dilations, tap counts,
ConvTranspose phases, small and large channel counts, ragged lengths.

Tolerance: max |y - y64| <= 1e-5 * max|y64| (fp32-level; both modes measure ~1e-7..1e-6)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [
    # cin, cout, k, dil, transposed, stride, L
    (512, 512, 3, 1, False, 1, 300),
    (512, 512, 11, 5, False, 1, 257),
    (256, 256, 7, 3, False, 1, 1000),
    (128, 128, 11, 5, False, 1, 515),
    (64, 64, 11, 5, False, 1, 700),
    (32, 32, 7, 3, False, 1, 1333),
    (32, 32, 3, 1, False, 1, 64),
    (1024, 1024, 13, 1, False, 1, 97),
    (128, 256, 7, 1, False, 1, 93),
    (1024, 4096, 1, 1, False, 1, 190),
    (3584, 1024, 1, 1, False, 1, 77),
    (1024, 512, 16, 1, True, 8, 50),
    (512, 256, 12, 1, True, 4, 61),
    (256, 128, 4, 1, True, 2, 129),
    (64, 32, 4, 1, True, 2, 333),
    (1024, 1024, 1, 1, True, 1, 45),
    # fewer K16 steps than the LDS-DMA prefetch depth (2 and 6 steps)
    (32, 128, 1, 1, False, 1, 300),
    (32, 256, 3, 1, False, 1, 200),
    # 256-column LDS-DMA kernel: 2 steps (ConvT phases), 12 steps with dilation
    (16, 256, 4, 1, True, 2, 100),
    (64, 512, 3, 2, False, 1, 260),
    # 512-row tiles (Cout 128): three row tiles, the last ragged
    (128, 128, 3, 1, False, 1, 1100),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("gemm", ["x6", "f32"])
def test_conv_matches_fp64(case, gemm):
    from distilcodec_nabeel_amd.engine import NativeConv

    cin, cout, k, d, tr, s, L = case
    r = np.random.default_rng(abs(hash(case)) % 2 ** 32)
    w = (r.standard_normal((cin, cout, k) if tr else (cout, cin, k)) / np.sqrt(cin * k)).astype(np.float32)
    b = r.standard_normal(cout).astype(np.float32) * 0.1
    x = r.standard_normal((2, L, cin)).astype(np.float32)
    conv = NativeConv(w, b, dilation=d, transposed=tr, stride=s)
    res = torch.from_numpy(r.standard_normal((2, L * (s if tr else 1), cout)).astype(np.float32)).cuda()
    y, ys = conv(torch.from_numpy(x).cuda(), gemm=gemm, epi=3, res=res, want_silu=True)
    xt = torch.from_numpy(x).double().transpose(1, 2)
    if tr:
        ref = F.conv_transpose1d(xt, torch.from_numpy(w).double(), torch.from_numpy(b).double(), stride=s, padding=(k - s) // 2)
    else:
        ref = F.conv1d(xt, torch.from_numpy(w).double(), torch.from_numpy(b).double(), dilation=d, padding=d * (k - 1) // 2)
    ref = ref.transpose(1, 2) + res.cpu().double()
    err = (y.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err
    sref = ref * torch.sigmoid(ref)
    assert (ys.cpu().double() - sref).abs().max().item() / sref.abs().max().item() < 1e-5
