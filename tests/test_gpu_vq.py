"""GPU VQ search in x6 mode against an exact fp64 argmin.

x6 mode searches with a one-product bf16 prefilter (vq_prefilter_b1; vq_prefilter_x3 on planes
where it does not take the shape) and then an fp64 rescore (launch_vq_prefilter /
vq_rescore_kernel). The prefilter's winner is accepted only when no other code can be inside
its rigorous error bound. Every other row is rescored in fp64. The search must therefore return
the exact nearest code for every row, with the lowest index on exact ties (the reference's
first-index argmax of -dist, vector_quantize_pytorch.py:41-45, :96).

The check runs on our own x_pjt_in, so no tolerance is involved. The fp64 argmin is computed
with torch on the GPU. It differs from the rescore only in summation order, which cannot move an
argmin unless two distances agree to about 1e-13.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEY = "grvq.rvqs.0.layers.0._codebook.embed"


def _argmin_fp64(P: torch.Tensor, E: torch.Tensor, chunk: int = 1024) -> np.ndarray:
    E64 = E.to("cuda:0", torch.float64)
    e2 = (E64 ** 2).sum(1)
    out = []
    for s in range(0, P.shape[0], chunk):
        x = P[s: s + chunk].to("cuda:0", torch.float64)
        d = (x ** 2).sum(1)[:, None] + e2[None, :] - 2.0 * (x @ E64.T)
        # first index of the minimum, exact ties included: the fp64 GEMM may round identical codebook
        # rows differently in different column tiles, so distances within 1e-12 relative of the
        # minimum (far below any fp32-valued gap) count as ties
        m = d.min(dim=1, keepdim=True).values
        tie = d <= m + 1e-12 * m.abs()
        out.append(torch.argmax(tie.to(torch.int8), dim=1).cpu())
    return torch.cat(out).numpy()


@pytest.fixture(scope="module")
def veng(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return NativeCodec(cfg, state, "cuda:0", with_generator=False, gemm="x6")


def _search(eng, feat):
    codes, pin, _, _ = eng.vq_encode(feat, want_fup=False, want_quantized=False)
    return codes.cpu().numpy().reshape(-1), pin.reshape(-1, pin.shape[-1])


@pytest.mark.parametrize("name", ["e2e_batch", "e2e_3s", "e2e_real"])
def test_search_exact_on_fixture_audio(veng, golden, state, name):
    g = golden[name]
    feat = veng.encode(torch.from_numpy(g["mel"]).transpose(1, 2))
    codes, pin = _search(veng, feat)
    from oracle import reference_cpu as R

    E = R.codebook(state["quantizer"])
    assert np.array_equal(codes, _argmin_fp64(pin, E))


def test_search_exact_many_rows(veng, state):
    # 4 x 1200 frames: 19 row panels, so the grouped tile order has a partial 16-panel group.
    g = torch.Generator().manual_seed(5)
    feat = torch.randn(4, 1200, 1024, generator=g) * 0.5
    veng.vq_rescore_stats(reset=True)
    codes, pin = _search(veng, feat)
    from oracle import reference_cpu as R

    E = R.codebook(state["quantizer"])
    assert np.array_equal(codes, _argmin_fp64(pin, E))
    rows, n = veng.vq_rescore_stats()
    assert 0 <= rows <= codes.size and n >= 2 * rows


def test_search_duplicate_codes_lowest_index(cfg, state):
    """Exact ties: copies of each row's chosen code at other indices, in the same 128-code tile
    (which forces the whole-tile rescore) and in another tile. The lowest index must win."""
    from distilcodec_nabeel_amd.engine import NativeCodec
    from oracle import reference_cpu as R

    g = torch.Generator().manual_seed(11)
    feat = torch.randn(1, 64, 1024, generator=g) * 0.5
    base = NativeCodec(cfg, state, "cuda:0", with_generator=False, gemm="x6")
    codes0, _ = _search(base, feat)
    del base
    E = R.codebook(state["quantizer"]).clone()
    NC = E.shape[0]
    chosen = sorted(set(codes0.tolist()))[:8]
    expect = {}
    for c in chosen:
        same_tile = c ^ 1
        other_tile = (c + 4096 + 64) % NC
        if same_tile in chosen or other_tile in chosen:
            continue
        E[same_tile] = E[c]
        E[other_tile] = E[c]
        expect[c] = min(c, same_tile, other_tile)
    assert expect
    st = {k: dict(v) for k, v in state.items()}
    st["quantizer"][KEY] = E[None].numpy() if isinstance(state["quantizer"][KEY], np.ndarray) else E[None]
    eng = NativeCodec(cfg, st, "cuda:0", with_generator=False, gemm="x6")
    eng.vq_rescore_stats(reset=True)
    codes, pin = _search(eng, feat)
    assert np.array_equal(codes, _argmin_fp64(pin, E))
    hit = [i for i, c in enumerate(codes0) if int(c) in expect]
    assert hit
    for i in hit:
        assert codes[i] == expect[int(codes0[i])]
    rows, n = eng.vq_rescore_stats()
    assert rows >= len(hit) and n >= 128 * len(hit)


def test_workspace_without_generator(veng):
    # a handle finalized without generator weights sizes its workspace for encode + VQ only
    # (the generator's 13 buffers of B*T*8192 values are about 16 GB at 32 x 10 s)
    ws = int(veng.L.dcx_workspace_size(veng.h, 32, 937))
    gen = (5 * 4 + 8 * 6) * 32 * 937 * 8192
    assert 0 < ws < gen // 3


def test_compact_layout_same_codes(veng, cfg, state):
    """x6 mode hands x_pjt_in to vq_prefilter_b1 in the compact bf16 layout with the codebook's hi
    plane packed per K32 step; DCX_NO_COMPACT=1 keeps the planes layout (vq_prefilter_x3). Both
    searches are exact, so x_pjt_in and the codes agree bit for bit."""
    import os

    from distilcodec_nabeel_amd.engine import NativeCodec

    os.environ["DCX_NO_COMPACT"] = "1"
    try:
        plain = NativeCodec(cfg, {"encoder": state["encoder"], "quantizer": state["quantizer"]}, "cuda:0",
                            with_generator=False, gemm="x6")
    finally:
        del os.environ["DCX_NO_COMPACT"]
    g = torch.Generator().manual_seed(3)
    feat = (torch.randn(3, 700, 1024, generator=g) * 0.7).cuda()
    a = veng.vq_encode(feat, want_fup=False, want_quantized=False)
    b = plain.vq_encode(feat, want_fup=False, want_quantized=False)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])
    np.testing.assert_array_equal(a[0].cpu().numpy().reshape(-1), _argmin_fp64(a[1].reshape(-1, a[1].shape[-1]),
                                                                                 torch.from_numpy(state["quantizer"][KEY][0])))


@pytest.mark.parametrize("rows", [1, 93, 139, 256, 257])
def test_search_exact_single_row_panel(veng, state, rows):
    """Searches of at most one 256-row panel (a streaming hop: most of each tile's rows are past the
    end) and just over one: exact."""
    from oracle import reference_cpu as R

    g = torch.Generator().manual_seed(rows)
    feat = torch.randn(1, rows, 1024, generator=g) * 0.5
    codes, pin = _search(veng, feat)
    assert np.array_equal(codes, _argmin_fp64(pin, R.codebook(state["quantizer"])))


def test_search_near_duplicates_exact(cfg, state):
    """Codes that differ from each row's chosen code only below bf16 resolution (relative 1e-6
    perturbations, in the same 256-code tile and in other tiles): the one-product prefilter sees
    equal or nearly equal distances, so only the rescore can separate them. The search must
    still return the exact fp64 argmin."""
    from distilcodec_nabeel_amd.engine import NativeCodec
    from oracle import reference_cpu as R

    g = torch.Generator().manual_seed(13)
    feat = torch.randn(2, 300, 1024, generator=g) * 0.5
    base = NativeCodec(cfg, state, "cuda:0", with_generator=False, gemm="x6")
    codes0, _ = _search(base, feat)
    del base
    E = R.codebook(state["quantizer"]).clone()
    NC = E.shape[0]
    chosen = sorted(set(codes0.tolist()))[:24]
    for k, c in enumerate(chosen):
        for t in (c ^ 3, (c + 256 * (k % 7 + 1)) % NC, (c + 9000) % NC):
            if t in chosen:
                continue
            E[t] = E[c] * (1 + 1e-6 * torch.randn(E.shape[1], generator=g))
    st = {k: dict(v) for k, v in state.items()}
    st["quantizer"][KEY] = E[None].numpy() if isinstance(state["quantizer"][KEY], np.ndarray) else E[None]
    eng = NativeCodec(cfg, st, "cuda:0", with_generator=False, gemm="x6")
    eng.vq_rescore_stats(reset=True)
    codes, pin = _search(eng, feat)
    assert np.array_equal(codes, _argmin_fp64(pin, E))
    rows, n = eng.vq_rescore_stats()
    assert rows > 0 and n >= 2 * rows


@pytest.mark.parametrize("per_row", ["0", "2"])
def test_rescore_in_place_path_same_codes(veng, cfg, state, per_row):
    """DCX_VQ_PAIRS_PER_ROW=0 leaves the rescore's candidate list no room, so every uncertified
    row is rescored by its own wave in vq_certify_kernel (the overflow path) instead of through
    vq_pair_eval_kernel / vq_pair_reduce_kernel; with 2 per row the list fills part way (rows
    listed, then an overflowing block padded with sentinels, then rows rescored in place). The
    same fp64 arithmetic either way, so the same codes."""
    import os

    from distilcodec_nabeel_amd.engine import NativeCodec

    os.environ["DCX_VQ_PAIRS_PER_ROW"] = per_row
    try:
        inplace = NativeCodec(cfg, {"encoder": state["encoder"], "quantizer": state["quantizer"]}, "cuda:0",
                              with_generator=False, gemm="x6")
    finally:
        del os.environ["DCX_VQ_PAIRS_PER_ROW"]
    g = torch.Generator().manual_seed(21)
    feat = (torch.randn(2, 400, 1024, generator=g) * 0.6).cuda()
    a = veng.vq_encode(feat, want_fup=False, want_quantized=False)
    inplace.vq_rescore_stats(reset=True)
    b = inplace.vq_encode(feat, want_fup=False, want_quantized=False)
    rows, _ = inplace.vq_rescore_stats()
    assert rows > 0
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])

