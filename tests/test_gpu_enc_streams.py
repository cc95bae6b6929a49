"""The encoder's two half-batches on two streams (Knobs::enc_streams, round 6) give the
bits of the one-stream run: every encoder kernel computes a clip's rows alone (encoders.py:68-76:
stem, LayerNorms, downsample convs and ConvNeXt blocks are per-frame or per-clip operations), so
splitting the batch moves no arithmetic.  Checked on ragged-length batches (odd and even clip
counts), in the default (h3 / x6) and the bf16 arithmetic, through the staged encoder call and the
fused encode_decode, and with the range flags clear."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _audio(B, n, seed):
    from distilcodec_nabeel_amd import synth

    a = torch.zeros(B, n + 1)
    for i, c in enumerate(synth.clips(B, n, seed=seed, kind="mix")):
        a[i, 1:] = torch.from_numpy(c)
    return a.cuda()


@pytest.fixture(scope="module")
def engines(cfg, state):
    from distilcodec_nabeel_amd.engine import NativeCodec

    return {"x6": NativeCodec(cfg, state, "cuda:0", gemm="x6"),
            "bf16": NativeCodec(cfg, state, "cuda:0", gemm="bf16")}


@pytest.mark.parametrize("mode", ["x6", "bf16"])
@pytest.mark.parametrize("B", [2, 5])
def test_staged_encoder_same_bits(engines, mode, B):
    eng = engines[mode]
    assert eng.get_knob("DCX_ENC_STREAMS") == 2  # the shipped default (the encoder forks at >= 1)
    mel = eng.mel(_audio(B, 3 * 24000 + 77, seed=B))
    two = eng.encode(mel).clone()
    with eng.knobs(DCX_ENC_STREAMS=0):
        one = eng.encode(mel).clone()
    torch.cuda.synchronize()
    assert torch.equal(two, one)
    assert eng.range_flags(reset=True) == 0


@pytest.mark.parametrize("B", [3, 4])
def test_encode_decode_same_bits(engines, B):
    """dcx_encode_decode with the half-batches forked at every level: 2 (the default: mel, encoder,
    VQ encode / decode per half, the generator on the whole batch), 3 (the generator per half too),
    1 (the encoder only) against one stream (0); each mode's workspace within a few % of one stream's."""
    eng = engines["x6"]
    audio = _audio(B, 2 * 24000 + 5, seed=11)
    T = eng.num_frames(audio.shape[1])
    with eng.knobs(DCX_ENC_STREAMS=0):
        codes1, wav1 = [t.clone() for t in eng.encode_decode(audio)]
        ws0 = eng.workspace_size(B, T)
    for mode in (1, 3, 2):
        with eng.knobs(DCX_ENC_STREAMS=mode):
            codes, wav = [t.clone() for t in eng.encode_decode(audio)]
            assert eng.workspace_size(B, T) <= ws0 * 1.1
        torch.cuda.synchronize()
        assert torch.equal(codes, codes1) and torch.equal(wav, wav1), mode
    codes2, wav2 = codes, wav
    # and a clip alone equals its row of the batch (batch invariance through the split)
    c_alone, w_alone = [t.clone() for t in eng.encode_decode(audio[2:3])]
    torch.cuda.synchronize()
    assert torch.equal(codes2, codes1) and torch.equal(wav2, wav1)
    assert torch.equal(c_alone[0], codes2[2]) and torch.equal(w_alone[0], wav2[2])
    assert eng.range_flags(reset=True) == 0



def test_graph_capture_keeps_one_stream(engines):
    """A call captured into a hipGraph (the stream is capturing) does not fork; its replay gives the
    bits of the eager call, which does (B = 2 hops of 1 s; the workspace covers both plans)."""
    from distilcodec_nabeel_amd.streaming import GraphedHop

    eng = engines["x6"]
    hop = GraphedHop(eng, 24000, batch=2)
    chunk = _audio(2, 24000, seed=9)[:, 1:].contiguous()
    gc, gw = [t.clone() for t in hop(chunk)]
    padded = torch.nn.functional.pad(chunk, (1, 0))
    ec, ew = [t.clone() for t in eng.encode_decode(padded)]
    torch.cuda.synchronize()
    assert torch.equal(gc, ec) and torch.equal(gw, ew)
