"""Generate the committed golden fixtures by running the REAL reference in this container.

    python tests/golden/make_golden.py          (build container only: needs /root/reference)

The reference is imported from /root/reference with placeholders for its absent third-party
deps (`_ref_loader.py`), built from its own config file, loaded with the deterministic
synthetic weights of `distilcodec_nabeel_amd.weights.synthetic_state_dict(seed=1234)`, put in
eval mode, and run on CPU in fp32 with 8 torch threads.  Outputs are saved as small npz
fixtures (inputs + expected outputs only; no reference source travels).

Fixtures
--------
* `e2e_batch.npz`   : 2 ragged speech/music clips (1.00 s, 0.71 s) through `DistilCodec.encode`
                      (raw_audio=True) and `quantizer.decode` + `generator` (the body of
                      `decode_from_codes` with layout (G=1,B,T,R=1)); mel, encoder features,
                      codes, x_pjt_in (clip 0), quantized, decoded waveform, fp64 top-2 VQ gaps.
* `e2e_3s.npz`      : one 3 s speech clip, same stages (features omitted to keep it small).
* `e2e_real.npz`    : the first 2 s of two real 24 kHz speech recordings shipped with the reference
                      (`data/org_audios/0000.wav`, `0001.wav`; PCM16 read with the stdlib `wave`),
                      batched (ragged: 2.0 s and 1.5 s); codes, fp64 gaps, quantized, waveform.
* `modules.npz`     : per-module cases called on the reference's own modules: ConvNeXtBlock(256),
                      channels-first LayerNorm(256), ResBlock1(64, k=11), ParralelBlock(32),
                      each ConvTranspose1d of the generator, EuclideanCodebook search on a
                      1024-code slice, `quantizer.decode` of codes holding the masked code -1,
                      and `spec_transform(..., return_linear=True)` of e2e_batch clip 0.
* `bf16.npz`        : the reference with `enable_bfloat16=True`, i.e. under CUDA autocast's op policy
                      applied on the CPU (`_autocast_cuda.py`): e2e features / x_pjt_in / codes / decode
                      of the e2e_batch clips and per-module cases (see `make_bf16`).
                      `python tests/golden/make_golden.py bf16` regenerates it alone.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from distilcodec_nabeel_amd import synth, weights  # noqa: E402
from oracle import reference_cpu as R  # noqa: E402  (fp64 gap analysis only)

SEED = 1234
THREADS = 8


def _ref_root():
    import _ref_loader

    return _ref_loader.REF_ROOT


def _np(t):
    return t.detach().cpu().numpy()


def build_reference():
    import _ref_loader

    dc = _ref_loader.import_reference()
    cfg = json.load(open(os.path.join(_ref_loader.REF_ROOT, "configs", "model_config.json")))
    codec = dc.DistilCodec(cfg)
    sd = weights.synthetic_state_dict(cfg, seed=SEED)
    for part in ("encoder", "quantizer", "generator"):
        mod = getattr(codec, part)
        tsd = {k: torch.from_numpy(v) for k, v in sd[part].items()}
        missing, unexpected = mod.load_state_dict(tsd, strict=False)
        allowed = {"grvq.rvqs.0.layers.0._codebook.embed_avg", "grvq.rvqs.0.layers.0._codebook.cluster_size"}
        assert not unexpected, unexpected
        assert set(missing) <= allowed, missing
    codec.eval()
    codec.device = torch.device("cpu")
    return codec, cfg


def run_e2e(codec, clips):
    with torch.no_grad():
        ret, gen_lens, hop_lens = codec.encode([[c, 24000] for c in clips], enable_bfloat16=False, raw_audio=True)
        audios, mel, _, _ = codec.preprocess_raw_audio_batch([[c, 24000] for c in clips])
        feat = codec.encoder(mel)
        codes = ret.codes  # (1, B, T, 1)
        z = codec.quantizer.decode(codes)
        wav = codec.generator(z)
    return dict(audio=_np(audios[:, 0]), mel=_np(mel), feat=_np(feat), codes=_np(codes[0, :, :, 0]).astype(np.int64),
                x_pjt_in=_np(ret.x_pjt_in), quantized=_np(ret.quantized), z=_np(z), wav=_np(wav[:, 0]),
                n_hop=np.array(hop_lens), gen_len=np.array(gen_lens),
                tokens0=np.array([d["absolute_token_id"] for d in ret.codes_list[0]]))


def main():
    torch.manual_seed(0)
    torch.set_num_threads(THREADS)
    codec, cfg = build_reference()
    embed = codec.quantizer.grvq.rvqs[0].layers[0]._codebook.embed[0]

    clips = [synth.speech_like(24000, 11), synth.music_like(17000, 12)]
    out = run_e2e(codec, clips)
    best, second, arg64 = R.top2_gap_fp64(torch.from_numpy(out["x_pjt_in"]), embed)
    out.update(gap_best=_np(best), gap_second=_np(second), argmin_fp64=_np(arg64).reshape(out["codes"].shape))
    assert np.array_equal(out["z"], out["quantized"])  # decode(codes) == forward's up-path
    out.pop("z")
    out["x_pjt_in"] = out["x_pjt_in"][:1]  # clip 0 only: keeps the fixture small
    out.update(threads=np.array(THREADS), seed=np.array(SEED))
    np.savez_compressed(os.path.join(HERE, "e2e_batch.npz"), **out)
    print("e2e_batch", {k: v.shape for k, v in out.items()})

    out3 = run_e2e(codec, [synth.speech_like(72000, 21)])
    best, second, arg64 = R.top2_gap_fp64(torch.from_numpy(out3["x_pjt_in"]), embed)
    out3.update(gap_best=_np(best), gap_second=_np(second), argmin_fp64=_np(arg64).reshape(out3["codes"].shape))
    for k in ("feat", "x_pjt_in", "z"):
        out3.pop(k)
    out3.update(threads=np.array(THREADS), seed=np.array(SEED))
    np.savez_compressed(os.path.join(HERE, "e2e_3s.npz"), **out3)
    print("e2e_3s", {k: v.shape for k, v in out3.items()})

    from distilcodec_nabeel_amd import audio_io

    real = []
    for name, secs in (("0000.wav", 2.0), ("0001.wav", 1.5)):
        a, _ = audio_io.load_wav(os.path.join(_ref_root(), "data", "org_audios", name), 24000)
        real.append(a[: int(secs * 24000)])
    outr = run_e2e(codec, real)
    best, second, arg64 = R.top2_gap_fp64(torch.from_numpy(outr["x_pjt_in"]), embed)
    outr.update(gap_best=_np(best), gap_second=_np(second), argmin_fp64=_np(arg64).reshape(outr["codes"].shape))
    for k in ("feat", "x_pjt_in", "z"):
        outr.pop(k)
    outr.update(threads=np.array(THREADS), seed=np.array(SEED))
    np.savez_compressed(os.path.join(HERE, "e2e_real.npz"), **outr)
    print("e2e_real", {k: v.shape for k, v in outr.items()})

    # ---- per-module cases on the reference's own modules --------------------------------
    g = np.random.Generator(np.random.PCG64(99))
    mods = {}
    with torch.no_grad():
        blk = codec.encoder.stages[0][0]
        x = torch.from_numpy(g.standard_normal((2, 256, 50), dtype=np.float32))
        mods["convnext256_in"], mods["convnext256_out"] = _np(x), _np(blk(x))
        ln = codec.encoder.downsample_layers[1][0]
        mods["ln256_out"] = _np(ln(x))
        rb = codec.generator.resblocks[3].blocks[2]  # ResBlock1(64, k=11, dil 1/3/5)
        x = torch.from_numpy(g.standard_normal((2, 64, 300), dtype=np.float32))
        mods["resblock64_in"], mods["resblock64_out"] = _np(x), _np(rb(x))
        pb = codec.generator.resblocks[4]
        x = torch.from_numpy(g.standard_normal((1, 32, 400), dtype=np.float32))
        mods["parallel32_in"], mods["parallel32_out"] = _np(x), _np(pb(x))
        for i, up in enumerate(codec.generator.ups):
            x = torch.from_numpy(g.standard_normal((1, up.in_channels, 40), dtype=np.float32))
            mods[f"ups{i}_in"], mods[f"ups{i}_out"] = _np(x), _np(up(x))
        cb = codec.quantizer.grvq.rvqs[0].layers[0]._codebook
        emb_small = embed[:1024].clone()
        saved = cb.embed.data.clone()
        cb.embed.data = emb_small[None]
        cb.codebook_size = 1024
        x = torch.from_numpy(out["x_pjt_in"][0, :64].copy())
        q, ind, _ = cb(x[None])
        cb.embed.data = saved
        cb.codebook_size = embed.shape[0]
        mods["vq1024_in"], mods["vq1024_codes"], mods["vq1024_quant"] = _np(x), _np(ind[0]).astype(np.int64), _np(q[0])
        mods["mel_fb"] = _np(codec.spec_transform.fb)
        # masked code -1 (residual_vq.py:120-127) and a wrapping -32768 through quantizer.decode
        mc = np.random.Generator(np.random.PCG64(7)).integers(0, 32768, 24)
        mc[[0, 5, 6, 23]] = -1
        mc[2] = -32768
        zq = codec.quantizer.decode(torch.from_numpy(mc)[None, None, :, None])
        mods["masked_codes"], mods["masked_z"] = mc.astype(np.int64), _np(zq)
        # LogMelSpectrogram.forward(return_linear=True) (mel_spec.py:119-120) on e2e_batch clip 0
        mel_l, lin_l = codec.spec_transform(torch.from_numpy(out["audio"][:1])[:, None, :], return_linear=True)
        mods["linear_mel"], mods["linear_log"] = _np(mel_l), _np(lin_l)
    np.savez_compressed(os.path.join(HERE, "modules.npz"), **mods)
    print("modules", sorted(mods))
    make_bf16(codec, out["audio"])
    for f in ("e2e_batch.npz", "e2e_3s.npz", "e2e_real.npz", "modules.npz", "bf16.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)) // 1024, "KiB")


# ---- enable_bfloat16=True: the reference under CUDA autocast's dtypes ------------------------------
def _bits(t):
    """A bf16 tensor as its raw 16-bit patterns (exact, half the bytes of fp32)."""
    assert t.dtype == torch.bfloat16, t.dtype
    return _np(t.contiguous().view(torch.int16)).view(np.uint16)


def _store(d, key, t):
    if t.dtype == torch.bfloat16:
        d[key + "_bf16"] = _bits(t)
    else:
        d[key] = _np(t.float())


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


# the encoder / quantizer modules see rows [0, ENC_ROWS) of clip 0 of e2e_batch as captured, the
# generator modules the decode of its first GEN_FRAMES codes
ENC_ROWS = 32
GEN_FRAMES = 8


def _bf16_modules(codec):
    enc, q, g = codec.encoder, codec.quantizer, codec.generator
    mods = [("encoder.downsample_layers.0", enc.downsample_layers[0])]
    for i in range(1, 4):
        mods.append((f"encoder.downsample_layers.{i}", enc.downsample_layers[i]))
    for i in range(4):
        mods.append((f"encoder.stages.{i}.0", enc.stages[i][0]))
    mods += [("encoder.stages.2.4", enc.stages[2][4]),
             ("quantizer.downsample.0", q.downsample[0]), ("quantizer.grvq.rvqs.0.project_in", q.grvq.rvqs[0].project_in),
             ("quantizer.upsample.0", q.upsample[0]), ("generator.conv_pre", g.conv_pre)]
    for i in range(len(g.ups)):
        mods += [(f"generator.ups.{i}", g.ups[i])]
        nb = len(g.resblocks[i].blocks) if i >= 3 else 1  # every ResBlock1 of the small-C stages
        mods += [(f"generator.resblocks.{i}.blocks.{j}", g.resblocks[i].blocks[j]) for j in range(nb)]
        mods += [(f"generator.resblocks.{i}", g.resblocks[i])]
    mods.append(("generator.conv_post", g.activation_post))  # input of the tail: SiLU -> conv_post -> tanh
    return mods


def _bf16_module_forward(codec, name, mod, x, exact=False, wn64=False):
    """The reference module on x under the CUDA autocast policy; for the two fused module names the
    generator's own following ops (generators.py:125/141-145) are applied the same way."""
    from _autocast_cuda import cuda_autocast_bf16

    with torch.no_grad(), cuda_autocast_bf16(exact, wn64):
        if name == "generator.conv_post":
            return torch.tanh(codec.generator.conv_post(torch.nn.functional.silu(x)))
        y = mod(x)
        if name.startswith("generator.resblocks.") and name.count(".") == 2:
            y = torch.nn.functional.silu(y)  # dcx's ParallelBlock module returns silu(mean)
        return y


def make_bf16(codec, audio_batch):
    """bf16.npz: the reference's enable_bfloat16 path (`torch.autocast("cuda", bfloat16)`,
    distil_codec.py:550,590) with CUDA's op policy applied on the CPU (`_autocast_cuda.py`):
    * e2e on the e2e_batch clips: encoder features, x_pjt_in (bf16), codes, fp64 gaps of the
      bf16 x_pjt_in; the bf16 decode of those codes; the reference's own spread (8 vs 1 CPU threads:
      fp32 accumulation order) of each;
    * per-module cases: every module's input as captured in the bf16 run (clip 0; generator modules on
      the decode of the first GEN_FRAMES codes; encoder modules cropped to ENC_ROWS rows), its output, the reference's 8-vs-1-thread spread
      and its distance to the same module in fp32 (how far the dtypes move the result)."""
    from _autocast_cuda import cuda_autocast_bf16

    clips = [a for a in audio_batch]
    ng = len(clips)
    d = {}
    embed = codec.quantizer.grvq.rvqs[0].layers[0]._codebook.embed[0]
    mods = _bf16_modules(codec)
    captured = {}

    def hook(name):
        def f(_m, inp, _out):
            if name not in captured:
                captured[name] = inp[0].detach().clone()
        return f

    def run(threads, capture=False):
        torch.set_num_threads(threads)
        hs = [m.register_forward_hook(hook(n)) for n, m in mods] if capture else []
        try:
            with torch.no_grad():
                mel = torch.from_numpy(np.load(os.path.join(HERE, "e2e_batch.npz"))["mel"])
                with cuda_autocast_bf16():
                    feat = codec.encoder(mel)
                    ret = codec.quantizer(feat)
                codes = ret.codes
                if capture:  # generator modules: the decode of clip 0's first GEN_FRAMES codes
                    with cuda_autocast_bf16():
                        codec.generator(codec.quantizer.decode(codes[:, :1, :GEN_FRAMES]))
                with cuda_autocast_bf16():
                    wav = codec.generator(codec.quantizer.decode(codes))
        finally:
            for h_ in hs:
                h_.remove()
        return dict(feat=feat, x_pjt_in=ret.x_pjt_in, codes=codes, wav=wav[:, 0])

    a = run(THREADS, capture=True)
    b = run(1)
    with torch.no_grad(), cuda_autocast_bf16():  # 1 thread, decoding the same (8-thread) codes
        wav1 = codec.generator(codec.quantizer.decode(a["codes"]))[:, 0]
    torch.set_num_threads(THREADS)
    with torch.no_grad(), cuda_autocast_bf16(wn64=True):  # the weight norm folded in fp64 (as the library)
        wav_wn = codec.generator(codec.quantizer.decode(a["codes"]))[:, 0]
    _store(d, "wav_wn64", wav_wn)
    d["wn64_dist_wav"] = np.float64(_rel(wav_wn, a["wav"]))
    for k in ("feat", "x_pjt_in", "wav"):  # the decode also with the fp64 weight-norm fold (wav_wn64)
        _store(d, k, a[k])
        d[f"spread_{k}"] = np.float64(_rel(b[k], a[k]))
    d["spread_wav_same_codes"] = np.float64(_rel(wav1, a["wav"]))
    d["codes"] = _np(a["codes"][0, :, :, 0]).astype(np.int64)
    d["spread_codes_equal"] = np.float64((a["codes"] == b["codes"]).double().mean())
    best, second, arg64 = R.top2_gap_fp64(a["x_pjt_in"].float(), embed)
    d.update(gap_best=_np(best), gap_second=_np(second), argmin_fp64=_np(arg64).reshape(d["codes"].shape))
    # per-module cases
    names = []
    for name, mod in mods:
        x = captured[name][:1]
        if not name.startswith("generator."):  # (B, C, T) except project_in's (B, T, C)
            x = x[:, :ENC_ROWS] if name.endswith("project_in") else x[..., :ENC_ROWS]
        x = x.contiguous()
        names.append(name)
        y = _bf16_module_forward(codec, name, mod, x)
        torch.set_num_threads(1)
        y1 = _bf16_module_forward(codec, name, mod, x)
        torch.set_num_threads(THREADS)
        ye = _bf16_module_forward(codec, name, mod, x, exact=True)
        yw = _bf16_module_forward(codec, name, mod, x, wn64=True) if name.startswith("generator.") else y
        with torch.no_grad():
            xf = x.float()
            if name == "generator.conv_post":
                yf = torch.tanh(codec.generator.conv_post(torch.nn.functional.silu(xf)))
            else:
                yf = mod(xf)
                if name.startswith("generator.resblocks.") and name.count(".") == 2:
                    yf = torch.nn.functional.silu(yf)
        _store(d, f"m:{name}:in", x)
        _store(d, f"m:{name}:out", y)
        if name.startswith("generator."):  # weight-normed convs: also the output with the library's fp64 fold
            _store(d, f"m:{name}:out_wn64", yw)
            d[f"m:{name}:wn64_dist"] = np.float64(_rel(yw, y))
        d[f"m:{name}:spread"] = np.float64(_rel(y1, y))
        d[f"m:{name}:exact_spread"] = np.float64(_rel(ye, y))
        d[f"m:{name}:fp32_dist"] = np.float64(_rel(yf, y))
        print(f"  {name:40s} in {tuple(x.shape)} {str(x.dtype):15s} out {str(y.dtype):15s} exact {d[f'm:{name}:exact_spread']:.2e}"
              f" fp32 {d[f'm:{name}:fp32_dist']:.2e}")
    d["module_names"] = np.array(names)
    d.update(threads=np.array(THREADS), seed=np.array(SEED), n_clips=np.array(ng))
    np.savez_compressed(os.path.join(HERE, "bf16.npz"), **d)
    print("bf16", {k: v.shape for k, v in d.items() if not k.startswith("m:")})


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "bf16":  # only the bf16 fixture (the others unchanged)
        torch.manual_seed(0)
        torch.set_num_threads(THREADS)
        codec, _ = build_reference()
        make_bf16(codec, np.load(os.path.join(HERE, "e2e_batch.npz"))["audio"])
    else:
        main()
