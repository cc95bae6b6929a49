"""MP3 front end (csrc/dcx_mp3.cpp; replaces librosa.load's MP3 path, meldataset.py:18-20,
distil_codec.py:667, for C1's test.mp3, README.md:116).

No MP3 decoder exists in this image to compare with (librosa, audioread, soundfile, ffmpeg, mpg123
are absent), so parity with the reference's decoder is unpinned and the decoder is checked by
properties of the standard it restates:
  * every Huffman code book of ISO/IEC 11172-3 Annex B is prefix-free and complete (Kraft sum 1);
  * the synthesis window D[i] (Table 3-B.3) gives a prototype lowpass at -3.01 dB at pi/64 with more
    than 100 dB stop-band attenuation, and the standard's analysis filterbank (window D / 32)
    followed by the decoder's synthesis reconstructs a signal to >= 80 dB (the filterbank is near-PR);
  * decoding tests/golden/test.mp3 (the reference's own demo input, 88 LAME VBR frames): every one of
    its 176 granules ends its Huffman data exactly at part2_3_length, gapless trimming gives the
    LAME tag's length (88 * 1152 - 576 - 1472 samples), and nothing above LAME's lowpass comes out;
  * the decoded samples are pinned by checksums (regression only: computed by this decoder).
These run on the CPU: the decoder is host code inside libdcx.so.
"""
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "distilcodec_nabeel_amd", "csrc", "dcx_mp3.cpp")
MP3 = os.path.join(REPO, "tests", "golden", "test.mp3")


def _arrays(name_re):
    src = open(SRC).read()
    out = {}
    for m in re.finditer(r"const (?:uint16_t|uint8_t|int32_t) " + name_re + r"\[\d*\] = \{([^}]*)\};", src):
        out[m.group(1)] = [int(v) for v in m.group(2).replace("\n", " ").split(",") if v.strip()]
    return out


def test_code_books_prefix_free_and_complete():
    from fractions import Fraction

    arr = _arrays(r"(kH\d+[cl]|kQA[cl])")
    books = sorted({k[:-1] for k in arr})
    assert len(books) == 16  # 15 pair books + count1 table A
    for b in books:
        codes, lens = arr[b + "c"], arr[b + "l"]
        assert len(codes) == len(lens)
        assert all(0 <= c < (1 << n) for c, n in zip(codes, lens)), b
        assert sum(Fraction(1, 1 << n) for n in lens) == 1, b
        words = sorted(format(c, f"0{n}b") for c, n in zip(codes, lens))
        assert all(not words[i + 1].startswith(words[i]) for i in range(len(words) - 1)), b


def _window():
    d = np.array(_arrays(r"(kDwin)")["kDwin"], np.float64) / 65536.0
    assert len(d) == 257
    D = np.zeros(512)
    D[:257] = d
    for i in range(1, 256):
        D[512 - i] = (1.0 if i % 64 == 0 else -1.0) * D[i]
    return D


def test_synthesis_window_prototype():
    D = _window()
    c = D * np.array([-1.0 if (i // 64) % 2 else 1.0 for i in range(512)])  # the smooth prototype
    assert np.allclose(c[1:256], c[511:256:-1])
    H = np.abs(np.fft.rfft(c, 1 << 16))
    H /= H[0]
    at = lambda f: 20 * np.log10(H[int(round(f / 2 * (1 << 16)))])  # noqa: E731  (f in units of pi)
    assert abs(at(1 / 64) + 3.01) < 0.02
    assert 20 * np.log10(H[int(1.5 / 32 / 2 * (1 << 16)):].max()) < -100


def test_analysis_synthesis_reconstruction():
    """The standard's analysis (C = D / 32, M[k][i] = cos((2k+1)(i-16)pi/64)) followed by the
    decoder's synthesis (V = N S, N[i][k] = cos((16+i)(2k+1)pi/64); U from V; sum of U * D):
    near-perfect reconstruction, 481 samples of delay."""
    D = _window()
    C = D / 32
    x = np.random.default_rng(0).standard_normal(32 * 120)
    M = np.cos(np.outer(2 * np.arange(32) + 1, np.arange(64) - 16) * np.pi / 64)
    N = np.cos(np.outer(16 + np.arange(64), 2 * np.arange(32) + 1) * np.pi / 64)
    X = np.zeros(512)
    V = np.zeros(1024)
    y = []
    for t in range(0, len(x), 32):
        X = np.concatenate([x[t:t + 32][::-1], X[:-32]])
        Z = C * X
        S = M @ Z.reshape(8, 64).sum(axis=0)
        V = np.concatenate([N @ S, V[:-64]])
        U = np.concatenate([np.concatenate([V[128 * i:128 * i + 32], V[128 * i + 96:128 * i + 128]]) for i in range(8)])
        y.append((U * D).reshape(16, 32).sum(axis=0))
    y = np.concatenate(y)
    a, b = x[: len(y) - 481], y[481:]
    snr = 10 * np.log10((a @ a) / ((b - a) @ (b - a)))
    assert snr >= 80, snr


def test_decode_reference_demo_input():
    from distilcodec_nabeel_amd import audio_io, mp3

    x, sr = mp3.read_mp3(MP3)
    granules, exact = mp3.last_stats()
    assert (granules, exact) == (176, 176)
    assert sr == 44100 and x.shape == (88 * 1152 - 576 - 1472, 1)
    assert np.isfinite(x).all() and np.abs(x).max() < 1.0
    X = np.abs(np.fft.rfft(x[:, 0].astype(np.float64) * np.hanning(len(x)))) ** 2
    f = np.fft.rfftfreq(len(x), 1 / sr)
    assert 10 * np.log10(X[f > 17000].sum() / X.sum()) < -80  # LAME's lowpass: nothing above it
    x64 = x.astype(np.float64)
    assert abs(x64.sum() - -34.50062952920567) < 1e-3
    assert abs((x64 ** 2).sum() / 237.7427061618785 - 1) < 1e-6
    y, sr2 = audio_io.read_audio(MP3)  # dispatch by leading bytes
    assert sr2 == sr and np.array_equal(y, x)


def test_truncated_and_garbage_input():
    from distilcodec_nabeel_amd import mp3

    data = open(MP3, "rb").read()
    y, sr = mp3.decode_mp3_bytes(data[: len(data) // 2])
    assert sr == 44100 and 0 < len(y) < 88 * 1152 - 576 - 1472
    with pytest.raises(mp3.Mp3Error):
        mp3.decode_mp3_bytes(bytes(range(256)) * 8)


def _frame_offsets(data: bytes) -> list:
    """Offsets of the MPEG-1 Layer III frames after the ID3v2 tag (test helper)."""
    rates, kbps = (44100, 48000, 32000), (0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320)
    i = 0
    if data[:3] == b"ID3":
        i = 10 + ((data[6] & 127) << 21 | (data[7] & 127) << 14 | (data[8] & 127) << 7 | (data[9] & 127))
    out = []
    while i + 4 <= len(data) and data[i] == 0xFF and (data[i + 1] & 0xFE) == 0xFA:
        out.append(i)
        i += 144000 * kbps[data[i + 2] >> 4] // rates[(data[i + 2] >> 2) & 3] + ((data[i + 2] >> 1) & 1)
    return out


def test_junk_between_frames_resyncs():
    """Junk inside the stream: the decoder skips it like mpg123 / ffmpeg, resyncing on the
    next header that the following header confirms; a clean frame boundary gives the same samples."""
    from distilcodec_nabeel_amd import mp3

    data = open(MP3, "rb").read()
    clean, sr = mp3.decode_mp3_bytes(data)
    assert mp3.last_junk_bytes() == 0
    offs = _frame_offsets(data)
    assert len(offs) >= 80
    junk = np.random.RandomState(3).randint(0, 256, 517).astype(np.uint8).tobytes()
    k = offs[40]
    y, sr2 = mp3.decode_mp3_bytes(data[:k] + junk + data[k:])
    assert mp3.last_junk_bytes() == 517 and mp3.last_bad_frames() == 0 and sr2 == sr
    assert np.array_equal(y, clean)
    # junk cutting frame 40 short: its header still declares a full frame, whose tail is junk; the scan
    # resyncs on frame 41.  Damaged frames decode as silence (error concealment), the stream goes on
    # with the same length, and the audio before the damage is unchanged.
    y2, _ = mp3.decode_mp3_bytes(data[:k + 100] + junk + data[offs[41]:])
    assert mp3.last_junk_bytes() > 0 and len(y2) == len(clean)
    n_ok = 38 * 1152 - (576 + 1152 - 529)  # whole frames before the damage, after the gapless skip
    assert np.array_equal(y2[:n_ok], clean[:n_ok])
    assert np.isfinite(y2).all()


@pytest.mark.parametrize("header,what", [
    (b"\xff\xf3\x64\xc4", "MPEG-2 Layer III"),
    (b"\xff\xe3\x64\xc4", "MPEG-2.5 Layer III"),
    (b"\xff\xfd\x94\x44", "MPEG-1 Layer II"),
    (b"\xff\xfb\x04\x44", "MPEG-1 Layer III free format"),
])
def test_unsupported_streams_raise_loudly(tmp_path, cfg, header, what):
    """MPEG audio of a kind the host decoder lacks raises Mp3Unsupported, and the path-input encode
    re-raises it instead of substituting noise (librosa would decode these files)."""
    from distilcodec_nabeel_amd import DistilCodec, mp3

    data = (header + bytes(400)) * 20
    with pytest.raises(mp3.Mp3Unsupported):
        mp3.decode_mp3_bytes(data)
    p = tmp_path / "lsf.mp3"
    p.write_bytes(b"ID3\x03\x00\x00\x00\x00\x00\x00" + data)
    with pytest.raises(mp3.Mp3Unsupported):
        DistilCodec(cfg)._read_audio_files([str(p)])
    # a corrupt file is still an ordinary read failure (the reference's noise fallback applies)
    with pytest.raises(mp3.Mp3Error) as e:
        mp3.decode_mp3_bytes(b"\xff\xfb\xf0\x00" + bytes(300))
    assert not isinstance(e.value, mp3.Mp3Unsupported)
