"""MP3 input for the file front end (`librosa.load`'s MPEG path: distilcodec/models/meldataset.py:18-20,
distil_codec.py:667; C1's `test.mp3`, README.md:116).

Decoding is the host MPEG-1 Layer III decoder in libdcx.so (`csrc/dcx_mp3.cpp`, `dcx_mp3_info` /
`dcx_mp3_decode`), with Xing/LAME gapless trimming like mpg123 and ffmpeg.  No reference decoder is
importable here (librosa, audioread, soundfile, ffmpeg are absent), so parity with the reference's
decoder is unpinned; tests/test_mp3.py checks the code books, the synthesis window and the decode of
test.mp3 by properties.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native


class Mp3Error(ValueError):
    """The data is not a decodable MPEG audio stream (what librosa would also fail to read)."""


class Mp3Unsupported(Mp3Error):
    """A valid MPEG audio stream using a feature this decoder lacks (MPEG-2/2.5, Layer I/II, free
    format, intensity stereo).  librosa would decode it, so callers must not treat it as an
    unreadable file: `DistilCodec.encode` re-raises it instead of substituting noise."""


def _raise(L, rc):
    msg = L.dcx_mp3_last_error().decode()
    raise (Mp3Unsupported if rc == _native.DCX_ERR_UNSUPPORTED else Mp3Error)(msg)


def decode_mp3_bytes(data: bytes) -> tuple[np.ndarray, int]:
    """(float32 (samples, channels), sample_rate) of an MPEG-1 Layer III stream."""
    L = _native.lib()
    buf = ctypes.create_string_buffer(data, len(data))
    n, sr, ch = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
    rc = L.dcx_mp3_info(buf, len(data), ctypes.byref(n), ctypes.byref(sr), ctypes.byref(ch))
    if rc != 0:
        _raise(L, rc)
    out = np.zeros((ch.value, max(n.value, 1)), np.float32)
    rc = L.dcx_mp3_decode(buf, len(data), out.ctypes.data, n.value)
    if rc != 0:
        _raise(L, rc)
    return np.ascontiguousarray(out[:, : n.value].T), sr.value


def read_mp3(path: str) -> tuple[np.ndarray, int]:
    with open(path, "rb") as f:
        return decode_mp3_bytes(f.read())


def last_stats() -> tuple[int, int]:
    """(granules decoded, granules whose Huffman data ended exactly at part2_3_length) of the last
    decode on this thread."""
    g, e = ctypes.c_int64(), ctypes.c_int64()
    _native.lib().dcx_mp3_stats(ctypes.byref(g), ctypes.byref(e))
    return g.value, e.value


def last_junk_bytes() -> int:
    """Bytes the last decode on this thread skipped to resync on a frame header (0: clean stream)."""
    return int(_native.lib().dcx_mp3_junk_bytes())


def last_bad_frames() -> int:
    """Frames of the last decode on this thread whose data was damaged; they decode as silence."""
    return int(_native.lib().dcx_mp3_bad_frames())
