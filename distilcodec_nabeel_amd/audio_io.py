"""WAV file I/O for the path-input mode of `DistilCodec.encode` (host-only).

The reference reads files with `librosa.load(path, sr=24000)` (`distilcodec/models/meldataset.py:18-20`)
and writes them with `soundfile.write` (`distil_codec.py:640-654`); neither library exists in this
image.  This module reads/writes RIFF/WAVE PCM (8/16/24/32-bit integer and 32-bit float) with the
standard library, scaling integers like libsndfile (int16 / 32768) and averaging channels to mono
like librosa.  A file at another rate is resampled on the GPU by `resample.py` (a polyphase FIR in
scipy.signal.resample_poly's form, not librosa's soxr_hq).
"""
from __future__ import annotations

import struct
import wave

import numpy as np


def _read_float_wav(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8: pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    tag, ch, sr, _, _, bits = fmt
    if tag != 3 or bits not in (32, 64):
        raise ValueError(f"{path}: unsupported WAVE format tag {tag} / {bits} bit")
    x = np.frombuffer(payload, dtype="<f4" if bits == 32 else "<f8").astype(np.float32)
    return x.reshape(-1, ch), sr


def read_wav(path: str) -> tuple[np.ndarray, int]:
    """Returns (float32 array (frames, channels), sample_rate)."""
    try:
        with wave.open(path, "rb") as w:
            ch, width, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
            raw = w.readframes(n)
    except wave.Error:
        return _read_float_wav(path)
    if width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        x = np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"{path}: unsupported sample width {width}")
    return x.reshape(-1, ch), sr


def _is_mp3(head: bytes) -> bool:
    """ID3v2 tag or an MPEG audio frame sync (11 set bits) at the start of the file."""
    return head[:3] == b"ID3" or (len(head) >= 2 and head[0] == 0xFF and (head[1] & 0xE0) == 0xE0)


def read_audio(path: str) -> tuple[np.ndarray, int]:
    """(float32 (frames, channels), sample_rate) of a WAV or MP3 file, chosen by its leading bytes
    (librosa.load reads both; meldataset.py:18-20)."""
    with open(path, "rb") as f:
        head = f.read(4)
    if head[:4] != b"RIFF" and _is_mp3(head):
        from . import mp3

        return mp3.read_mp3(path)
    return read_wav(path)


def load_audio_mono(path: str) -> tuple[np.ndarray, int]:
    """Mono float32 samples (channel mean, as librosa.load(mono=True)) and the file's rate."""
    x, file_sr = read_audio(path)
    x = x.mean(axis=1) if x.shape[1] > 1 else x[:, 0]
    return np.ascontiguousarray(x, dtype=np.float32), file_sr


def load_wav_mono(path: str) -> tuple[np.ndarray, int]:
    """Mono float32 samples (channel mean, as librosa.load(mono=True)) and the file's rate."""
    x, file_sr = read_wav(path)
    x = x.mean(axis=1) if x.shape[1] > 1 else x[:, 0]
    return np.ascontiguousarray(x, dtype=np.float32), file_sr


def load_wav(path: str, sr: int) -> tuple[np.ndarray, int]:
    """`load_wav(full_path, sr)` (meldataset.py:18-20): mono float32 at `sr`, resampled on the GPU
    (distilcodec_nabeel_amd/resample.py) when the file has another rate."""
    x, file_sr = load_audio_mono(path)
    if file_sr != sr:
        from . import resample

        x = resample.resample(x, file_sr, sr).cpu().numpy()
    return x, sr


def write_wav(path: str, audio: np.ndarray, sr: int) -> None:
    """PCM_16 mono WAV, clipping like libsndfile's float->int16 conversion."""
    a = np.clip(np.asarray(audio, np.float64), -1.0, 1.0)
    pcm = np.clip(np.round(a * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())
