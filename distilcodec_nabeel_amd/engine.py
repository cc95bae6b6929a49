"""Device-side engine: one libdcx handle per GPU, torch tensors as device buffers.

Every method is stream-ordered on `torch.cuda.current_stream(device)` and hands raw device
pointers to the C ABI.  Tensors are channels-last ([B][T][C]) as the kernels produce them.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np
import torch

from . import _native
from .config import check_supported


# codebook EMA statistics a trained checkpoint carries (vector_quantize_pytorch.py:508-531); eval
# never reads them, and embed_avg alone is as large as the codebook (470 MB), so they are not copied
_TRAINING_ONLY = ("_codebook.embed_avg", "_codebook.cluster_size")

# dcx_set_knob switches and their shipped values (include/distilcodec_amd.h; dcx::Knobs)
KNOB_DEFAULTS = {
    "DCX_RP_R": 0, "DCX_RP_OLD": 0, "DCX_RP_G64": 0, "DCX_RP_SYNC": 0, "DCX_RP_W4": 0, "DCX_GELU_LUT": -1,
    "DCX_BF16_PERSIST": 1, "DCX_BF16_REG_EPI": 1, "DCX_DWCONV_TILED": 0, "DCX_SPLIT_MIN_STEPS": 0,
    "DCX_SPLIT_GROUP_OFF": 0, "DCX_H3": 1, "DCX_H3_BN": 0, "DCX_H3_1X1": 1, "DCX_H3_SPLIT": 1, "DCX_H3_PAIRS": 1, "DCX_RP_RING": 1,
    "DCX_ENC_STREAMS": 2,
}

GEMM_MODES = {"f32": _native.DCX_GEMM_F32, "x6": _native.DCX_GEMM_X6, "bf16": _native.DCX_GEMM_BF16}


class NativeCodec:
    """`gemm`: "x6" (default; fp32 operands as three bf16 planes, six exact products, fp32
    accumulation), "f32" (v_mfma_f32_32x32x2_f32) or "bf16" (the reference's enable_bfloat16:
    bf16 operands and results, fp32 accumulation; see DCX_GEMM_BF16).  Env DCX_GEMM overrides
    the default."""

    def __init__(self, cfg: dict, state: dict, device, with_generator: bool = True, gemm: str | None = None):
        check_supported(cfg)
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _native.NativeUnavailable("the DistilCodec MI355X path needs a GPU device (cuda:N on ROCm)")
        if not torch.cuda.is_available():
            raise _native.NativeUnavailable("no GPU visible to torch: the HIP path cannot run here")
        self.L = _native.lib()
        self.c = _native.config_from_dict(cfg)
        self.D = cfg["quantizer"]["input_dim"]
        self.CD = cfg["quantizer"]["codebook_dim"]
        self.NC = cfg["quantizer"]["codebook_size"]
        self.n_mels = cfg["spec_transform"]["num_mels"]
        self.hop = cfg["spec_transform"]["hop_size"]
        self.with_generator = with_generator
        self._ws = None
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_create(ctypes.byref(self.c), ctypes.byref(h)), None)
            self.h = h
            self.gemm = gemm or os.environ.get("DCX_GEMM", "x6")
            if self.gemm not in GEMM_MODES:
                raise ValueError(f"unknown GEMM mode {self.gemm!r}; expected one of {sorted(GEMM_MODES)}")
            self._check(self.L.dcx_set_gemm_mode(self.h, GEMM_MODES[self.gemm]))
            for part in ("encoder", "quantizer") + (("generator",) if with_generator else ()):
                for k, v in state[part].items():
                    if k.endswith(_TRAINING_ONLY):
                        continue
                    a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
                    shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
                    self._check(self.L.dcx_set_tensor(self.h, f"{part}.{k}".encode(), a.ctypes.data_as(ctypes.c_void_p),
                                                      a.ndim, shape))
            self._check(self.L.dcx_finalize(self.h, 1 if with_generator else 0))

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc, h="self"):
        if rc == _native.DCX_OK:
            return
        msg = ""
        handle = self.h if h == "self" else h
        if handle:
            msg = self.L.dcx_last_error(handle).decode()
        msg = msg or self.L.dcx_status_string(rc).decode()
        if rc == _native.DCX_ERR_INVALID_ARG:
            raise ValueError(msg)
        if rc == _native.DCX_ERR_MISSING_WEIGHT:
            raise KeyError(msg)
        raise _native.NativeError(rc, msg)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                self.L.dcx_destroy(h)
            except Exception:
                pass
            self.h = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def workspace_size(self, batch: int, frames: int) -> int:
        return int(self.L.dcx_workspace_size(self.h, batch, frames))

    def workspace(self, batch: int, frames: int, ws: torch.Tensor | None = None) -> torch.Tensor:
        """The workspace of one stage call.  A caller-owned `ws` (e.g. the one a captured hipGraph
        was recorded with) is checked and used as is; otherwise the engine's shared buffer, which
        grows (is reallocated) when a call needs more."""
        need = self.workspace_size(batch, frames)
        if ws is not None:
            if ws.device != self.device or ws.dtype != torch.uint8 or not ws.is_contiguous() or ws.numel() < need:
                raise ValueError(f"workspace must be a contiguous uint8 tensor on {self.device} of >= {need} bytes")
            return ws
        if self._ws is None or self._ws.numel() < need:
            self._ws = None
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    @staticmethod
    def _ptr(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def _dev(self, t, dtype):
        t = torch.as_tensor(t)
        if t.device != self.device or t.dtype != dtype or not t.is_contiguous():
            t = t.to(device=self.device, dtype=dtype).contiguous()
        return t

    def set_gemm(self, mode: str) -> None:
        self._check(self.L.dcx_set_gemm_mode(self.h, GEMM_MODES[mode]))
        self.gemm = mode

    def set_split_k(self, max_splits: int) -> None:
        """Split-K latency mode (dcx_set_split_k): few-tile convs run as up to `max_splits` K-slices.
        Opt-in for small batches; results then depend on the tile count (not batch-invariant)."""
        self._check(self.L.dcx_set_split_k(self.h, int(max_splits)))
        self._ws = None  # the workspace size changed

    def set_knob(self, name: str, value: int) -> None:
        """A/B and test switch of the kernel selection (dcx_set_knob; names are the DCX_* environment
        variables dcx_create reads once).  Takes effect for later calls on this engine."""
        self._check(self.L.dcx_set_knob(self.h, name.encode(), int(value)))

    def get_knob(self, name: str) -> int:
        """The current value of a switch (dcx_get_knob)."""
        v = ctypes.c_int32(0)
        self._check(self.L.dcx_get_knob(self.h, name.encode(), ctypes.byref(v)))
        return v.value

    @contextlib.contextmanager
    def knobs(self, **values):
        """Switches set for the calls inside the block, then back to the values they had before
        (an environment override given at creation included): `with eng.knobs(DCX_RP_OLD=1): ...`."""
        saved = {k: self.get_knob(k) for k in values}
        for k, v in values.items():
            self.set_knob(k, v)
        try:
            yield self
        finally:
            for k, v in saved.items():
                self.set_knob(k, v)

    def range_flags(self, reset: bool = False) -> int:
        """The h3 range flags (dcx_range_flags; synchronises): bit 0 a non-finite operand bound, bit 1
        a saturated h3 operand.  0 for every finite input."""
        v = ctypes.c_int32(0)
        self._check(self.L.dcx_range_flags(self.h, ctypes.byref(v), int(reset)))
        return v.value

    def num_frames(self, n_samples: int) -> int:
        return int(self.L.dcx_num_frames(self.h, n_samples))

    # ------------------------------------------------------------------ stages
    # Every stage takes an optional caller-owned workspace `ws` (see `workspace`): a captured hipGraph
    # must keep the buffer it was recorded with.
    def mel(self, audio: torch.Tensor, ws: torch.Tensor | None = None, linear: bool = False):
        """audio (B, N) fp32 (with the reference's leading zero) -> mel (B, T, n_mels); with
        `linear`, also log(clamp(|STFT|, 1e-5)) (B, T, n_fft/2 + 1) (return_linear, mel_spec.py:119-120)."""
        audio = self._dev(audio, torch.float32)
        B, N = audio.shape
        T = self.num_frames(N)
        out = torch.empty(B, T, self.n_mels, device=self.device)
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            if linear:
                lin = torch.empty(B, T, self.cfg["spec_transform"]["n_fft"] // 2 + 1, device=self.device)
                self._check(self.L.dcx_mel_linear(self.h, self._ptr(audio), B, N, self._ptr(out), self._ptr(lin),
                                                  self._ptr(ws), ws.numel(), self._stream()))
                return out, lin
            self._check(self.L.dcx_mel(self.h, self._ptr(audio), B, N, self._ptr(out), self._ptr(ws), ws.numel(), self._stream()))
        return out

    def encode(self, mel: torch.Tensor, ws: torch.Tensor | None = None) -> torch.Tensor:
        mel = self._dev(mel, torch.float32)
        B, T, _ = mel.shape
        out = torch.empty(B, T, self.cfg["encoder"]["dims"][-1], device=self.device)
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_encode(self.h, self._ptr(mel), B, T, self._ptr(out), self._ptr(ws), ws.numel(), self._stream()))
        return out

    def vq_encode(self, feat: torch.Tensor, want_pjt_in=True, want_fup=True, want_quantized=True,
                  ws: torch.Tensor | None = None):
        feat = self._dev(feat, torch.float32)
        B, T, _ = feat.shape
        codes = torch.empty(B, T, dtype=torch.int32, device=self.device)
        pin = torch.empty(B, T, self.CD, device=self.device) if want_pjt_in else None
        fup = torch.empty(B, T, self.CD, device=self.device) if want_fup else None
        q = torch.empty(B, T, self.D, device=self.device) if want_quantized else None
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_vq_encode(self.h, self._ptr(feat), B, T, self._ptr(codes), self._ptr(pin), self._ptr(fup),
                                             self._ptr(q), self._ptr(ws), ws.numel(), self._stream()))
        return codes, pin, fup, q

    def vq_decode(self, codes: torch.Tensor, ws: torch.Tensor | None = None) -> torch.Tensor:
        codes = self._dev(codes, torch.int32)
        B, T = codes.shape
        z = torch.empty(B, T, self.D, device=self.device)
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_vq_decode(self.h, self._ptr(codes), B, T, self._ptr(z), None, self._ptr(ws), ws.numel(),
                                             self._stream()))
        return z

    def generate(self, z: torch.Tensor, ws: torch.Tensor | None = None) -> torch.Tensor:
        if not self.with_generator:
            raise RuntimeError("this engine was built without generator weights")
        z = self._dev(z, torch.float32)
        B, T, _ = z.shape
        wav = torch.empty(B, self.hop * T, device=self.device)
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_generate(self.h, self._ptr(z), B, T, self._ptr(wav), self._ptr(ws), ws.numel(), self._stream()))
        return wav

    def encode_decode(self, audio: torch.Tensor, codes: torch.Tensor | None = None, wav: torch.Tensor | None = None,
                      ws: torch.Tensor | None = None):
        audio = self._dev(audio, torch.float32)
        B, N = audio.shape
        T = self.num_frames(N)
        if codes is None:
            codes = torch.empty(B, T, dtype=torch.int32, device=self.device)
        if wav is None:
            wav = torch.empty(B, self.hop * T, device=self.device)
        ws = self.workspace(B, T, ws)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_encode_decode(self.h, self._ptr(audio), B, N, self._ptr(codes), self._ptr(wav), self._ptr(ws),
                                                 ws.numel(), self._stream()))
        return codes, wav

    def module_io(self, name: str) -> tuple[int, int, int]:
        """(input channels, output channels (0: int32 codes), output rows per input row) of a module."""
        ci, co, r = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self.L.dcx_module_io(self.h, name.encode(), ctypes.byref(ci), ctypes.byref(co), ctypes.byref(r)))
        return ci.value, co.value, r.value

    def module(self, name: str, x: torch.Tensor) -> torch.Tensor:
        """One reference module by its state-dict prefix (dcx_module_forward): x channels-last
        (B, L, C) fp32 -> y (see the header for shapes; int32 codes for "quantizer.search").
        ValueError for an unknown name or an input whose channel count is not the module's."""
        cin, cout, rate = self.module_io(name)
        x = self._dev(x, torch.float32)
        if x.ndim != 3 or x.shape[2] != cin:
            raise ValueError(f"{name} takes (B, L, {cin}) input, got {tuple(x.shape)}")
        B, L, C = x.shape
        n = name.encode()
        need = int(self.L.dcx_module_workspace_size(self.h, n, B, L))
        if need == 0:
            raise ValueError(f"module {name!r} cannot run on this handle")
        if cout == 0:
            y = torch.empty(B, L, dtype=torch.int32, device=self.device)
        else:
            y = torch.empty(B, L * rate, cout, device=self.device)
        ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self.L.dcx_module_forward(self.h, n, self._ptr(x), B, L, C, self._ptr(y), self._ptr(ws), ws.numel(),
                                                  self._stream()))
        return y

    def transpose(self, x: torch.Tensor) -> torch.Tensor:
        """(B, R, C) -> (B, C, R) contiguous, on device, by the HIP transpose kernel."""
        x = self._dev(x, torch.float32)
        B, R, C = x.shape
        out = torch.empty(B, C, R, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.L.dcx_transpose(self._ptr(x), self._ptr(out), B, R, C, self._stream())
        if rc != _native.DCX_OK:
            raise _native.NativeError(rc, "dcx_transpose failed")
        return out

    # ------------------------------------------------------------------ profiling
    def profile(self, on: bool):
        self._check(self.L.dcx_profile_enable(self.h, 1 if on else 0))

    def vq_rescore_stats(self, reset: bool = False) -> tuple[int, int]:
        """(rows rescored, codes rescored) by the x6 VQ search since the last reset (synchronises)."""
        import ctypes
        r, c = ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self.L.dcx_vq_rescore_stats(self.h, ctypes.byref(r), ctypes.byref(c), int(reset)))
        return r.value, c.value

    def profile_reset(self):
        self._check(self.L.dcx_profile_reset(self.h))

    def profile_read(self) -> dict:
        out = {}
        n = self.L.dcx_profile_count(self.h)
        for i in range(n):
            name = ctypes.c_char_p()
            launches = ctypes.c_int64()
            ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            self._check(self.L.dcx_profile_read(self.h, i, ctypes.byref(name), ctypes.byref(launches), ctypes.byref(ms),
                                                ctypes.byref(fl), ctypes.byref(by)))
            out[name.value.decode()] = {"launches": launches.value, "ms": ms.value, "flops": fl.value, "bytes": by.value}
        return out


class NativeConv:
    """The conv primitive of libdcx (dcx_conv_*): Conv1d ("same" padding, dilation) or
    ConvTranspose1d (padding (k-stride)/2) on channels-last fp32 tensors."""

    def __init__(self, weight: np.ndarray, bias=None, dilation: int = 1, transposed: bool = False, stride: int = 1):
        self.L = _native.lib()
        w = np.ascontiguousarray(weight, dtype=np.float32)
        if transposed:
            self.cin, self.cout, self.k = w.shape
        else:
            self.cout, self.cin, self.k = w.shape
        b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
        self.stride = stride if transposed else 1
        self._b = b
        h = ctypes.c_void_p()
        rc = self.L.dcx_conv_create(w.ctypes.data_as(ctypes.c_void_p), None if b is None else b.ctypes.data_as(ctypes.c_void_p),
                                    self.cin, self.cout, self.k, dilation, 1 if transposed else 0, stride, ctypes.byref(h))
        if rc != _native.DCX_OK:
            raise ValueError(f"dcx_conv_create failed: {self.L.dcx_status_string(rc).decode()}")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.L.dcx_conv_destroy(h)
            self.h = None

    def __call__(self, x: torch.Tensor, gemm: str = "x6", epi: int = 0, res: torch.Tensor | None = None,
                 want_y: bool = True, want_silu: bool = False):
        B, Lin, C = x.shape
        assert C == self.cin and x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
        Lout = Lin * self.stride
        y = torch.empty(B, Lout, self.cout, device=x.device) if want_y else None
        ys = torch.empty(B, Lout, self.cout, device=x.device) if want_silu else None
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        rc = self.L.dcx_conv_forward(self.h, GEMM_MODES[gemm], ptr(x), B, Lin, ptr(y), ptr(ys), ptr(res), epi,
                                     ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != _native.DCX_OK:
            raise _native.NativeError(rc, "dcx_conv_forward failed")
        return (y, ys) if want_silu else y
