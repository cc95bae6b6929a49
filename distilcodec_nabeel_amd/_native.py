"""ctypes binding of the C ABI in include/distilcodec_amd.h (libdcx.so, built for gfx950).

There is no fallback: if the library is missing or fails to load, every product entry point
raises `NativeUnavailable`.  torch is imported first on purpose: libdcx.so links the HIP runtime
by soname (libamdhip64.so.7), so it binds to the copy torch has already loaded and both share
one runtime, one device context and torch's streams.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os

import torch  # noqa: F401  (see module docstring)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCX_LIB") or os.path.join(_PKG, "libdcx.so")
CSRC = os.path.join(_PKG, "csrc")
HEADER = os.path.join(os.path.dirname(_PKG), "include", "distilcodec_amd.h")

DCX_OK = 0
DCX_ERR_INVALID_ARG = -1
DCX_ERR_MISSING_WEIGHT = -2
DCX_ERR_STATE = -3
DCX_ERR_HIP = -4
DCX_ERR_OOM = -5
DCX_ERR_WORKSPACE = -6
DCX_ERR_UNSUPPORTED = -7
DCX_GEMM_F32 = 0
DCX_GEMM_X6 = 1
DCX_GEMM_BF16 = 2


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"dcx status {status}: {msg}")
        self.status = status


class DcxConfig(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32),
        ("n_fft", ctypes.c_int32), ("hop", ctypes.c_int32), ("win", ctypes.c_int32),
        ("n_mels", ctypes.c_int32),
        ("f_min", ctypes.c_float), ("f_max", ctypes.c_float),
        ("enc_depths", ctypes.c_int32 * 4), ("enc_dims", ctypes.c_int32 * 4),
        ("vq_dim", ctypes.c_int32), ("codebook_dim", ctypes.c_int32), ("codebook_size", ctypes.c_int32),
        ("gen_channels", ctypes.c_int32), ("gen_pre_k", ctypes.c_int32), ("gen_post_k", ctypes.c_int32),
        ("n_ups", ctypes.c_int32), ("up_rates", ctypes.c_int32 * 8), ("up_kernels", ctypes.c_int32 * 8),
        ("n_res", ctypes.c_int32), ("res_kernels", ctypes.c_int32 * 4),
        ("res_dilations", (ctypes.c_int32 * 4) * 4),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); must list every function declared in include/distilcodec_amd.h
SIGNATURES = {
    "dcx_default_config": (None, [ctypes.POINTER(DcxConfig)]),
    "dcx_create": (ctypes.c_int, [ctypes.POINTER(DcxConfig), ctypes.POINTER(_P)]),
    "dcx_destroy": (None, [_P]),
    "dcx_last_error": (ctypes.c_char_p, [_P]),
    "dcx_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "dcx_abi_version": (ctypes.c_int, []),
    "dcx_build_id": (ctypes.c_char_p, []),
    "dcx_set_tensor": (ctypes.c_int, [_P, ctypes.c_char_p, _P, _I32, ctypes.POINTER(_I64)]),
    "dcx_finalize": (ctypes.c_int, [_P, _I32]),
    "dcx_num_frames": (_I64, [_P, _I64]),
    "dcx_workspace_size": (_SZ, [_P, _I32, _I64]),
    "dcx_mel": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _SZ, _P]),
    "dcx_mel_linear": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _SZ, _P]),
    "dcx_encode": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _SZ, _P]),
    "dcx_vq_encode": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "dcx_vq_decode": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _SZ, _P]),
    "dcx_generate": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _SZ, _P]),
    "dcx_encode_decode": (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _SZ, _P]),
    "dcx_transpose": (ctypes.c_int, [_P, _P, _I32, _I64, _I64, _P]),
    "dcx_mp3_info": (ctypes.c_int, [_P, _SZ, ctypes.POINTER(_I64), ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "dcx_mp3_decode": (ctypes.c_int, [_P, _SZ, _P, _I64]),
    "dcx_mp3_last_error": (ctypes.c_char_p, []),
    "dcx_mp3_stats": (ctypes.c_int, [ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "dcx_mp3_junk_bytes": (_I64, []),
    "dcx_mp3_bad_frames": (_I64, []),
    "dcx_resample_poly": (ctypes.c_int, [_P, _I32, _I64, _I64, _P, _I32, _I32, _I32, _I64, _P, _I64, _I64, _P]),
    "dcx_set_gemm_mode": (ctypes.c_int, [_P, _I32]),
    "dcx_get_gemm_mode": (_I32, [_P]),
    "dcx_set_split_k": (ctypes.c_int, [_P, _I32]),
    "dcx_set_knob": (ctypes.c_int, [_P, ctypes.c_char_p, _I32]),
    "dcx_get_knob": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.POINTER(_I32)]),
    "dcx_range_flags": (ctypes.c_int, [_P, ctypes.POINTER(_I32), _I32]),
    "dcx_conv_create": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "dcx_conv_forward": (ctypes.c_int, [_P, _I32, _P, _I32, _I64, _P, _P, _P, _I32, _P]),
    "dcx_conv_destroy": (None, [_P]),
    "dcx_module_workspace_size": (_SZ, [_P, ctypes.c_char_p, _I32, _I64]),
    "dcx_module_io": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.POINTER(_I32), ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "dcx_module_forward": (ctypes.c_int, [_P, ctypes.c_char_p, _P, _I32, _I64, _I32, _P, _P, _SZ, _P]),
    "dcx_vq_rescore_stats": (ctypes.c_int, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), _I32]),
    "dcx_profile_enable": (ctypes.c_int, [_P, _I32]),
    "dcx_profile_reset": (ctypes.c_int, [_P]),
    "dcx_profile_count": (_I32, [_P]),
    "dcx_profile_read": (ctypes.c_int, [_P, _I32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I64),
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double)]),
}

_lib = None


def source_build_id() -> str | None:
    """The hash csrc/Makefile embeds in libdcx.so: SHA-256 over the library's sources in sorted
    order (csrc/*.cpp, *.hip, *.h), then include/distilcodec_amd.h; first 16 hex digits.  None when
    the sources are not next to the library."""
    names = sorted(os.path.basename(p) for ext in ("cpp", "hip", "h") for p in glob.glob(os.path.join(CSRC, f"*.{ext}")))
    if not names or not os.path.isfile(HEADER):
        return None
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, n) for n in names] + [HEADER]:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib() -> ctypes.CDLL:
    """Load libdcx.so once; raise NativeUnavailable (never fall back) when it cannot be used."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise NativeUnavailable(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.dcx_abi_version() != 4:
        raise NativeUnavailable("libdcx.so ABI version mismatch")
    # A library selected explicitly with DCX_LIB (A/B tooling, diagnostic builds) is taken as is;
    # the in-tree library must have been built from the sources next to it.
    if not os.environ.get("DCX_LIB"):
        want, have = source_build_id(), L.dcx_build_id().decode()
        if want is not None and have != want:
            raise NativeUnavailable(f"{LIB_PATH} is stale: built from sources {have}, the sources here hash to {want}; "
                                    f"rebuild with `make -C {CSRC}`")
    _lib = L
    return L


def config_from_dict(cfg: dict) -> DcxConfig:
    c = DcxConfig()
    lib().dcx_default_config(ctypes.byref(c))
    s, e, d, q = cfg["spec_transform"], cfg["encoder"], cfg["decoder"], cfg["quantizer"]
    c.sample_rate, c.n_fft, c.hop, c.win = s["sampling_rate"], s["n_fft"], s["hop_size"], s["win_size"]
    c.n_mels, c.f_min, c.f_max = s["num_mels"], float(s["fmin"]), float(s["fmax"] or s["sampling_rate"] // 2)
    for i in range(4):
        c.enc_depths[i], c.enc_dims[i] = e["depths"][i], e["dims"][i]
    c.vq_dim, c.codebook_dim, c.codebook_size = q["input_dim"], q["codebook_dim"], q["codebook_size"]
    c.gen_channels, c.gen_pre_k, c.gen_post_k = d["upsample_initial_channel"], d["pre_conv_kernel_size"], d["post_conv_kernel_size"]
    c.n_ups = len(d["upsample_rates"])
    for i, (u, k) in enumerate(zip(d["upsample_rates"], d["upsample_kernel_sizes"])):
        c.up_rates[i], c.up_kernels[i] = u, k
    c.n_res = len(d["resblock_kernel_sizes"])
    for i, (k, dl) in enumerate(zip(d["resblock_kernel_sizes"], d["resblock_dilation_sizes"])):
        c.res_kernels[i] = k
        for j, v in enumerate(dl):
            c.res_dilations[i][j] = v
    return c
