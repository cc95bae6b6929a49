"""The C-ABI library loads and exports every function declared in include/distilcodec_amd.h.
Host-only calls (no kernel launches), so this runs without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "distilcodec_amd.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dcx_[a-z_0-9]+)\s*\(", src)))


def test_header_symbols_exported_and_bound():
    from distilcodec_nabeel_amd import _native

    L = _native.lib()
    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
        assert n in _native.SIGNATURES, f"{n} has no ctypes signature"
    assert set(_native.SIGNATURES) == set(names)
    assert L.dcx_abi_version() == 4


def test_config_struct_matches_default(cfg):
    from distilcodec_nabeel_amd import _native

    L = _native.lib()
    a = _native.DcxConfig()
    L.dcx_default_config(ctypes.byref(a))
    b = _native.config_from_dict(cfg)
    assert bytes(a) == bytes(b)
    assert list(a.up_rates)[:5] == [8, 4, 2, 2, 2] and a.codebook_size == 32768


def test_host_queries_and_validation(cfg):
    from distilcodec_nabeel_amd import _native

    L = _native.lib()
    c = _native.config_from_dict(cfg)
    h = ctypes.c_void_p()
    assert L.dcx_create(ctypes.byref(c), ctypes.byref(h)) == 0
    try:
        # T = floor((N + 768 - 1024) / 256) + 1 on the padded length
        for n in (256, 24001, 72001, 240001):
            assert L.dcx_num_frames(h, n) == (n + 768 - 1024) // 256 + 1
        assert L.dcx_num_frames(h, 240001) == 937
        # the shortest padded clips the reflect pad accepts: frame count equals the oracle's STFT
        import torch
        from oracle import reference_cpu as R

        for n in (385, 386, 512, 640, 641, 1001, 3002):
            assert L.dcx_num_frames(h, n) == R.log_mel(torch.zeros(1, n)).shape[-1], n
        ws = L.dcx_workspace_size(h, 32, 937)
        # generator: 5 fp32 buffers + 8 bf16-planes buffers (6 bytes per value) of B*T*8192 values
        gen = (5 * 4 + 8 * 6) * 32 * 937 * 8192
        assert gen < ws < 1.2 * gen
        # a stage call before finalize is a state error, not a crash
        assert L.dcx_encode(h, None, 1, 10, None, None, 0, None) == _native.DCX_ERR_STATE
        # finalize validates every tensor before touching the device
        assert L.dcx_finalize(h, 1) == _native.DCX_ERR_MISSING_WEIGHT
        assert b"encoder.downsample_layers.0.0" in L.dcx_last_error(h)
        x = np.zeros((3,), np.float32)
        shape = (ctypes.c_int64 * 1)(3)
        assert L.dcx_set_tensor(h, b"encoder.norm.weight", x.ctypes.data_as(ctypes.c_void_p), 1, shape) == 0
        assert L.dcx_set_tensor(h, None, None, 1, shape) == _native.DCX_ERR_INVALID_ARG
    finally:
        L.dcx_destroy(h)
    bad = _native.config_from_dict(cfg)
    bad.codebook_size = 1000
    h2 = ctypes.c_void_p()
    assert L.dcx_create(ctypes.byref(bad), ctypes.byref(h2)) == _native.DCX_ERR_INVALID_ARG


def test_status_strings():
    from distilcodec_nabeel_amd import _native

    L = _native.lib()
    for st in range(0, -7, -1):
        assert L.dcx_status_string(st)
    assert L.dcx_transpose(None, None, 1, 1, 1, None) == _native.DCX_ERR_INVALID_ARG


def test_engine_refuses_cpu(cfg, state):
    from distilcodec_nabeel_amd import _native
    from distilcodec_nabeel_amd.engine import NativeCodec

    with pytest.raises(_native.NativeUnavailable):
        NativeCodec(cfg, state, "cpu")


def test_knobs_are_per_handle(cfg, monkeypatch):
    """A/B switches are read from the environment once, at dcx_create, and changed per handle by
    dcx_set_knob (round 5: no launcher reads the environment); unknown names are rejected."""
    from distilcodec_nabeel_amd import _native
    from distilcodec_nabeel_amd.engine import KNOB_DEFAULTS

    L = _native.lib()
    c = _native.config_from_dict(cfg)
    h = ctypes.c_void_p()
    assert L.dcx_create(ctypes.byref(c), ctypes.byref(h)) == 0
    try:
        for name, v in KNOB_DEFAULTS.items():
            assert L.dcx_set_knob(h, name.encode(), v) == 0, name
        assert L.dcx_set_knob(h, b"DCX_RP_OLD", 1) == 0
        assert L.dcx_set_knob(h, b"DCX_NOT_A_KNOB", 1) == _native.DCX_ERR_INVALID_ARG
        assert b"unknown knob" in L.dcx_last_error(h)
        assert L.dcx_set_knob(None, b"DCX_RP_OLD", 1) == _native.DCX_ERR_INVALID_ARG
    finally:
        L.dcx_destroy(h)
    # a handle created with a knob in the environment: still settable, and unknown module names are
    # rejected by the read-only dcx_module_io without writing the handle's error text
    monkeypatch.setenv("DCX_RP_W4", "1")
    h = ctypes.c_void_p()
    assert L.dcx_create(ctypes.byref(c), ctypes.byref(h)) == 0
    try:
        assert L.dcx_set_knob(h, b"DCX_RP_W4", 0) == 0
        before = L.dcx_last_error(h)
        ci, co, r = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        assert L.dcx_module_io(h, b"no.such.module", ctypes.byref(ci), ctypes.byref(co), ctypes.byref(r)) == \
            _native.DCX_ERR_INVALID_ARG
        assert L.dcx_last_error(h) == before
    finally:
        L.dcx_destroy(h)
