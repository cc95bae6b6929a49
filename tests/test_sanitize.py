"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizer runs of
the host code on the CPU build).  `make -C distilcodec_nabeel_amd/csrc sanitize` builds
tests/sanitize/host_driver.cpp against dcx_api.cpp and dcx_mp3.cpp instrumented on the host (the
kernels as built).  The driver exercises the C ABI's argument checks, checkpoint ingestion (name and
shape validation, weight packing up to the first device allocation), workspace planning for 35
shapes x 3 arithmetic modes x split-K on/off, the conv primitive's checks, and the MP3 decoder on
the reference's test.mp3, its prefixes, 400 corrupted copies and random garbage.  Any sanitizer
report aborts the driver (-fno-sanitize-recover=all).  On a GPU box the same driver also finalizes
the handle and runs a small encode_decode through the instrumented host runtime."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "distilcodec_nabeel_amd", "csrc")
DRIVER = os.path.join(REPO, "distilcodec_nabeel_amd", "dcx_asan_driver")
MP3 = os.path.join(REPO, "tests", "golden", "test.mp3")


@pytest.fixture(scope="module")
def driver():
    # make is a no-op when the driver is up to date (build() makes it too).  The driver is a test-only
    # artifact: without the host sanitizer runtimes it cannot be built, and these tests skip.
    r = subprocess.run(["make", "-C", CSRC, "-j8", "sanitize"], capture_output=True, text=True, timeout=900)
    if r.returncode != 0 or not os.path.exists(DRIVER):
        pytest.skip("the ASan/UBSan host driver does not build here: " + (r.stderr or "")[-400:])
    return DRIVER


def _run(driver, args, leaks, timeout=240):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = f"detect_leaks={int(leaks)}:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([driver] + args, capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_mp3_decoder_under_asan(driver):
    out = _run(driver, ["mp3", MP3], leaks=True)
    assert "400 corrupted" in out


def _specs(state, path):
    with open(path, "w") as f:
        for part in ("encoder", "quantizer", "generator"):
            for k, v in state[part].items():
                f.write(f"{part}.{k} {v.ndim} {' '.join(map(str, v.shape))}\n")


def test_host_runtime_under_asan(driver, state, tmp_path):
    spec = tmp_path / "tensors.txt"
    _specs(state, spec)
    # the HIP runtime's own allocations outlive main: leak checking covers the MP3 run only
    out = _run(driver, ["abi", str(spec)], leaks=False)
    assert "plans checked" in out


@pytest.mark.gpu
def test_host_runtime_under_asan_gpu(state, tmp_path):
    """The same driver with a GPU: finalize (packing, decode-table build) and a 2 x 1 s encode_decode
    through the instrumented host runtime."""
    if not os.path.exists(DRIVER):
        pytest.skip("the sanitizer driver was not built (make -C distilcodec_nabeel_amd/csrc sanitize failed)")
    spec = tmp_path / "tensors.txt"
    _specs(state, spec)
    out = _run(DRIVER, ["abi", str(spec)], leaks=False, timeout=200)
    assert "GPU present" in out and "plans checked" in out
