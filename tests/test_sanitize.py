"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizer runs of
the host code on the CPU build).  `make -C distilcodec_nabeel_amd/csrc sanitize` builds
tests/sanitize/host_driver.cpp against dcx_api.cpp and dcx_mp3.cpp instrumented on the host (the
kernels as built).  The driver exercises the C ABI's argument checks, checkpoint ingestion (name and
shape validation, weight packing up to the first device allocation), workspace planning for 35
shapes x 3 arithmetic modes x split-K on/off, the conv primitive's checks, and the MP3 decoder on
the reference's test.mp3, its prefixes, 400 corrupted copies and random garbage.  Any sanitizer
report aborts the driver (-fno-sanitize-recover=all).  Sanitizers run on the CPU build only: GPU
sanitizer runs are not available on the GPU pool, and the host runtime's paths are covered here."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "distilcodec_nabeel_amd", "csrc")
DRIVER = os.path.join(REPO, "distilcodec_nabeel_amd", "dcx_asan_driver")
MP3 = os.path.join(REPO, "tests", "golden", "test.mp3")


def _sanitizer_runtime_available(tmp) -> bool:
    """Whether hipcc can link a host program with ASan + UBSan at all (the runtimes are part of the
    toolchain install, not of this repository)."""
    src = os.path.join(tmp, "probe.cpp")
    with open(src, "w") as f:
        f.write("int main() { return 0; }\n")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-fno-gpu-sanitize", "-fsanitize=address", "-fsanitize=undefined", src,
                        "-o", os.path.join(tmp, "probe")], capture_output=True, text=True, timeout=300)
    return r.returncode == 0


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    # make is a no-op when the driver is up to date (build() makes it too).  Skipped only when the
    # sanitizer runtimes are missing from the toolchain; any other build error of the instrumented
    # host sources fails the test.
    if not _sanitizer_runtime_available(str(tmp_path_factory.mktemp("asan_probe"))):
        pytest.skip("hipcc cannot link ASan/UBSan host programs on this machine")
    r = subprocess.run(["make", "-C", CSRC, "-j8", "sanitize"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and os.path.exists(DRIVER), "sanitizer build failed:\n" + (r.stdout + r.stderr)[-4000:]
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
