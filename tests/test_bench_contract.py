"""bench.py's output contract without a GPU: the roofline record computed from per-kernel HIP-event
timings (the dominant kernel, its achieved FLOP/s against the x6 or fp32 MFMA ceiling, the PMC
traffic committed in profiles/pmc_latest.json), the workload table (BASELINE.json configs[1] and
configs[3]) and the CPU-baseline record (the oracle timed with all host threads and one)."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_roofline_picks_the_dominant_kernel():
    dom = "conv_gemm_x3dw_group<256,256,halo>"
    prof = {
        dom: {"launches": 20, "ms": 200.0, "flops": 20 * 2.6e12, "bytes": 0.0},
        "conv_gemm_f32<128,128>": {"launches": 4, "ms": 10.0, "flops": 1e12, "bytes": 0.0},
    }
    r = bench.roofline(prof, steps=2)
    assert r["kernel"] == dom
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - 20 * 2.6e12 / 0.2 / 1e12) < 0.01
    assert r["peak"] == round(bench.BF16_MFMA_PEAK_TFLOPS / 3, 1)  # h3: 3 fp16 products per fp32 product
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["launches_per_step"] == 10 and abs(r["avg_launch_ms"] - 10.0) < 1e-9
    assert abs(r["share_of_device_time"] - 200 / 210) < 1e-3
    # traffic: HBM bytes per launch of that kernel from the committed PMC pass, or None
    pmc = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))
    assert r["traffic"] == pmc["kernels"][dom]["hbm_bytes_per_launch"]
    assert bench.traffic_for("no_such_kernel") is None
    x6 = bench.roofline({"conv_gemm_x6dq<256,256,halo>": {"launches": 1, "ms": 1.0, "flops": 1e11, "bytes": 0}}, 1)
    assert x6["peak"] == round(bench.BF16_MFMA_PEAK_TFLOPS / 6, 1)
    f = bench.roofline({"conv_gemm_f32<128,128>": {"launches": 1, "ms": 1.0, "flops": 1e11, "bytes": 0}}, 1)
    assert f["peak"] == bench.FP32_MFMA_PEAK_TFLOPS
    assert bench.roofline({}, 1) is None


def test_workloads_are_the_baseline_configs():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert "batch=32 × 10 s" in base["configs"][1].replace("x", "×")
    assert bench.WORKLOADS["c2"] == (32, 240000, 240000)
    per_gpu, longest, shortest = bench.WORKLOADS["c4"]
    assert per_gpu * 8 == 1024 and longest == 240000 and shortest < longest


def test_cpu_baseline_record(cfg, state):
    rec = bench.cpu_baseline(cfg, state)
    assert rec["kind"] == "port" and rec["unit"] == "samples/s"
    assert rec["value"] > 0 and rec["value_1thread"] > 0
    assert rec["cores"] >= 1 and rec["cpu_model"]
    assert "median of 3" in rec["sample"]
