#!/usr/bin/env python3
"""Throughput benchmark of the MI355X DistilCodec encode -> VQ -> decode path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seconds S]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload (BASELINE.json configs[1], "C2"): per GPU, a batch of 32 synthetic 10 s 24 kHz clips
(speech-like / music-like mix), fp32, the full path mel -> ConvNeXt encoder -> GRFVQ search ->
decode(codes) -> HiFiGAN generator, i.e. `DistilCodec.encode` followed by `decode_from_codes`.
A step = one pass of the path over the rank's batch, inputs already resident in HBM.  Clips are
independent, so ranks shard clips with no collective on the data path (weak scaling); the only
collectives are the timing barrier and the max-over-ranks reduction.

Rank 0 prints one JSON line.  `roofline` reports the dominant kernel (largest summed device
time, HIP events around each launch on its stream during the timed steps) as algorithmic
FLOP/s against the fp32 MFMA peak; `cpu_baseline` times the CPU oracle (the reference's
algorithm on PyTorch-CPU, oracle/reference_cpu.py) on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from distilcodec_nabeel_amd import config as dconfig  # noqa: E402
from distilcodec_nabeel_amd import synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (= fp32 vector peak)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
# x6 mode executes 6 exact bf16 products per fp32 product: its ceiling in fp32-algorithmic FLOP/s
X6_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6
HBM_PEAK_GBS = 8000.0
SR = 24000


def traffic_for(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass (profiles/pmc_latest.json:
    2*FETCH_SIZE + WRITE_SIZE, gfx950 correction), or None when that kernel was not profiled."""
    path = os.path.join(HERE, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(cfg, state, seconds: float, batch: int):
    """Oracle (PyTorch-CPU restatement of the reference) on a bounded sample of the workload."""
    from oracle import reference_cpu as R

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    warm, _ = R.pad_batch(synth.clips(1, SR // 2, seed=999))
    R.encode_decode(warm, state, cfg)
    audio, _ = R.pad_batch(synth.clips(batch, int(seconds * SR), seed=0, kind="mix"))
    t0 = time.perf_counter()
    R.encode_decode(audio, state, cfg)
    dt = time.perf_counter() - t0
    return {"value": round(batch * seconds * SR / dt, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{batch} x {seconds:g} s clips, full encode->VQ->decode, fp32, oracle/reference_cpu.py, "
                      f"{dt:.1f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--seconds", type=float, default=10.0, help="clip length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-batch", type=int, default=2)
    ap.add_argument("--no-profile", action="store_true", help="skip the per-launch HIP-event roofline timing")
    ap.add_argument("--gemm", choices=["x6", "f32"], default="x6",
                    help="x6: fp32 operands as 3 bf16 planes, 6 exact products, f32 accumulate; f32: fp32 MFMA")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    cfg = dconfig.default_config()
    state = weights.synthetic_state_dict(cfg, seed=1234)
    eng = NativeCodec(cfg, state, dev, gemm=args.gemm)

    n = int(args.seconds * SR)
    clips = synth.clips(args.batch, n, seed=1000 * rank, kind="mix")
    audio = torch.zeros(args.batch, n + 1)  # reference layout: 1 leading zero (distil_codec.py:133-136)
    for i, c in enumerate(clips):
        audio[i, 1:] = torch.from_numpy(c)
    audio = audio.to(dev)
    T = eng.num_frames(n + 1)
    codes = torch.empty(args.batch, T, dtype=torch.int32, device=dev)
    wav = torch.empty(args.batch, 256 * T, device=dev)

    for _ in range(args.warmup):
        eng.encode_decode(audio, codes, wav)
    torch.cuda.synchronize(dev)
    assert int(codes.min()) >= 0 and int(codes.max()) < cfg["quantizer"]["codebook_size"]
    assert bool(torch.isfinite(wav).all())

    if not args.no_profile:
        eng.profile(True)
        eng.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.encode_decode(audio, codes, wav)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = {}
    if not args.no_profile:
        prof = eng.profile_read()
        eng.profile(False)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_step = dt / args.steps * 1e3
    samples = args.batch * n * world
    value = samples / (dt / args.steps)

    roof = None
    if prof:
        name, rec = max(prof.items(), key=lambda kv: kv[1]["ms"])
        avg_ms = rec["ms"] / rec["launches"]
        achieved = rec["flops"] / (rec["ms"] * 1e-3) / 1e12
        peak = X6_PEAK_TFLOPS if "x6" in name else FP32_MFMA_PEAK_TFLOPS
        roof = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic_for(name),
                "peak_basis": ("bf16 dense MFMA 2500 TF / 6 bf16 products per fp32 product" if "x6" in name
                               else "fp32 MFMA v_mfma_f32_32x32x2_f32"),
                "launches_per_step": rec["launches"] // args.steps, "avg_launch_ms": round(avg_ms, 4),
                "share_of_device_time": round(rec["ms"] / sum(r["ms"] for r in prof.values()), 4)}
        if rank == 0 and os.environ.get("DCX_BENCH_KERNELS"):
            with open(os.environ["DCX_BENCH_KERNELS"], "w") as f:
                json.dump({"steps": args.steps, "kernels": prof}, f, indent=1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, state, args.cpu_seconds, args.cpu_batch)

    if rank == 0:
        out = {
            "metric": "24 kHz samples/s encode+decode at 1/8 GPU; code-index bit-exact vs CPU",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "arith": ("fp32 operands split into 3 bf16 planes, 6 exact bf16 products per fp32 product, fp32 "
                      "accumulation (v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16)" if args.gemm == "x6" else
                      "fp32 MFMA (v_mfma_f32_32x32x2_f32)"),
            "data": "synthetic (speech/music-like 24 kHz clips; seeded synthetic weights, no checkpoint offline)",
            "config": {"workload": f"C2: {args.batch} x {args.seconds:g} s clips per GPU, full mel->encoder->VQ->"
                                   f"decode->generator, fp32", "global_batch": args.batch * world,
                       "clip_samples": n, "frames_per_clip": T, "parallelism": f"clip-sharded x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
