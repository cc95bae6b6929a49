#!/usr/bin/env python3
"""C5 latency path: streaming 1 s hops, encode->decode per hop as one captured HIP graph.

    python tools/stream_bench.py [--hops 200] [--warmup 20] [--hop-samples 24000]

Prints one JSON line: eager and graph-replay latency per hop (p50 / p99 / mean, ms, measured
with HIP events around each step on the stream it runs on, input already resident in HBM), the
real-time factor and a bit-exactness check of graph replay vs eager on the same chunks.
Synthetic speech-like audio, seeded synthetic weights.
"""
import argparse
import json
import time
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distilcodec_nabeel_amd import config, synth, weights  # noqa: E402
from distilcodec_nabeel_amd.engine import NativeCodec  # noqa: E402
from distilcodec_nabeel_amd.streaming import GraphedHop, HaloStream  # noqa: E402


def stats(ms):
    a = np.asarray(ms)
    return {"p50": round(float(np.percentile(a, 50)), 4), "p99": round(float(np.percentile(a, 99)), 4),
            "mean": round(float(a.mean()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hops", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--hop-samples", type=int, default=24000)
    ap.add_argument("--gemm", default="x6", choices=["x6", "f32"])
    ap.add_argument("--kernels", default=None, help="also write a per-kernel profile of 10 eager hops (json)")
    ap.add_argument("--split-k", type=int, default=0, help="split-K latency mode: max K-slices per few-tile conv")
    a = ap.parse_args()
    cfg = config.default_config()
    eng = NativeCodec(cfg, weights.synthetic_state_dict(cfg, seed=1234), "cuda:0", gemm=a.gemm)
    if a.split_k:
        eng.set_split_k(a.split_k)
    n = a.hop_samples
    stream = np.concatenate(synth.clips(1, n * (a.hops + a.warmup), seed=3, kind="speech"))
    chunks = torch.from_numpy(stream.reshape(-1, 1, n).astype(np.float32)).cuda()
    hop = GraphedHop(eng, n)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.hops)]

    def run(step):  # step(i) processes hop i
        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        for i in range(a.hops):
            ev[i][0].record()
            step(a.warmup + i)
            ev[i][1].record()
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) for e0, e1 in ev]

    codes_e = torch.empty(1, hop.frames, dtype=torch.int32, device="cuda")
    wav_e = torch.empty(1, eng.hop * hop.frames, device="cuda")
    padded = torch.nn.functional.pad(chunks, (1, 0))  # the reference's 1-sample left pad per clip
    eager = run(lambda i: eng.encode_decode(padded[i], codes_e, wav_e))
    graph = run(lambda i: hop(chunks[i]))
    # bit-exactness of replay vs eager on a few chunks
    exact = True
    for i in (0, a.hops // 2, a.hops - 1):
        c = chunks[a.warmup + i]
        eng.encode_decode(padded[a.warmup + i], codes_e, wav_e)
        gc, gw = hop(c)
        torch.cuda.synchronize()
        exact &= bool(torch.equal(gc, codes_e)) and bool(torch.equal(gw, wav_e))
    if a.kernels:
        eng.profile(True)
        eng.profile_reset()
        for i in range(10):
            eng.encode_decode(padded[i], codes_e, wav_e)
        json.dump({"steps": 10, "kernels": eng.profile_read()}, open(a.kernels, "w"), indent=1)
        eng.profile(False)
    hop_ms = 1000.0 * n / 24000
    g = stats(graph)
    print(json.dumps({
        "config": "C5: streaming encode->decode, hop %d samples (B=1), one hipGraph-captured step" % n,
        "frames_per_hop": hop.frames, "output_samples_per_hop": eng.hop * hop.frames, "hops": a.hops,
        "gemm": a.gemm, "split_k": a.split_k, "eager_ms": stats(eager), "graph_ms": g,
        "real_time_factor_p99": round(g["p99"] / hop_ms, 5), "graph_equals_eager": exact,
        "data": "synthetic speech-like audio, seeded synthetic weights",
    }), flush=True)
    # halo-overlapped stream (streaming.HaloStream): output equal to the full clip, per-push wall time
    hs = HaloStream(eng)
    wall = []
    for i in range(a.warmup + a.hops):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs.push(chunks[i, 0])
        torch.cuda.synchronize()
        if i >= a.warmup:
            wall.append(1000.0 * (time.perf_counter() - t0))
    h = stats(wall)
    print(json.dumps({
        "config": "C5 halo stream: push %d samples (B=1), output equal to the full-clip run" % n,
        "enc_halo_frames": hs.enc_halo, "gen_halo_frames": hs.gen_halo,
        "lookahead_ms": round(1000.0 * (hs.enc_halo + hs.gen_halo + 3) * eng.hop / 24000, 1),
        "pushes": a.hops, "push_wall_ms": h, "real_time_factor_p99": round(h["p99"] / hop_ms, 5),
        "note": "eager stage calls on windows of hop + 2 x halo frames (not graph-captured)",
    }), flush=True)
    # the same stream on fixed windows, both steps replayed from HIP graphs
    hg = HaloStream(eng, push_samples=n, graph=True)
    wall = []
    for i in range(a.warmup + a.hops):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hg.push(chunks[i, 0])
        torch.cuda.synchronize()
        if i >= a.warmup:
            wall.append(1000.0 * (time.perf_counter() - t0))
    h = stats(wall)
    print(json.dumps({
        "config": "C5 halo stream, hipGraph-captured: push %d samples (B=1), output equal to the full-clip run" % n,
        "enc_window_samples": hg.n_enc, "gen_window_frames": hg.t_gen,
        "lookahead_ms": round(1000.0 * (hg.enc_halo + hg.gen_halo + 3) * eng.hop / 24000, 1),
        "pushes": a.hops, "push_wall_ms": h, "real_time_factor_p99": round(h["p99"] / hop_ms, 5),
        "note": "two graph replays per push (encoder window, generator window) plus the host-side slicing",
    }))


if __name__ == "__main__":
    main()
