#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes).

    python tools/rocprof_summary.py --stats DIR/run_kernel_stats.csv [--fetch DIR/run_counter_collection.csv]
        [--write DIR/run_counter_collection.csv] [--bench-kernels kernels.json] > profiles/rNN_summary.md

HBM bytes per launch follow MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE (KiB) counts half of
a wide coalesced streaming read, so it is doubled; WRITE_SIZE (KiB) is taken as is.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    name = name.strip('"')
    m = re.match(r"(?:void )?(?:dcx::)?([A-Za-z_0-9]+)(<[^()]*>)?", name)
    if not m:
        return name[:60]
    base, targs = m.group(1), m.group(2) or ""
    parts = [p.strip() for p in targs.strip("<>").split(",")] if targs else []
    if base == "conv_gemm_f32":
        kind = "vq_dist_argmin_f32" if parts[-1] == "true" else "conv_gemm_f32"
        return f"{kind}<{parts[0]},{parts[1]}>"
    if base == "conv_gemm_x6pp" and len(parts) > 2 and parts[2] == "true":
        return "conv_gemm_x6pf<512,64,halo>"
    if base in ("conv_gemm_x6pp", "conv_gemm_x6lm"):
        return f"{base}<256,128,halo>" if parts and parts[0] != "0" else f"{base}<256,128>"
    if base == "conv_gemm_x6dm":  # <HALO, BN>: BM = 65536 / BN
        bm, bn = 65536 // int(parts[1]), int(parts[1])
        return f"{base}<{bm},{bn},halo>" if parts[0] != "0" else f"{base}<{bm},{bn}>"
    if base == "conv_gemm_bf16dm":  # <REG>
        return "conv_gemm_bf16dm<256,256,reg>" if parts and parts[0] == "true" else "conv_gemm_bf16dm<256,256>"
    if base == "conv_gemm_x6dq_group":  # <BN>, halo
        return f"{base}<{65536 // int(parts[0])},{parts[0]},halo>"
    if base == "conv_gemm_x6dq":  # <BN>, halo
        return f"{base}<{65536 // int(parts[0])},{parts[0]},halo>"
    if base == "conv_gemm_x3dw_group":  # <SPLIT[, BN]>
        return "conv_gemm_x3dw_group<384,128,halo>" if len(parts) > 1 and parts[1] == "128" else "conv_gemm_x3dw_group<256,256,halo>"
    if base == "conv_gemm_x3dw":  # <HALO, SPLIT[, BN]>
        tile = "384,128" if len(parts) > 2 and parts[2] == "128" else "256,256"
        return f"conv_gemm_x3dw<{tile},halo>" if parts and parts[0] != "0" else f"conv_gemm_x3dw<{tile}>"
    if base == "conv_gemm_x3dq_group":  # <BN>, halo
        return f"{base}<{32768 // int(parts[0])},{parts[0]},halo>"
    if base == "conv_gemm_x3dq":  # <BN, HALO>; HALO = 0: the one-tap conv_gemm_x3dm
        bm, bn = 32768 // int(parts[0]), int(parts[0])
        return f"conv_gemm_x3dq<{bm},{bn},halo>" if parts[1] != "0" else f"conv_gemm_x3dm<{bm},{bn}>"
    if base == "vq_prefilter_b1":
        return "vq_prefilter_b1<256,256>"
    if base in ("conv_res_pair", "conv_res_pair_g", "conv_res_pair_w4", "conv_res_pair_h3"):  # <C, MEAN, ROWS>
        return f"{base}<{parts[0]}{',mean' if len(parts) > 1 and parts[1] == 'true' else ''}>"
    if base == "vq_prefilter_dm":  # <XMID>
        return "vq_prefilter_dm<256,256>" if parts and parts[0] == "true" else "vq_prefilter_dm_x2<256,256>"
    if base == "vq_prefilter_x3":
        kind = "vq_prefilter_x3" if len(parts) < 5 or parts[4] == "true" else "vq_prefilter_x2"
        return f"{kind}<{parts[0]},{parts[1]}>"
    if base == "conv_gemm_x6w8":  # <BM, BN, WM, WN, HALO, ARGMIN, PROD, AF32>: bench.py's names
        waves = int(parts[2]) * int(parts[3])
        halo = ",halo" if parts[4] != "0" else ""
        kind = "bf16" if len(parts) > 6 and parts[6] == "1" else "x6"
        f = "f" if len(parts) > 7 and parts[7] == "true" else ""
        return f"conv_gemm_{kind}w{waves}{f}<{parts[0]},{parts[1]}{halo}>"
    return base + targs.replace(" ", "")


def pmc(path):
    acc = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            acc[k][0] += 1
            acc[k][1] += float(r["Counter_Value"])
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench-kernels")
    a = ap.parse_args()
    rows = []
    with open(a.stats) as f:
        for r in csv.DictReader(f):
            rows.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                         float(r["Percentage"])))
    fetch = pmc(a.fetch) if a.fetch else {}
    write = pmc(a.write) if a.write else {}
    bench = json.load(open(a.bench_kernels)) if a.bench_kernels else None
    print("| kernel | calls | total ms | avg ms | % | HBM MB/launch (2*FETCH+WRITE) | algorithmic MB/launch |")
    print("|---|---|---|---|---|---|---|")
    for name, calls, tot, avg, pct in rows:
        hbm = ""
        if name in fetch and name in write:
            n = fetch[name][0]
            hbm = f"{(2 * fetch[name][1] + write[name][1]) * 1024 / n / 1e6:.1f}"
        alg = ""
        if bench and name in bench["kernels"]:
            k = bench["kernels"][name]
            alg = f"{k['bytes'] / k['launches'] / 1e6:.1f}"
        print(f"| {name} | {calls} | {tot / 1e6:.2f} | {avg / 1e6:.4f} | {pct:.2f} | {hbm} | {alg} |")


if __name__ == "__main__":
    main()
