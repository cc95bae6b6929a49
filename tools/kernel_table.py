#!/usr/bin/env python3
"""Per-kernel table from bench.py's DCX_BENCH_KERNELS json."""
import json
import sys

d = json.load(open(sys.argv[1]))
steps = d["steps"]
tot = sum(v["ms"] for v in d["kernels"].values())
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["ms"]):
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
    gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0
    print(f"{k:34s} launches/step {v['launches'] // steps:4d}  ms/step {v['ms'] / steps:8.2f} ({100 * v['ms'] / tot:5.1f}%)  "
          f"TF/s {tf:7.2f}  GB/s {gbs:8.1f}")
print("total device ms/step", round(tot / steps, 2))
