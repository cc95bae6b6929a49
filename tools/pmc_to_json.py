#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from FETCH_SIZE / WRITE_SIZE rocprofv3 passes -> JSON
(gfx950: 2*FETCH_SIZE + WRITE_SIZE, both in KiB; MI355X_MICROARCH.md §HBM).

    python tools/pmc_to_json.py FETCH_DIR WRITE_DIR > profiles/pmc_latest.json
"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import pmc  # noqa: E402


def find(d):
    return glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]


f, w = pmc(find(sys.argv[1])), pmc(find(sys.argv[2]))
out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes over bench.py (separate runs)",
       "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch (gfx950 FETCH_SIZE correction)",
       "kernels": {}}
for k in f:
    if k in w:
        out["kernels"][k] = {"launches": f[k][0],
                             "hbm_bytes_per_launch": round((2 * f[k][1] / f[k][0] + w[k][1] / w[k][0]) * 1024)}
print(json.dumps(out, indent=1))
