#!/usr/bin/env python3
"""Markdown table of the per-kernel ratios in a tools/pmc_summary.py output: MFMA busy per SIMD-cycle,
non-MFMA VALU, SALU and LDS instructions per MFMA, wait fraction, LDS bank conflicts per LDS instruction."""
import re
import sys

rows, cur, vals = [], None, {}
for line in open(sys.argv[1]):
    if line and not line.startswith(" "):
        if cur:
            rows.append((cur, vals))
        cur, vals = line.strip(), {}
        continue
    m = re.match(r"\s+(\S+)\s+([0-9.]+)\s+\(n=", line)
    if m:
        vals[m.group(1)] = float(m.group(2))
    m = re.match(r"\s+MFMA busy per SIMD-cycle ~ ([0-9.]+)", line)
    if m:
        vals["busy"] = float(m.group(1))
if cur:
    rows.append((cur, vals))
print("| kernel | MFMA busy | VALU/MFMA | SALU/MFMA | LDS/MFMA | wait/wave-cycles | bank conflicts/LDS inst |")
print("|---|---|---|---|---|---|---|")
for name, v in rows:
    mf = v.get("SQ_INSTS_MFMA", 0)
    if mf < 1e6:
        continue
    f = lambda k: v.get(k, 0) / mf  # noqa: E731
    valu = (v.get("SQ_INSTS_VALU", 0) - mf) / mf
    wait = v.get("SQ_WAIT_ANY", 0) / v["SQ_WAVE_CYCLES"] if v.get("SQ_WAVE_CYCLES") else float("nan")
    bc = v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_INSTS_LDS"] if v.get("SQ_INSTS_LDS") else float("nan")
    print(f"| {name[:48]} | {v.get('busy', float('nan')):.3f} | {valu:.2f} | {f('SQ_INSTS_SALU'):.2f} | "
          f"{f('SQ_INSTS_LDS'):.2f} | {wait:.3f} | {bc:.3f} |")
