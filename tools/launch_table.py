"""Per-launch table of a rocprofv3 --kernel-trace CSV (tools/gpu_trace.sh): the last step's launches in
order (found by the last occurrence of a marker kernel), with grid, duration and the gap to the
previous launch.  Usage: python tools/launch_table.py trace.csv [marker_kernel_substring] [filter]"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"dcx::(\(anonymous namespace\)::)?", "", n)
    n = re.sub(r"\(.*\)$", "", n)
    return n[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marker = sys.argv[2] if len(sys.argv) > 2 else "frame_pad"
    filt = sys.argv[3] if len(sys.argv) > 3 else ""
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    start = idx[-1] if idx else 0
    last = rows[start:]
    t0 = int(last[0]["Start_Timestamp"])
    prev_end = None
    tot = 0.0
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        us = (e - s) / 1e3
        tot += us
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        name = short(r["Kernel_Name"])
        if filt and filt not in name:
            continue
        wg = int(r["Workgroup_Size_X"])
        grid = int(r["Grid_Size_X"]) // max(wg, 1)
        print(f"{(s - t0) / 1e3:10.1f}  {us:9.1f} us  gap {gap:6.1f}  wg {grid:6d}x{wg:<4d} vgpr {r['VGPR_Count']:>3s} lds {r['LDS_Block_Size']:>6s}  {name}")
    print(f"sum of launch durations {tot / 1e3:.2f} ms, span {(prev_end - t0) / 1e6:.2f} ms, launches {len(last)}")


if __name__ == "__main__":
    main()
