#!/usr/bin/env python3
"""Timeline of one streaming hop from a rocprofv3 kernel trace (tools/gpu_c5trace.sh): the kernels
between two consecutive launches of the hop's first kernel (frame_pad_kernel), their durations, the
idle time between them and the hop's span.  stream_bench.py runs warmup + hops eager hops, then as
many graph replays, then the halo streams: --hop 50 (default) is a graph replay with the defaults of
gpu_c5trace.sh (5 + 30).

    python tools/hop_timeline.py gpurun_out/c5t_kernel_trace.csv [--hop 50] [--top 40] [--list]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--hop", type=int, default=50)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--list", action="store_true", help="print every kernel of the hop in order")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                         int(r["Workgroup_Size_X"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "frame_pad" in r[2]]
    i0, i1 = starts[a.hop - 1], starts[a.hop]
    hop = rows[i0:i1]
    # the hop ends at its last kernel before the gap to the next hop's first kernel
    span = (hop[-1][1] - hop[0][0]) / 1e3
    busy = sum(e - s for s, e, *_ in hop) / 1e3
    gaps = [(b[0] - a_[1]) / 1e3 for a_, b in zip(hop, hop[1:])]
    print(f"hop {a.hop}: {len(hop)} kernels, span {span:.1f} us, kernel time {busy:.1f} us, "
          f"idle between kernels {span - busy:.1f} us (median gap {sorted(gaps)[len(gaps) // 2]:.2f} us)")
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, n, *_ in hop:
        k = n.split("(")[0][:60]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{k:62s} {c:4d} launches {t:8.1f} us  ({t / c:6.2f} us each)")
    if a.list:
        t0 = hop[0][0]
        for s, e, n, g, wg in hop:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f} us  grid {g // wg:5d}  {n.split('(')[0][:70]}")


if __name__ == "__main__":
    main()
