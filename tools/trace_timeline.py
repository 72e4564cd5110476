#!/usr/bin/env python3
"""Timeline of the last frames of a rocprofv3 kernel trace (tools/frame_loop.py under --kernel-trace): each
kernel's start and end in us relative to its frame's rtc_tile_cull start.  Not part of the product.
Usage: trace_timeline.py <run_kernel_trace.csv> [frames]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 4
short = lambda n: n.split("(")[0].replace("void ", "")
starts = [i for i, r in enumerate(rows) if "rtc_tile_cull" in r["Kernel_Name"]]
for a, b in zip(starts[-nf - 1:-1], starts[-nf:]):
    t0 = int(rows[a]["Start_Timestamp"])
    print(f"frame period {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    for r in rows[a:b]:
        print(f"  {short(r['Kernel_Name']):32s} {(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - t0) / 1e3:8.1f}")
