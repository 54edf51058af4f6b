#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive kernels of one
rocprofv3 --kernel-trace run (kernel_trace.csv), for the step-overhead budget.

usage: python tools/trace_gaps.py TRACE_DIR [NAME_SUBSTR ...]

Prints, per kernel name (substring filter optional): launches, mean / median
duration (us), and the median gap (us) from the end of the previous kernel on
the same queue to its start.
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    keep = sys.argv[2:]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r.get("Queue_Id", 0) or 0), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"]))
    rows.sort(key=lambda x: (x[0], x[1]))
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev = {}
    for q, s, e, n in rows:
        short = n.split("(")[0][:90]
        dur[short].append((e - s) / 1e3)
        if q in prev:
            gap[short].append((s - prev[q]) / 1e3)
        prev[q] = e
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if keep and not any(k in n for k in keep):
            continue
        g = gap.get(n, [])
        print(f"{n:90s} n={len(v):5d} mean={statistics.mean(v):9.2f} med={statistics.median(v):9.2f} "
              f"gap_med={statistics.median(g) if g else float('nan'):7.2f} us")


if __name__ == "__main__":
    main()
