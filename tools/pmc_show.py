#!/usr/bin/env python3
"""Per-kernel SQ counter totals (last dispatch of each kernel) from tools/pmc_kernel.sh output.
usage: python tools/pmc_show.py gpurun_out/pmc_NAME [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
last = {}
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"][:60], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, disp), cs in per.items():
        if k not in last or disp >= last[k][0]:
            last.setdefault(k, [disp, {}])
            last[k][0] = disp
            last[k][1].update(cs)
for k, (disp, cs) in last.items():
    w = cs.get("SQ_WAVES", 1) or 1
    print(k)
    print("  per wave:", {c: round(v / w, 1) for c, v in sorted(cs.items())})
