#!/usr/bin/env python3
"""Per-wave SQ counters of one kernel from tools/pmc_kernel.sh's two passes (p1, p2):
each counter summed over a dispatch, divided by that dispatch's SQ_WAVES (pass 1), the
median over dispatches.  Prints one JSON object.

  python tools/sq_kernel_summary.py gpurun_out/pmc_<name> "interval_kernel<4, 0>"
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, kernel):
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            c = out[int(r["Dispatch_Id"])]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    base, kernel = sys.argv[1], sys.argv[2]
    p1, p2 = per_dispatch(os.path.join(base, "p1"), kernel), per_dispatch(os.path.join(base, "p2"), kernel)
    waves = statistics.median(c["SQ_WAVES"] for c in p1.values())
    res = {"kernel": kernel, "dispatches": [len(p1), len(p2)], "waves_per_dispatch": waves, "per_wave": {}}
    for p in (p1, p2):
        names = sorted({k for c in p.values() for k in c})
        for k in names:
            if k == "SQ_WAVES":
                continue
            res["per_wave"][k] = statistics.median(c[k] for c in p.values() if k in c) / waves
    pw = res["per_wave"]
    if pw.get("SQ_WAVE_CYCLES"):
        res["wait_any_over_wave_cycles"] = pw.get("SQ_WAIT_ANY", 0) / pw["SQ_WAVE_CYCLES"]
        res["active_inst_over_wave_cycles"] = pw.get("SQ_ACTIVE_INST_ANY", 0) / pw["SQ_WAVE_CYCLES"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
